#!/bin/bash
# kbench timings of one library under several settings of an environment knob.
# usage (GPU box): bash tools/ab_env.sh "<kbench --only regex>" VAR v1 v2 ...
set -e -o pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/abenv; mkdir -p "$O"
ONLY=$1; VAR=$2; shift 2
for v in "$@"; do
  env "$VAR=$v" timeout -k 10 200 python3 "$R/tools/kbench.py" --reps 20 --only "$ONLY" > "$O/k_${VAR}_$v.txt" 2>&1
  echo "== $VAR=$v"; grep " ms" "$O/k_${VAR}_$v.txt" | cut -c1-100
done
