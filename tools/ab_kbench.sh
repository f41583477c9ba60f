#!/bin/bash
# kbench timings of library variants (variants/libeelg_<tag>.so via EELG_LIB; "main" = in-tree).
# usage (GPU box): bash tools/ab_kbench.sh "<kbench --only regex>" main <tag> [<tag> ...]
set -e -o pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/ab; mkdir -p "$O"
ONLY=$1; shift
for v in "$@"; do
  if [ "$v" = main ]; then L=""; else L=$R/variants/libeelg_$v.so; fi
  EELG_LIB=$L timeout -k 10 200 python3 "$R/tools/kbench.py" --reps 20 --only "$ONLY" > "$O/k_$v.txt" 2>&1
  echo "== $v"; grep " ms" "$O/k_$v.txt" | cut -c1-90
done
