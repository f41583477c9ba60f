#!/bin/bash
# Generic GPU-box step runner: gpu_run.sh <tag> <test-selector> [extra python script args...]
#   runs `pytest -m gpu <selector>` (if not "-"; env K = a pytest -k expression), then each
#   remaining argument as a python
#   command line (quoted), each under its own time limit, writing under gpurun_out/<tag>/.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; SEL=$2; shift 2
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
cd "$R"
if [ "$SEL" != "-" ]; then
  timeout -k 10 900 python -u -m pytest $SEL ${K:+-k "$K"} -m gpu -v -x --timeout 400 --timeout-method thread \
      > "$O/tests.log" 2>&1 || { echo "tests rc=$?" >> "$O/tests.log"; exit 3; }
fi
i=0
for cmd in "$@"; do
  i=$((i+1))
  timeout -k 10 400 $cmd > "$O/cmd$i.out" 2> "$O/cmd$i.err"
done
echo done > "$O/ok"
