#!/bin/bash
# Full GPU suite + default bench line + smoke, each under its own time limit (first failure
# ends the script).  usage (GPU box): bash tools/gpu_full.sh <tag>
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/${1:-full}
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
cd "$R"
EELG_PARITY_OUT=$O/parity.json timeout -k 10 900 python -u -m pytest tests -m gpu -v -x \
   --timeout 400 --timeout-method thread > "$O/tests.log" 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
timeout -k 10 300 python bench.py > "$O/bench.json" 2> "$O/bench.err"
echo done > "$O/ok"
