#!/bin/bash
# r02a: full GPU suite (with the new full-size oracle / DDP / checkpoint tests), the default
# bench line, and the self-launched 2-rank bench (gloo on the one device of a 1-GPU box).
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/${1:-r02a}
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
cd "$R"
EELG_PARITY_OUT=$O/parity.json timeout -k 10 900 python -u -m pytest tests -m gpu -v -s \
   --timeout 400 --timeout-method thread > "$O/tests.log" 2>&1 || echo "tests rc=$?" >> "$O/tests.log"
grep -q "Fatal\|core dumped\|HSA_STATUS" "$O/tests.log" && exit 3
timeout -k 10 300 python bench.py > "$O/bench.json" 2> "$O/bench.err"
timeout -k 10 300 python bench.py --gpus 2 --steps 5 --warmup 3 --no-cpu-baseline > "$O/bench_g2.json" 2> "$O/bench_g2.err"
echo done > "$O/ok"
