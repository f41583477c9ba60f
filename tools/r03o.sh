#!/bin/bash
# fast-linear weight staging with a per-K batch (main) vs HEAD (prev): parity + kbench; then an
# in-line (EELG_OVERLAP=0) kernel trace of the bench step for the per-kernel cost table
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"; mkdir -p gpurun_out/r03o
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "linear or model_forward" \
    > gpurun_out/r03o/t.log 2>&1 || { tail -30 gpurun_out/r03o/t.log; exit 3; }
tail -1 gpurun_out/r03o/t.log
bash tools/ab_kbench.sh "sc_bwd_coef|lin " main prev
cd /tmp && export TMPDIR=/tmp
EELG_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/r03o/inline" -o run \
    -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$R/gpurun_out/r03o/inline.log" 2>&1
tail -1 "$R/gpurun_out/r03o/inline.log"
