#!/bin/bash
# single-round-trip staging in the coefficient gradient and the fast linear's weight tile /
# residual epilogue (main) vs HEAD (prev): parity, kbench, bench A/B
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"; mkdir -p gpurun_out/r03n
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r03n/t.log 2>&1 || { tail -30 gpurun_out/r03n/t.log; exit 3; }
tail -1 gpurun_out/r03n/t.log
bash tools/ab_kbench.sh "sc_bwd_coef|lin " main prev
bash tools/gpu_bench_ab.sh r03n_ab "EELG_LIB=$R/variants/libeelg_prev.so" "EELG_LIB=$R/variants/libeelg_ntw.so" "EELG_LIB=$R/variants/libeelg_ntb.so"
