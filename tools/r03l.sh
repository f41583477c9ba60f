#!/bin/bash
# tp_fwd nontemporal aggregate stores / weight loads (variants ntst, ntw, ntb) and the XCD-grouped
# contraction tiles (main) vs the previous library (prev): parity, kbench, bench A/B
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"; mkdir -p gpurun_out/r03l
EELG_LIB=$R/variants/libeelg_ntb.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
    -k "interaction or model_forward" > gpurun_out/r03l/t_ntb.log 2>&1 || { tail -30 gpurun_out/r03l/t_ntb.log; exit 3; }
tail -1 gpurun_out/r03l/t_ntb.log
bash tools/ab_kbench.sh "tp_fwd" main ntst ntw ntb
bash tools/gpu_bench_ab.sh r03l_ab "EELG_LIB=$R/variants/libeelg_prev.so" "EELG_LIB=$R/variants/libeelg_ntst.so" "EELG_LIB=$R/variants/libeelg_ntb.so"
