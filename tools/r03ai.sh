#!/bin/bash
# LDS-DMA tp_fwd with two edges in flight (glds2) vs one (glds) vs the register pipeline (main)
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"; mkdir -p gpurun_out/r03ai
EELG_LIB=$R/variants/libeelg_glds2.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread \
    -k "interaction or model_forward_backward_matches_oracle" > gpurun_out/r03ai/t_glds2.log 2>&1 || { tail -40 gpurun_out/r03ai/t_glds2.log; exit 3; }
echo "glds2: $(tail -1 gpurun_out/r03ai/t_glds2.log)"
bash tools/ab_kbench.sh "tp_fwd" main glds glds2
bash tools/gpu_bench_ab.sh r03ai_ab "EELG_LIB=$R/variants/libeelg_glds.so" "EELG_LIB=$R/variants/libeelg_glds2.so"
