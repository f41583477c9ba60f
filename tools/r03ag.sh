#!/bin/bash
# tp_fwd with the next edge's rows prefetched into LDS by LDS-DMA (glds) vs the register
# pipeline (main): parity, kbench, bench A/B
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"; mkdir -p gpurun_out/r03ag
EELG_LIB=$R/variants/libeelg_glds.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread \
    -k "interaction or model_forward_backward_matches_oracle" > gpurun_out/r03ag/t_glds.log 2>&1 || { tail -40 gpurun_out/r03ag/t_glds.log; exit 3; }
echo "glds: $(tail -1 gpurun_out/r03ag/t_glds.log)"
bash tools/ab_kbench.sh "tp_fwd" main glds
bash tools/gpu_bench_ab.sh r03ag_ab "EELG_LIB=$R/variants/libeelg_glds.so"
