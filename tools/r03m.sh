#!/bin/bash
# contraction staging rewrite (float4 loads all in flight, branch-free offsets; main) and a
# grad-x coefficient prefetch depth of 2 (pfd2) vs the previous library (prev); tp_fwd
# group-major order (gmaj, built before the staging rewrite): kbench, bench A/B
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"; mkdir -p gpurun_out/r03m
EELG_LIB=$R/variants/libeelg_gmaj.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
    -k "interaction or model_forward" > gpurun_out/r03m/t_gmaj.log 2>&1 || { tail -30 gpurun_out/r03m/t_gmaj.log; exit 3; }
echo "gmaj: $(tail -1 gpurun_out/r03m/t_gmaj.log)"
bash tools/ab_kbench.sh "sc_|tp_fwd" main pfd2 prev gmaj
bash tools/gpu_bench_ab.sh r03m_ab "EELG_LIB=$R/variants/libeelg_prev.so" "EELG_LIB=$R/variants/libeelg_pfd2.so"
