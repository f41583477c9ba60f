#!/bin/bash
# residual-templated fast linear (main) vs HEAD (prev): parity + kbench; contraction kernels
# with cache-resident coefficients (scdiag, wrong results, timing only); SQ counter passes of
# the contraction kernels after the staging rewrite
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"; mkdir -p gpurun_out/r03p
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "linear or model_forward or product" \
    > gpurun_out/r03p/t.log 2>&1 || { tail -30 gpurun_out/r03p/t.log; exit 3; }
tail -1 gpurun_out/r03p/t.log
bash tools/ab_kbench.sh "sc_|lin " main prev scdiag
bash tools/pmc_passes.sh r03p_sc "sc_"
