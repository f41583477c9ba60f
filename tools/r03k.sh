#!/bin/bash
# XCD-grouped channel quads in the contraction kernels: parity, kbench A/B against the previous
# library, then SQ/TCC counter passes of the contraction and tp_fwd kernels
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"; mkdir -p gpurun_out/r03k
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_api.py -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r03k/tests.log 2>&1 || { tail -30 gpurun_out/r03k/tests.log; exit 3; }
tail -1 gpurun_out/r03k/tests.log
bash tools/ab_kbench.sh "sc_" main prev
bash tools/pmc_passes.sh r03k_sc "sc_"
bash tools/pmc_passes.sh r03k_tp "tp_fwd"
