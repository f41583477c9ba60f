#!/bin/bash
# coop tp_fwd variants (parity + timing), then the new data-path and config-3 entry-point tests
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"; mkdir -p gpurun_out/r03f
bash tools/ab_variants.sh main acc64 coA coB coC
timeout -k 10 600 python -u -m pytest tests/test_gpu_datapath.py tests/test_gpu_bench_dp.py -x -v --timeout 400 --timeout-method thread \
    > gpurun_out/r03f/tests.log 2>&1 || { tail -40 gpurun_out/r03f/tests.log; exit 3; }
tail -5 gpurun_out/r03f/tests.log
