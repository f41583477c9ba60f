#!/bin/bash
# bench entry points of BASELINE configs 4 and 5 (tests/test_gpu_bench_configs.py)
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"; mkdir -p gpurun_out/r03ae
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_configs.py -v --timeout 300 --timeout-method thread \
    > gpurun_out/r03ae/t.log 2>&1 || { tail -40 gpurun_out/r03ae/t.log; exit 3; }
tail -5 gpurun_out/r03ae/t.log
