#!/bin/bash
# new API GPU tests, then the tp kernel A/B over path-group sizes and tp_fwd SQ counters
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"; mkdir -p gpurun_out/r03b
timeout -k 10 600 python -u -m pytest tests/test_gpu_api.py tests/test_gpu_checkpoint.py tests/test_gpu_radial.py \
    "tests/test_gpu_parity.py::test_model_global_reductions_match_oracle" -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/r03b/tests.log 2>&1 || { tail -40 gpurun_out/r03b/tests.log; exit 3; }
tail -3 gpurun_out/r03b/tests.log
bash tools/r03a.sh
