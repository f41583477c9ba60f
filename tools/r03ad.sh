#!/bin/bash
# coefficient chain issued up front for every layer (EELG_COEF_AHEAD=1, default) vs at each
# layer (0): parity of the overlapped step, bench A/B
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"; mkdir -p gpurun_out/r03ad
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
    -k "overlap or model_forward_backward_matches_oracle or product_block" > gpurun_out/r03ad/t.log 2>&1 || { tail -30 gpurun_out/r03ad/t.log; exit 3; }
echo "tests: $(tail -1 gpurun_out/r03ad/t.log)"
bash tools/gpu_bench_ab.sh r03ad_ab "EELG_COEF_AHEAD=0"
