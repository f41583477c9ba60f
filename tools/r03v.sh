#!/bin/bash
# tp_bwd with 2 / 3 paths of grad_agg + weight loads in flight (bp2 / bp3) vs 1 (main): parity,
# kbench, bench A/B
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"; mkdir -p gpurun_out/r03v
for v in bp2 bp3; do
  EELG_LIB=$R/variants/libeelg_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bf16.py -x -q --timeout 300 --timeout-method thread \
      -k "interaction or model_forward or tp_bwd" > gpurun_out/r03v/t_$v.log 2>&1 || { tail -30 gpurun_out/r03v/t_$v.log; exit 3; }
  echo "$v: $(tail -1 gpurun_out/r03v/t_$v.log)"
done
bash tools/ab_kbench.sh "tp_bwd" main bp2 bp3
bash tools/gpu_bench_ab.sh r03v_ab "EELG_LIB=$R/variants/libeelg_bp2.so" "EELG_LIB=$R/variants/libeelg_bp3.so"
