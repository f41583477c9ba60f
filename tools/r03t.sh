#!/bin/bash
# tp_bwd block order: 2-D round-robin (main) vs XCD-contiguous edge ranges with the l1 groups
# adjacent (bm1) or per group (bm2): parity, kbench, bench A/B
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"; mkdir -p gpurun_out/r03t
for v in bm1 bm2; do
  EELG_LIB=$R/variants/libeelg_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bf16.py -x -q --timeout 300 --timeout-method thread \
      -k "interaction or model_forward or tp_bwd" > gpurun_out/r03t/t_$v.log 2>&1 || { tail -30 gpurun_out/r03t/t_$v.log; exit 3; }
  echo "$v: $(tail -1 gpurun_out/r03t/t_$v.log)"
done
bash tools/ab_kbench.sh "tp_bwd|segment_sum gxe" main bm1 bm2
bash tools/gpu_bench_ab.sh r03t_ab "EELG_LIB=$R/variants/libeelg_bm1.so" "EELG_LIB=$R/variants/libeelg_bm2.so"
