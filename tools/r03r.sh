#!/bin/bash
# contraction coefficient blocks packed to even sizes (main: 32 terms, prefetch 1 / 2 blocks;
# b16p3: 16 terms, 3 / 4; b16p2: 16, 2 / 3; b24: 24, 2 / 2): parity, kbench, bench A/B
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"; mkdir -p gpurun_out/r03r
for v in main b16p2; do
  if [ $v = main ]; then L=""; else L=$R/variants/libeelg_$v.so; fi
  EELG_LIB=$L timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
      -k "product or symcon or model_forward" > gpurun_out/r03r/t_$v.log 2>&1 || { tail -30 gpurun_out/r03r/t_$v.log; exit 3; }
  echo "$v: $(tail -1 gpurun_out/r03r/t_$v.log)"
done
bash tools/ab_kbench.sh "sc_fwd|sc_bwd_x" main b16p3 b16p2 b24 scdiag
bash tools/gpu_bench_ab.sh r03r_ab "EELG_LIB=$R/variants/libeelg_b16p3.so" "EELG_LIB=$R/variants/libeelg_b16p2.so"
