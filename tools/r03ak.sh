#!/bin/bash
# two-edge LDS-DMA tp_fwd: 6 / 10 receivers per half-wave vs 8 (main)
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"; mkdir -p gpurun_out/r03ak
for v in g2nph6 g2nph10; do
  EELG_LIB=$R/variants/libeelg_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
      -k "interaction" > gpurun_out/r03ak/t_$v.log 2>&1 || { tail -30 gpurun_out/r03ak/t_$v.log; exit 3; }
  echo "$v: $(tail -1 gpurun_out/r03ak/t_$v.log)"
done
bash tools/ab_kbench.sh "tp_fwd" main g2nph6 g2nph10
bash tools/gpu_bench_ab.sh r03ak_ab "EELG_LIB=$R/variants/libeelg_g2nph6.so" "EELG_LIB=$R/variants/libeelg_g2nph10.so"
