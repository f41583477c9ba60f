#!/bin/bash
# LDS-DMA tp_fwd (glds) knobs: 12 / 16 receivers per half-wave, two-wave workgroups
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"; mkdir -p gpurun_out/r03ah
for v in gnph12 gnph16 gwpb2; do
  EELG_LIB=$R/variants/libeelg_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
      -k "interaction" > gpurun_out/r03ah/t_$v.log 2>&1 || { tail -30 gpurun_out/r03ah/t_$v.log; exit 3; }
  echo "$v: $(tail -1 gpurun_out/r03ah/t_$v.log)"
done
bash tools/ab_kbench.sh "tp_fwd" main glds gnph12 gnph16 gwpb2
bash tools/gpu_bench_ab.sh r03ah_ab "EELG_LIB=$R/variants/libeelg_glds.so" "EELG_LIB=$R/variants/libeelg_gnph12.so" "EELG_LIB=$R/variants/libeelg_gnph16.so"
