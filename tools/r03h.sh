#!/bin/bash
# symmetric contraction node tiles per workgroup: 2 (cur) vs 1 (nt1): parity + kbench + bench A/B
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"; mkdir -p gpurun_out/r03h
for v in cur nt1; do
  EELG_LIB=$R/variants/libeelg_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
      -k "product or symcon or model_forward" > gpurun_out/r03h/t_$v.log 2>&1 || { tail -30 gpurun_out/r03h/t_$v.log; exit 3; }
  echo "$v: $(tail -1 gpurun_out/r03h/t_$v.log)"
done
bash tools/ab_kbench.sh "sc_|tp_fwd" cur nt1 x64
bash tools/gpu_bench_ab.sh r03h_ab "EELG_LIB=$R/variants/libeelg_cur.so" "EELG_LIB=$R/variants/libeelg_nt1.so"
