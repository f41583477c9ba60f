#!/bin/bash
# contraction fwd / grad-x with 2 or 4 node tiles per workgroup (shared coefficient stream
# through the scalar cache): parity, kbench against 1 tile (main) and cache-resident
# coefficients (scdiag, timing only), bench A/B
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"; mkdir -p gpurun_out/r03q
for v in nt2 nt4; do
  EELG_LIB=$R/variants/libeelg_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
      -k "product or symcon or model_forward" > gpurun_out/r03q/t_$v.log 2>&1 || { tail -30 gpurun_out/r03q/t_$v.log; exit 3; }
  echo "$v: $(tail -1 gpurun_out/r03q/t_$v.log)"
done
bash tools/ab_kbench.sh "sc_" main nt2 nt4 scdiag
bash tools/gpu_bench_ab.sh r03q_ab "EELG_LIB=$R/variants/libeelg_nt2.so"
