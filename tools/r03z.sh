#!/bin/bash
# Clustered coefficient-gradient term groups (main) vs runs of the term order (coefrun);
# tp_fwd with 1 / 2 waves per workgroup (wpb1 / wpb2) vs 4 (main): parity, kbench, bench A/B
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"; mkdir -p gpurun_out/r03z
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
    -k "symcon or product_block or model_forward or interaction" > gpurun_out/r03z/t_main.log 2>&1 || { tail -30 gpurun_out/r03z/t_main.log; exit 3; }
echo "main: $(tail -1 gpurun_out/r03z/t_main.log)"
for v in wpb1 wpb2; do
  EELG_LIB=$R/variants/libeelg_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
      -k "interaction or model_forward_backward_matches_oracle and 4" > gpurun_out/r03z/t_$v.log 2>&1 || { tail -30 gpurun_out/r03z/t_$v.log; exit 3; }
  echo "$v: $(tail -1 gpurun_out/r03z/t_$v.log)"
done
bash tools/ab_kbench.sh "sc_bwd_coef" main coefrun
bash tools/ab_kbench.sh "tp_fwd" main wpb1 wpb2
bash tools/gpu_bench_ab.sh r03z_ab "EELG_LIB=$R/variants/libeelg_coefrun.so" "EELG_LIB=$R/variants/libeelg_wpb1.so"
