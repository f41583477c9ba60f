#!/bin/bash
# SC coefficient stream by LDS-DMA: parity of the new kernels (default + variants), kbench A/B
# against the round-3 SMEM stream (variants/head), then the full GPU suite + bench + profiles
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/r04b; mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 400 --timeout-method thread \
   -k "symcon or model_forward_backward_matches_oracle" > "$O/t_main.log" 2>&1 || { tail -30 "$O/t_main.log"; exit 3; }
echo "main: $(tail -1 $O/t_main.log)"
for v in csb16d4 csb16d2 csc256 csb32d3; do
  EELG_LIB=$R/variants/libeelg_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread \
     -k "symcon" > "$O/t_$v.log" 2>&1 || { tail -30 "$O/t_$v.log"; exit 3; }
  echo "$v: $(tail -1 $O/t_$v.log)"
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_radial.py -x -q --timeout 240 --timeout-method thread > "$O/t_radial.log" 2>&1 || { tail -30 "$O/t_radial.log"; exit 3; }
EELG_LIB=$R/variants/libeelg_rads2.so timeout -k 10 300 python -u -m pytest tests/test_gpu_radial.py -x -q --timeout 240 --timeout-method thread > "$O/t_radial_s2.log" 2>&1 || { tail -30 "$O/t_radial_s2.log"; exit 3; }
echo "radial s2: $(tail -1 $O/t_radial_s2.log)"
echo "radial: $(tail -1 $O/t_radial.log)"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread -k "linear" > "$O/t_lin.log" 2>&1 || { tail -30 "$O/t_lin.log"; exit 3; }
echo "linear: $(tail -1 $O/t_lin.log)"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 python3 "$R/variants/head/tools/kbench.py" --reps 20 --only "sc_|radial|lin" > "$O/k_head.txt" 2>&1
echo "== head"; grep " ms" "$O/k_head.txt" | cut -c1-90
bash "$R/tools/ab_kbench.sh" "sc_|radial|lin" main
EELG_LIN_X6=0 timeout -k 10 200 python3 "$R/tools/kbench.py" --reps 20 --only "lin" > "$O/k_main_linf32.txt" 2>&1
echo "== main, EELG_LIN_X6=0"; grep " ms" "$O/k_main_linf32.txt" | cut -c1-90
bash "$R/tools/ab_kbench.sh" "radial" rads2
bash "$R/tools/ab_kbench.sh" "sc_" csb16d4 csb16d2 csc256 csb32d3
cd "$R"
echo done > "$O/ok"
