#!/bin/bash
# Round-4 first GPU pass over the new kernels (SC coefficient stream by LDS-DMA, split-bf16 radial
# and linears, receiver-major tp_bwd, bf16 LDS-DMA tp_fwd, batched CGC): parity of each, then
# kbench A/B against the round-3 build (variants/head).  A failing test (pytest rc 1) does not
# stop the script; any other failure (fault, abort, timeout) does.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/r04b; mkdir -p "$O"
cd "$R"
step() {   # step <log> <timeout> <cmd...>: rc 0 / 1 continue, anything else ends the script
  local log=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?
  echo "[$log] rc=$rc $(tail -1 "$O/$log")"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; tail -20 "$O/$log"; exit $rc; fi
}
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
step t_lin.log 300 $PYT tests/test_gpu_parity.py -k "linear"
step t_radial.log 300 $PYT tests/test_gpu_radial.py
step t_tpbwr.log 300 $PYT tests/test_gpu_fullsize.py -k "receiver_major or edgeless or no_edges"
step t_model.log 600 $PYT tests/test_gpu_parity.py -k "model_forward_backward_matches_oracle or other_radial"
step t_bf16.log 400 $PYT tests/test_gpu_bf16.py
step t_cgc.log 400 $PYT tests/test_cgc.py -m gpu
cd /tmp && export TMPDIR=/tmp
step k_head.txt 200 python3 "$R/variants/head/tools/kbench.py" --reps 20
grep " ms" "$O/k_head.txt" | cut -c1-100
step k_main.txt 200 python3 "$R/tools/kbench.py" --reps 20
grep " ms" "$O/k_main.txt" | cut -c1-100
step k_linf32.txt 200 env EELG_LIN_X6=0 python3 "$R/tools/kbench.py" --reps 20 --only "lin"
grep " ms" "$O/k_linf32.txt" | cut -c1-100
for v in csb16d4 csb16d2 csc256 csb32d3 rads2; do
  step k_$v.txt 200 env EELG_LIB=$R/variants/libeelg_$v.so python3 "$R/tools/kbench.py" --reps 20 --only "sc_|radial"
  grep " ms" "$O/k_$v.txt" | cut -c1-100
done
echo done > "$O/ok"
