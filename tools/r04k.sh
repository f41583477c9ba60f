#!/bin/bash
# Round-4: split-bf16 linears with the single-chunk B tile in registers -- parity, then kbench of
# the linears on the fp32 kernels, the default rule, every descriptor packed (MINK=0), and
# 4 / 8 node groups per wave.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/r04k; mkdir -p "$O"
cd "$R"
step() {   # step <log> <timeout> <cmd...>: rc 0 / 1 continue, anything else ends the script
  local log=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?
  echo "[$log] rc=$rc $(tail -1 "$O/$log")"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; tail -20 "$O/$log"; exit $rc; fi
}
PYT="python -u -m pytest -q --timeout 300 --timeout-method thread"
step t_lin.log 300 $PYT tests/test_gpu_parity.py -k "linear"
for v in lgpw4 lgpw8; do
  step t_$v.log 300 env EELG_LIB=$R/variants/libeelg_$v.so $PYT tests/test_gpu_parity.py -k "packed_split"
done
cd /tmp && export TMPDIR=/tmp
step k_f32.txt 200 env EELG_LIN_X6=0 python3 "$R/tools/kbench.py" --reps 20 --only "lin"
grep " ms" "$O/k_f32.txt" | cut -c1-100
step k_main.txt 200 python3 "$R/tools/kbench.py" --reps 20 --only "lin"
grep " ms" "$O/k_main.txt" | cut -c1-100
step k_all.txt 200 env EELG_LIN_X6_MINK=0 python3 "$R/tools/kbench.py" --reps 20 --only "lin"
grep " ms" "$O/k_all.txt" | cut -c1-100
for v in lgpw4 lgpw8; do
  step k_$v.txt 200 env EELG_LIN_X6_MINK=0 EELG_LIB=$R/variants/libeelg_$v.so python3 "$R/tools/kbench.py" --reps 20 --only "lin"
  grep " ms" "$O/k_$v.txt" | cut -c1-100
done
echo done > "$O/ok"
