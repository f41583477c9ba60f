#!/bin/bash
# Round-4 pass 5: what bounds the contraction -- kbench of the packed / unpacked builds, their
# no-coefficient-load diagnostics (wrong results, timing only), and the packed coefficient
# gradient (64 / 32 terms per group) with its parity.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/r04e; mkdir -p "$O"
cd "$R"
step() {   # step <log> <timeout> <cmd...>: rc 0 / 1 continue, anything else ends the script
  local log=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?
  echo "[$log] rc=$rc $(tail -1 "$O/$log")"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; tail -20 "$O/$log"; exit $rc; fi
}
PYT="python -u -m pytest -q --timeout 300 --timeout-method thread"
for v in cpk64 cpk32; do
  step t_$v.log 300 env EELG_LIB=$R/variants/libeelg_$v.so $PYT tests/test_gpu_parity.py -k "coef_grad"
done
cd /tmp && export TMPDIR=/tmp
for v in main scpk0 diag0 diag1 cpk64 cpk32; do
  if [ $v = main ]; then L=""; else L="EELG_LIB=$R/variants/libeelg_$v.so"; fi
  step k_$v.txt 200 env $L python3 "$R/tools/kbench.py" --reps 20 --only "sc_"
  grep " ms" "$O/k_$v.txt" | cut -c1-100
done
echo done > "$O/ok"
