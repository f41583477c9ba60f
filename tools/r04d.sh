#!/bin/bash
# Round-4 pass 4: the contraction on packed f32 VALU (two nodes per lane): parity, kbench A/B
# against the one-node-per-lane build and the waves-per-EU variants, then the bench line.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/r04d; mkdir -p "$O"
cd "$R"
step() {   # step <log> <timeout> <cmd...>: rc 0 / 1 continue, anything else ends the script
  local log=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?
  echo "[$log] rc=$rc $(tail -1 "$O/$log")"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; tail -20 "$O/$log"; exit $rc; fi
}
PYT="python -u -m pytest -q --timeout 300 --timeout-method thread"
step t_sc.log 600 $PYT tests/test_gpu_parity.py tests/test_gpu_api.py tests/test_gpu_fullsize.py -k "symcon or symmetric or contraction or product or model_forward_backward"
grep -E "passed|failed|Error" "$O/t_sc.log" | tail -5
cd /tmp && export TMPDIR=/tmp
for v in main scpk0 scpkw3 scpkw33; do
  if [ $v = main ]; then L=""; else L="EELG_LIB=$R/variants/libeelg_$v.so"; fi
  step k_$v.txt 200 env $L python3 "$R/tools/kbench.py" --reps 20 --only "sc_"
  grep " ms" "$O/k_$v.txt" | cut -c1-100
done
cd "$R"
step bench.json 300 python3 bench.py
tail -1 "$O/bench.json" | cut -c1-300
echo done > "$O/ok"
