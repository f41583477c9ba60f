#!/bin/bash
# Round-4: two node chunks in flight per wave in the linears' fast grad-W (parity, kbench, step A/B).
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/r04y; mkdir -p "$O"
cd "$R"
run() { local log=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; [ $rc -le 1 ] || { echo "[$log] rc=$rc"; tail -20 "$O/$log"; exit $rc; }; echo "[$log] rc=$rc $(tail -1 "$O/$log" | cut -c1-120)"; }
PYT="python -u -m pytest -q --timeout 300 --timeout-method thread"
run t_wntx.log 400 env EELG_LIB=$R/variants/libeelg_wpfd2.so $PYT tests/test_gpu_parity.py -k "linear"
cd /tmp && export TMPDIR=/tmp
for v in main wpfd2; do
  if [ $v = main ]; then L=""; else L="EELG_LIB=$R/variants/libeelg_$v.so"; fi
  run k_$v.txt 200 env $L python3 "$R/tools/kbench.py" --reps 20 --only "lin"
  grep " ms" "$O/k_$v.txt" | cut -c1-100
done
cd "$R"
for v in main wpfd2 main wpfd2; do
  if [ $v = main ]; then L=""; else L="EELG_LIB=$R/variants/libeelg_$v.so"; fi
  timeout -k 10 300 env $L python3 bench.py --no-cpu-baseline > "$O/b.json" 2>&1 || exit 3
  python3 -c "import json; l=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print('$v', l['value'], l['ms_per_step'])"
done
echo done > "$O/ok"
