#!/bin/bash
# Round-4: CGC backward with batched edge gathers, and edges per batch 2 / 4 / 8 -- parity, then
# the cgc_modified bench line of each (roofline of cgc_fwd, step time).
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/r04m; mkdir -p "$O"
cd "$R"
step() {   # step <log> <timeout> <cmd...>: rc 0 / 1 continue, anything else ends the script
  local log=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?
  echo "[$log] rc=$rc $(tail -1 "$O/$log" | cut -c1-150)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; tail -20 "$O/$log"; exit $rc; fi
}
PYT="python -u -m pytest -q --timeout 300 --timeout-method thread"
step t_cgc.log 400 $PYT tests/test_cgc.py -m gpu
for v in cgc8 cgc2; do
  step t_$v.log 400 env EELG_LIB=$R/variants/libeelg_$v.so $PYT tests/test_cgc.py -m gpu -k "layer"
done
for v in main cgc8 cgc2 main; do
  if [ $v = main ]; then L=""; else L="EELG_LIB=$R/variants/libeelg_$v.so"; fi
  step b_$v.json 300 env $L python3 bench.py --model cgc_modified --batch 256 --no-cpu-baseline
  python3 -c "import json,sys; l=json.loads(open('$O/b_$v.json').read().strip().splitlines()[-1]); print('$v', l['value'], l['ms_per_step'], l['roofline']['frac'], l['roofline']['mean_ms'])"
done
echo done > "$O/ok"
