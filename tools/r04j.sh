#!/bin/bash
# Round-4: device partial sums (eelg_sum_rows) -- their test, the parity tests of every caller,
# the bench line and the torch-level glue profile.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/r04j; mkdir -p "$O"
cd "$R"
step() {   # step <log> <timeout> <cmd...>: rc 0 / 1 continue, anything else ends the script
  local log=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?
  echo "[$log] rc=$rc $(tail -1 "$O/$log")"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; tail -20 "$O/$log"; exit $rc; fi
}
PYT="python -u -m pytest -q --timeout 300 --timeout-method thread"
step t_red.log 300 $PYT tests/test_gpu_reduce.py
grep -E "FAILED|Error" "$O/t_red.log" | head -5
step t_par.log 700 $PYT tests/test_gpu_parity.py tests/test_gpu_api.py tests/test_gpu_radial.py tests/test_cgc.py tests/test_gpu_oracle_fullsize.py -m gpu
grep -E "FAILED|passed|failed" "$O/t_par.log" | tail -5
step bench.json 300 python3 bench.py --no-cpu-baseline
tail -1 "$O/bench.json" | cut -c1-220
step shapes.txt 300 python3 tools/torchprof_shapes.py --steps 2
grep "us/step" "$O/shapes.txt" | head -16 | cut -c1-150
echo done > "$O/ok"
