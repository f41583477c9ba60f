#!/bin/bash
# Round-4 pass 3: packed-FMA microbenchmark, parity of the round's fixes (packed-linear stride,
# edgeless batches, hi/lo radial accumulators), kbench of the restored scalar contraction, and a
# default bench line.  A failing test (pytest rc 1) does not stop the script; anything else does.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/r04c; mkdir -p "$O"
cd "$R"
step() {   # step <log> <timeout> <cmd...>: rc 0 / 1 continue, anything else ends the script
  local log=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?
  echo "[$log] rc=$rc $(tail -1 "$O/$log")"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; tail -20 "$O/$log"; exit $rc; fi
}
PYT="python -u -m pytest -q --timeout 300 --timeout-method thread"
step pkfma.txt 60 tools/proto/pkfma_bench
cat "$O/pkfma.txt"
step t_fix.log 600 $PYT tests/test_gpu_parity.py tests/test_gpu_radial.py tests/test_gpu_fullsize.py tests/test_gpu_bf16.py -k "linear or radial or edgeless or no_edges or sender_position or symcon"
grep -E "passed|failed" "$O/t_fix.log" | tail -3
cd /tmp && export TMPDIR=/tmp
step k_main.txt 200 python3 "$R/tools/kbench.py" --reps 20
grep " ms" "$O/k_main.txt" | cut -c1-100
cd "$R"
step bench.json 300 python3 bench.py
tail -1 "$O/bench.json"
echo done > "$O/ok"
