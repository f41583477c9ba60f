#!/bin/bash
# Round-4 measurement pass: the whole GPU suite and smoke, then the round's profiles (bench line,
# kernel trace, FETCH / WRITE PMC passes) of config 2, config 5 and the CGC benchmark model.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/r04u; mkdir -p "$O"
cd "$R"
step() {   # step <log> <timeout> <cmd...>: rc 0 / 1 continue, anything else ends the script
  local log=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?
  echo "[$log] rc=$rc $(tail -1 "$O/$log")"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; tail -20 "$O/$log"; exit $rc; fi
}
step tests.log 900 env EELG_PARITY_OUT=$O/parity.json python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread
grep -E "FAILED|passed|failed" "$O/tests.log" | tail -8
step smoke.log 300 python -c "import __graft_entry__ as g; g.smoke()"
step prof_c2.log 900 bash tools/profile_round.sh gpurun_out/r04u/c2
tail -1 "$O/c2/bench.json" | cut -c1-400
step prof_c5.log 900 env BENCH_ARGS="--config 5" bash tools/profile_round.sh gpurun_out/r04u/c5
tail -1 "$O/c5/bench.json" | cut -c1-400
step prof_cgc.log 900 env BENCH_ARGS="--model cgc_modified --batch 256" bash tools/profile_round.sh gpurun_out/r04u/cgc
tail -1 "$O/cgc/bench.json" | cut -c1-400
echo done > "$O/ok"
