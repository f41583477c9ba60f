#!/bin/bash
# Round-4: config-5 (bf16 storage, 5k-node lattices) and config-4 (mCGC) profiles with the
# closing build (bench line with CPU baseline, kernel trace, FETCH / WRITE passes).
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/r04ae; mkdir -p "$O"
cd "$R"
step() {   # step <log> <timeout> <cmd...>: rc 0 / 1 continue, anything else ends the script
  local log=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?
  echo "[$log] rc=$rc $(tail -1 "$O/$log" | cut -c1-200)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; tail -20 "$O/$log"; exit $rc; fi
}
step prof_c5.log 900 env BENCH_ARGS="--config 5" bash tools/profile_round.sh gpurun_out/r04ae/c5
tail -1 "$O/c5/bench.json" | cut -c1-300
step prof_cgc.log 900 env BENCH_ARGS="--model cgc_modified --batch 256" bash tools/profile_round.sh gpurun_out/r04ae/cgc
tail -1 "$O/cgc/bench.json" | cut -c1-300
echo done > "$O/ok"
