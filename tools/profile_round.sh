#!/bin/bash
# Round profile: bench line, rocprofv3 kernel-trace stats of the same bench command, and
# HBM traffic PMC passes (FETCH_SIZE and WRITE_SIZE in separate passes, MI355X_MICROARCH.md
# "HBM").  Every GPU step has its own time limit; the first failure ends the script.
# usage (on the GPU box): [BENCH_ARGS="--config 5"] tools/profile_round.sh gpurun_out/<tag>
# (BENCH_ARGS selects the workload: default config 2, "--config 5", "--model cgc_modified --batch 256")
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$(cd "$R" && mkdir -p "$1" && cd "$1" && pwd)
STEPS=${STEPS:-10}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 420 python3 "$R/bench.py" $BENCH_ARGS --steps "$STEPS" --warmup 3 --kernel-summary \
    > "$OUT/bench.json" 2> "$OUT/bench.err"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run \
    -- python3 "$R/bench.py" $BENCH_ARGS --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/trace.log" 2>&1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_$c" -o run \
      -- python3 "$R/bench.py" $BENCH_ARGS --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/pmc_$c.log" 2>&1
done
echo done > "$OUT/ok"
