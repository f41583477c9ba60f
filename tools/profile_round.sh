#!/bin/bash
# Round profile: bench line, rocprofv3 kernel-trace stats of the same bench command, and
# HBM traffic PMC passes (FETCH_SIZE and WRITE_SIZE in separate passes, MI355X_MICROARCH.md
# "HBM").  Every GPU step has its own time limit; the first failure ends the script.
# usage (on the GPU box): [BENCH_ARGS="--config 5"] tools/profile_round.sh gpurun_out/<tag>
# (BENCH_ARGS selects the workload: default config 2, "--config 5", "--model cgc_modified --batch 256")
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$(cd "$R" && mkdir -p "$1" && cd "$1" && pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 420 python3 "$R/bench.py" $BENCH_ARGS --gpus 1 --steps 20 --warmup 5 --kernel-summary \
    > "$OUT/bench.json" 2> "$OUT/bench.err"
# the trace runs the driver's own bench command (--steps 20 --warmup 5, BENCH_r04.json "cmd"), so
# the trace's per-launch durations over the timed steps compare with the HIP-event figure that
# the same process prints (trace.json) and with the driver's line
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run \
    -- python3 "$R/bench.py" $BENCH_ARGS --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline \
    > "$OUT/trace.json" 2> "$OUT/trace.log"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_$c" -o run \
      -- python3 "$R/bench.py" $BENCH_ARGS --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/pmc_$c.log" 2>&1
done
echo done > "$OUT/ok"
