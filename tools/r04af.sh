#!/bin/bash
# Round-4: config-5 and config-4 bench lines (CPU baseline and PMC traffic) after the traffic
# lookup fix, plus the default config-2 line.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/r04af; mkdir -p "$O"
cd "$R"
timeout -k 10 400 python3 bench.py --config 5 > "$O/bench_c5.json" 2> "$O/c5.err" || exit 3
tail -1 "$O/bench_c5.json" | cut -c1-200
sleep 20
timeout -k 10 400 python3 bench.py --model cgc_modified --batch 256 > "$O/bench_cgc.json" 2> "$O/cgc.err" || exit 4
tail -1 "$O/bench_cgc.json" | cut -c1-200
timeout -k 10 400 python3 bench.py > "$O/bench_c2.json" 2> "$O/c2.err" || exit 5
tail -1 "$O/bench_c2.json" | cut -c1-200
echo done > "$O/ok"
