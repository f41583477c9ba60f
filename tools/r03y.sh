#!/bin/bash
# in-line (EELG_OVERLAP=0) kernel trace of the bench step: the per-kernel cost table of DESIGN 3.7
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p "$R/gpurun_out/r03y"
cd /tmp && export TMPDIR=/tmp
EELG_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/r03y/inline" -o run \
    -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$R/gpurun_out/r03y/inline.log" 2>&1
EELG_OVERLAP=0 timeout -k 10 200 python3 "$R/bench.py" --no-cpu-baseline > "$R/gpurun_out/r03y/inline_bench.json"
timeout -k 10 200 python3 "$R/bench.py" --no-cpu-baseline > "$R/gpurun_out/r03y/bench.json"
cat "$R/gpurun_out/r03y/inline_bench.json" "$R/gpurun_out/r03y/bench.json" | cut -c1-200
