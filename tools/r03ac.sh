#!/bin/bash
# host-side cost of the training step: enqueue time vs synchronised step time, op table by CPU time
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p "$R/gpurun_out/r03ac"; cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 python3 "$R/tools/hosttime.py" --steps 20 > "$R/gpurun_out/r03ac/hosttime.txt" 2>&1
cat "$R/gpurun_out/r03ac/hosttime.txt"
timeout -k 10 300 python3 "$R/tools/torchprof.py" --steps 3 > "$R/gpurun_out/r03ac/torchprof.txt" 2>&1
echo done
