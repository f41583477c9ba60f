#!/bin/bash
# r02c: isolated per-kernel timings (kbench, radial_bench) and an in-line (no side streams)
# kernel-trace profile of the bench command.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/${1:-r02c}
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 "$R/tools/kbench.py" --reps 20 > "$O/kbench.txt" 2>&1
timeout -k 10 300 python3 "$R/tools/radial_bench.py" > "$O/radial.txt" 2>&1
EELG_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o run \
    -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$O/trace.log" 2>&1
echo done > "$O/ok"
