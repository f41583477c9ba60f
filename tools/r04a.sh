#!/bin/bash
# round-4 re-entry: full GPU suite (edgeless-batch tests new) + smoke + bench, then the isolated
# kbench of every kernel and an in-line (EELG_OVERLAP=0) kernel trace of the step
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
bash tools/gpu_full.sh r04a
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 "$R/tools/kbench.py" --reps 20 > "$R/gpurun_out/r04a/kbench.txt" 2>&1
EELG_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/r04a/inline" -o run \
    -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$R/gpurun_out/r04a/inline.log" 2>&1
echo done
