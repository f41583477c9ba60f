#!/bin/bash
# Round-4 PMC passes (one counter group per rocprofv3 run) over kbench's TP backward,
# contraction and 7360 -> 800 linear kernels.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
timeout -k 10 900 bash tools/pmc_passes.sh r04l "tp_bwd|sc_|lin 7360" > gpurun_out/r04l_passes.log 2>&1
rc=$?
echo "passes rc=$rc"; tail -5 gpurun_out/r04l_passes.log
ls gpurun_out/pmc_r04l
