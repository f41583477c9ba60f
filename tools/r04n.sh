#!/bin/bash
# Round-4 PMC passes over kbench's radial MLP (forward and backward kernels) and the 800-wide
# linears.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
timeout -k 10 900 bash tools/pmc_passes.sh r04n "radial fwd\+bwd \(HIP\)|lin 800" > gpurun_out/r04n_passes.log 2>&1
echo "passes rc=$?"; tail -3 gpurun_out/r04n_passes.log
