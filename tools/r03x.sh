#!/bin/bash
# round-3 closing profile: bench + kernel trace + FETCH/WRITE passes, MFMA counters by shape,
# SQ counters of tp_fwd (the roofline kernel) and the contraction kernels
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
STEPS=10 bash tools/profile_round.sh gpurun_out/r03x
bash tools/pmc_mfma.sh r03x
bash tools/pmc_passes.sh r03x_k "tp_fwd|sc_"
