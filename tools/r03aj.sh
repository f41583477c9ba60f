#!/bin/bash
# tp_fwd with two edges in flight by LDS-DMA as the default: full GPU suite + smoke + bench, then
# the round profile (kernel trace, FETCH/WRITE)
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
bash tools/gpu_full.sh r03aj
STEPS=10 bash tools/profile_round.sh gpurun_out/r03aj_prof
