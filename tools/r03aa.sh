#!/bin/bash
# Re-entry check of HEAD: full GPU suite + smoke + default bench, then the round profile
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
bash tools/gpu_full.sh r03aa
STEPS=10 bash tools/profile_round.sh gpurun_out/r03aa_prof
