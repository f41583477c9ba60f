#!/bin/bash
# round-3 profile: SC coefficient-latency diagnostic (kbench, cache-resident coefficients),
# round profile (bench + kernel trace + FETCH/WRITE passes), MFMA counters of the MFMA kernels
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
bash tools/ab_kbench.sh "sc_" main scdiag
STEPS=10 bash tools/profile_round.sh gpurun_out/r03j
bash tools/pmc_mfma.sh r03j
