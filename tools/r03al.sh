#!/bin/bash
# SQ counters of the LDS-DMA tp_fwd (default build)
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
export GRAFT_REPO_ROOT=$R
bash "$R/tools/pmc_passes.sh" r03al "tp_fwd"
echo done
