#!/bin/bash
# tp_fwd: memory-pattern floor (no-compute variants) vs real kernels, and SQ counters of main / tpmA
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
bash tools/ab_kbench.sh "tp_fwd" main nc32 nc64 acc64 tpmA tpmC
bash tools/pmc_passes.sh r03e_main "tp_fwd"
EELG_LIB=$R/variants/libeelg_tpmA.so bash tools/pmc_passes.sh r03e_tpmA "tp_fwd"
for t in main tpmA; do echo "== $t"; python3 tools/pmc_table.py gpurun_out/pmc_r03e_$t tp_fwd_tpB_l4 | tee gpurun_out/pmc_r03e_$t/table.txt; done
