#!/bin/bash
# XCD-contiguous tp_fwd variants (parity + timing), MFMA PMC table, bench A/B of the best candidate
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
bash tools/ab_variants.sh main acc64 x32 x64 xm
bash tools/pmc_mfma.sh r03g_mfma
bash tools/gpu_bench_ab.sh r03g_ab "EELG_LIB=$R/variants/libeelg_x64.so" "EELG_LIB=$R/variants/libeelg_acc64.so"
bash tools/pmc_passes.sh r03g_scf "sc_fwd"
bash tools/pmc_passes.sh r03g_scx "sc_bwd_x"
for t in scf scx; do python3 tools/pmc_table.py gpurun_out/pmc_r03g_$t "sc_" | tee gpurun_out/pmc_r03g_$t/table.txt; done
