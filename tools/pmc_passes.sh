#!/bin/bash
# SQ / SQC / TCC counter passes (one counter group per rocprofv3 run, as MI355X_MICROARCH.md
# prescribes) over tools/kbench.py for the kernels matching a regex.
# usage (GPU box): bash tools/pmc_passes.sh <tag> "<kbench --only regex>"; then
#   python tools/pmc_table.py gpurun_out/pmc_<tag> <kernel-name-regex>
set -e -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_$1; mkdir -p $O
ONLY=$2
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS" \
           "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_DCACHE_HITS SQC_DCACHE_MISSES" \
           "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $O/p$i -o p -- python3 $R/tools/kbench.py --reps 2 --only "$ONLY" > $O/p$i.log 2>&1
done
