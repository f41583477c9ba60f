#!/bin/bash
# PMC passes over tools/kbench.py (one counter group per pass, as MI355X_MICROARCH.md prescribes).
# usage: tools/pmc.sh OUTDIR ONLY_REGEX
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$(cd "$R" && mkdir -p "$1" && cd "$1" && pwd); ONLY=$2
cd /tmp && export TMPDIR=/tmp
mkdir -p "$OUT"
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SMEM SQ_BUSY_CYCLES" \
           "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_DCACHE_HITS SQC_DCACHE_MISSES" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o p -- python3 "$R/tools/kbench.py" --reps 2 --only "$ONLY" > "$OUT/p$i.log" 2>&1 || echo "pass $i failed ($grp)"
done
