#!/bin/bash
# The tools/pmc.sh counter groups (one group per rocprofv3 run) over any python script.
# usage: tools/pmc_cmd.sh OUTDIR script.py [args...]
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$(cd "$R" && mkdir -p "$1" && cd "$1" && pwd); shift
SCRIPT=$(cd "$R" && realpath "$1"); shift
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SMEM SQ_BUSY_CYCLES" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o p -- python3 "$SCRIPT" "$@" > "$OUT/p$i.log" 2>&1 || echo "pass $i failed ($grp)"
done
