#!/bin/bash
# MFMA-utilisation counters of the MFMA kernels (channel-mixing linears, radial MLP) at the bench
# shapes, one counter group per rocprofv3 pass (MI355X_MICROARCH.md), over tools/kbench.py.
# usage (GPU box): bash tools/pmc_mfma.sh <tag>   -> gpurun_out/pmc_<tag>/p*/  + mfma table
set -e -o pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/pmc_$1; mkdir -p "$O"
ONLY="lin 7360->800|lin 800->800|radial fwd"
i=0
for grp in "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU_MFMA_F32 SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$O/p$i" -o p -- \
      python3 "$R/tools/kbench.py" --reps 3 --only "$ONLY" > "$O/p$i.log" 2>&1
done
python3 "$R/tools/mfma_table.py" "$O" > "$O/table.md"
cat "$O/table.md"
