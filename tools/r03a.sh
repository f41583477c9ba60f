#!/bin/bash
# round-3 first GPU call: tp kernel A/B over path-group sizes, tp_fwd SQ counters
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
bash tools/ab_kbench.sh "tp_fwd|tp_bwd" main acc48 acc64
bash tools/pmc_passes.sh r03a "tp_fwd"
python3 tools/pmc_table.py gpurun_out/pmc_r03a tp_fwd_tpB_l4 > gpurun_out/pmc_r03a/table.txt
cat gpurun_out/pmc_r03a/table.txt
