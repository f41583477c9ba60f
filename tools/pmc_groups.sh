#!/bin/bash
# Named counter groups over tools/kbench.py for the kernels matching a regex, one rocprofv3 --pmc
# run per group (MI355X_MICROARCH.md: <= 8 SQ, <= 4 TCC counters per pass), each under a KILL
# time limit.  Groups are given with ',' between counters.
# usage (GPU box): bash tools/pmc_groups.sh <tag> "<kbench --only regex>" "C1,C2,..." ["C3,..."]
# then: python tools/pmc_table.py gpurun_out/pmcg_<tag> <kernel-name-regex>
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/pmcg_$1; mkdir -p "$O"
ONLY=$2; shift 2
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc ${grp//,/ } --output-format csv -d "$O/p$i" -o p \
      -- python3 "$R/tools/kbench.py" --reps 2 --only "$ONLY" > "$O/p$i.log" 2>&1
  rc=$?
  echo "[pmc $i: $grp] rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
echo done > "$O/ok"
