#!/bin/bash
# Round-4 closing pass after the grad-W grid change: the whole GPU suite, smoke, a default bench
# line (with the CPU baseline), the config-2 profile (kernel trace, FETCH / WRITE passes) and a
# kbench snapshot of every hot kernel.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/r04ad; mkdir -p "$O"
cd "$R"
step() {   # step <log> <timeout> <cmd...>: rc 0 / 1 continue, anything else ends the script
  local log=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?
  echo "[$log] rc=$rc $(tail -1 "$O/$log" | cut -c1-200)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; tail -20 "$O/$log"; exit $rc; fi
}
step tests.log 900 env EELG_PARITY_OUT=$O/parity.json python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread
grep -E "FAILED|passed|failed" "$O/tests.log" | tail -5
step smoke.log 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench.json 400 python3 bench.py
step prof_c2.log 900 bash tools/profile_round.sh gpurun_out/r04ad/c2
cd /tmp && export TMPDIR=/tmp
step kbench.txt 300 python3 "$R/tools/kbench.py" --reps 20
grep " ms" "$O/kbench.txt" | cut -c1-100
echo done > "$O/ok"
