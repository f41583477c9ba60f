#!/bin/bash
# Round-4: torch-level glue of the training step by op and shape (which copies / reductions sit
# around the HIP kernels), and the tie-aware max / min reduction test.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/r04i; mkdir -p "$O"
cd "$R"
step() {   # step <log> <timeout> <cmd...>: rc 0 / 1 continue, anything else ends the script
  local log=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?
  echo "[$log] rc=$rc $(tail -1 "$O/$log")"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; tail -20 "$O/$log"; exit $rc; fi
}
step t_red.log 300 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_api.py -k "reductions"
step shapes.txt 300 python3 tools/torchprof_shapes.py --steps 2
cat "$O/shapes.txt" | cut -c1-170
echo done > "$O/ok"
