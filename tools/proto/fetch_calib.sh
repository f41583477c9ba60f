#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration passes (one counter per rocprofv3 run).
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
O=$R/gpurun_out/fetch_calib; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d "$O/$c" -o p -- "$R/tools/proto/fetch_calib" > "$O/$c.log" 2>&1
done
echo done > "$O/ok"
