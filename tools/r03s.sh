#!/bin/bash
# larger contraction coefficient blocks with one block of prefetch (b40 / b48 / b64) vs 32-term
# blocks (main): kbench, then parity of the variants
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"; mkdir -p gpurun_out/r03s
bash tools/ab_kbench.sh "sc_fwd|sc_bwd_x" main b40 b48 b64
for v in b48 b64; do
  EELG_LIB=$R/variants/libeelg_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
      -k "product or symcon" > gpurun_out/r03s/t_$v.log 2>&1 || { tail -30 gpurun_out/r03s/t_$v.log; exit 3; }
  echo "$v: $(tail -1 gpurun_out/r03s/t_$v.log)"
done
