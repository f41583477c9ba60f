#!/bin/bash
# Round-4: step-level A/B of side-stream resource use -- the coefficient gradient with 256-node
# chunks (51 KB of LDS instead of 102 KB), in line instead of on the side stream, the radial
# forward at 3 waves/SIMD; two runs of the default build bracket them.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/r04p; mkdir -p "$O"
cd "$R"
step() {   # step <log> <timeout> <cmd...>: rc 0 / 1 continue, anything else ends the script
  local log=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "[$log] rc=$rc"; tail -20 "$O/$log"; exit $rc; fi
  python3 -c "import json; l=json.loads(open('$O/$log').read().strip().splitlines()[-1]); print('$log', l['value'], l['ms_per_step'])"
}
timeout -k 10 300 env EELG_LIB=$R/variants/libeelg_cc256.so python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "coef_grad or model_forward_backward" > "$O/t_cc256.log" 2>&1
rc=$?; echo "t_cc256 rc=$rc $(tail -1 "$O/t_cc256.log")"; [ $rc -le 1 ] || exit $rc
B="python3 bench.py --no-cpu-baseline"
step b_main1.json 300 $B
step b_cc256.json 300 env EELG_LIB=$R/variants/libeelg_cc256.so $B
step b_inline_coef.json 300 env EELG_SC_COEF_SIDE=0 $B
step b_rfw3.json 300 env EELG_LIB=$R/variants/libeelg_rfw3.so $B
step b_main2.json 300 $B
echo done > "$O/ok"
