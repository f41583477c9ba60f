#!/bin/bash
# Round-4: radial forward with its LDS region shared between the hidden activations and the
# W_o blocks, column tiles per stage (1 / 2) and waves per SIMD (compiler / 3) -- parity of each,
# then kbench of the radial MLP.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/r04o; mkdir -p "$O"
cd "$R"
step() {   # step <log> <timeout> <cmd...>: rc 0 / 1 continue, anything else ends the script
  local log=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?
  echo "[$log] rc=$rc $(tail -1 "$O/$log" | cut -c1-150)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; tail -20 "$O/$log"; exit $rc; fi
}
PYT="python -u -m pytest -q --timeout 300 --timeout-method thread"
step t_main.log 300 $PYT tests/test_gpu_radial.py
for v in rf2 rfw3 rf2w3; do
  step t_$v.log 300 env EELG_LIB=$R/variants/libeelg_$v.so $PYT tests/test_gpu_radial.py
done
cd /tmp && export TMPDIR=/tmp
for v in main rf2 rfw3 rf2w3 main; do
  if [ $v = main ]; then L=""; else L="EELG_LIB=$R/variants/libeelg_$v.so"; fi
  step k_$v.txt 200 env $L python3 "$R/tools/kbench.py" --reps 30 --only "radial.*HIP"
  grep " ms" "$O/k_$v.txt" | cut -c1-100
done
echo done > "$O/ok"
