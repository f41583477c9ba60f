#!/bin/bash
# Round-4: fp32 linear fast path (LINF) node groups per wave 2 / 8, two K chunks in flight, and
# 4-wave workgroups, with nontemporal stores on (parity, kbench of the linears, step).
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/r04ai; mkdir -p "$O"
cd "$R"
PYT="python -u -m pytest -q --timeout 300 --timeout-method thread"
for v in gpw2 gpw8 pfd2 w4g8; do
  timeout -k 10 400 env EELG_LIB=$R/variants/libeelg_$v.so $PYT tests/test_gpu_parity.py -k "linear or model_forward_backward" > "$O/t_$v.log" 2>&1
  rc=$?; echo "t_$v rc=$rc $(tail -1 "$O/t_$v.log")"; [ $rc -le 1 ] || exit $rc
done
cd /tmp && export TMPDIR=/tmp
for v in main gpw2 gpw8 pfd2 w4g8; do
  if [ $v = main ]; then L=""; else L="EELG_LIB=$R/variants/libeelg_$v.so"; fi
  timeout -k 10 200 env $L python3 "$R/tools/kbench.py" --reps 20 --only "lin" > "$O/k_$v.txt" 2>&1 || exit 3
  echo "== $v"; grep " ms" "$O/k_$v.txt" | cut -c1-100
done
cd "$R"
for v in main gpw2 gpw8 pfd2 w4g8 main; do
  if [ $v = main ]; then L=""; else L="EELG_LIB=$R/variants/libeelg_$v.so"; fi
  timeout -k 10 300 env $L python3 bench.py --no-cpu-baseline > "$O/b_$v.json" 2>&1 || exit 4
  python3 -c "import json; l=json.loads(open('$O/b_$v.json').read().strip().splitlines()[-1]); print('$v', l['value'], l['ms_per_step'], l['roofline']['frac'], l['roofline']['mean_ms'])"
done
echo done > "$O/ok"
