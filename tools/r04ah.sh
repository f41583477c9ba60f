#!/bin/bash
# Round-4: tp_bwd paths in flight (1 / 2 / 3) and tp_fwd waves per workgroup (2) / waves per EU (3)
# with the round-end build (parity of each, kbench, step with roofline).
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/r04ah; mkdir -p "$O"
cd "$R"
PYT="python -u -m pytest -q --timeout 300 --timeout-method thread"
for v in pfd3 pfd1 wpb2 wpe3; do
  timeout -k 10 400 env EELG_LIB=$R/variants/libeelg_$v.so $PYT tests/test_gpu_parity.py -k "interaction_block or model_forward_backward" > "$O/t_$v.log" 2>&1
  rc=$?; echo "t_$v rc=$rc $(tail -1 "$O/t_$v.log")"; [ $rc -le 1 ] || exit $rc
done
cd /tmp && export TMPDIR=/tmp
for v in main pfd3 pfd1 wpb2 wpe3; do
  if [ $v = main ]; then L=""; else L="EELG_LIB=$R/variants/libeelg_$v.so"; fi
  timeout -k 10 200 env $L python3 "$R/tools/kbench.py" --reps 20 --only "tp_fwd|tp_bwd" > "$O/k_$v.txt" 2>&1 || exit 3
  echo "== $v"; grep " ms" "$O/k_$v.txt" | cut -c1-100
done
cd "$R"
for v in main pfd3 pfd1 wpb2 wpe3 main; do
  if [ $v = main ]; then L=""; else L="EELG_LIB=$R/variants/libeelg_$v.so"; fi
  timeout -k 10 300 env $L python3 bench.py --no-cpu-baseline > "$O/b_$v.json" 2>&1 || exit 4
  python3 -c "import json; l=json.loads(open('$O/b_$v.json').read().strip().splitlines()[-1]); print('$v', l['value'], l['ms_per_step'], l['roofline']['frac'], l['roofline']['mean_ms'])"
done
echo done > "$O/ok"
