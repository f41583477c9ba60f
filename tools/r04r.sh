#!/bin/bash
# Round-4: nontemporal stores for the TP backward's grad_w / gxe and the radial forward's w
# (parity, kbench, step A/B against the default build with nontemporal linear outputs).
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/r04r; mkdir -p "$O"
cd "$R"
run() { local log=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; [ $rc -le 1 ] || { echo "[$log] rc=$rc"; tail -20 "$O/$log"; exit $rc; }; echo "[$log] rc=$rc $(tail -1 "$O/$log" | cut -c1-120)"; }
PYT="python -u -m pytest -q --timeout 300 --timeout-method thread"
run t_tpnt.log 400 env EELG_LIB=$R/variants/libeelg_tpnt.so $PYT tests/test_gpu_parity.py -k "interaction or model_forward_backward"
run t_rnt.log 300 env EELG_LIB=$R/variants/libeelg_rnt.so $PYT tests/test_gpu_radial.py
cd /tmp && export TMPDIR=/tmp
for v in main tpnt rnt; do
  if [ $v = main ]; then L=""; else L="EELG_LIB=$R/variants/libeelg_$v.so"; fi
  run k_$v.txt 200 env $L python3 "$R/tools/kbench.py" --reps 20 --only "tp_bwd|radial.*HIP|segment_sum gxe"
  grep " ms" "$O/k_$v.txt" | cut -c1-100
done
cd "$R"
for v in main tpnt rnt main tpnt rnt; do
  if [ $v = main ]; then L=""; else L="EELG_LIB=$R/variants/libeelg_$v.so"; fi
  timeout -k 10 300 env $L python3 bench.py --no-cpu-baseline > "$O/b.json" 2>&1 || exit 3
  python3 -c "import json; l=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print('$v', l['value'], l['ms_per_step'])"
done
echo done > "$O/ok"
