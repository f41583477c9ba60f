#!/bin/bash
# Round-4 pass 6: the contraction with its coefficients scalar-loaded as SGPR vectors (no
# per-term s_mov): parity, kbench against the packed builds, and bench lines for both forms.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/r04f; mkdir -p "$O"
cd "$R"
step() {   # step <log> <timeout> <cmd...>: rc 0 / 1 continue, anything else ends the script
  local log=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?
  echo "[$log] rc=$rc $(tail -1 "$O/$log")"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; tail -20 "$O/$log"; exit $rc; fi
}
PYT="python -u -m pytest -q --timeout 300 --timeout-method thread"
step t_sc.log 600 $PYT tests/test_gpu_parity.py tests/test_gpu_api.py -k "symcon or symmetric or contraction or product or model_forward_backward"
for v in cv1w3; do
  step t_$v.log 600 env EELG_LIB=$R/variants/libeelg_$v.so $PYT tests/test_gpu_parity.py -k "symcon"
done
cd /tmp && export TMPDIR=/tmp
for v in main cv1 cv1w3; do
  if [ $v = main ]; then L=""; else L="EELG_LIB=$R/variants/libeelg_$v.so"; fi
  step k_$v.txt 200 env $L python3 "$R/tools/kbench.py" --reps 20 --only "sc_"
  grep " ms" "$O/k_$v.txt" | cut -c1-100
done
cd "$R"
step bench_main.json 300 python3 bench.py --no-cpu-baseline
tail -1 "$O/bench_main.json" | cut -c1-200
step bench_cv1w3.json 300 env EELG_LIB=$R/variants/libeelg_cv1w3.so python3 bench.py --no-cpu-baseline
tail -1 "$O/bench_cv1w3.json" | cut -c1-200
echo done > "$O/ok"
