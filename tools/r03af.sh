#!/bin/bash
# tp_fwd with one-wave workgroups: receivers per half-wave 6 / 12 (nph6, nph12) and 48-accumulator
# path groups (acc48) vs main (8 receivers, 64 accumulators): parity of one, kbench, bench A/B
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"; mkdir -p gpurun_out/r03af
for v in nph6 nph12 acc48; do
  EELG_LIB=$R/variants/libeelg_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
      -k "interaction" > gpurun_out/r03af/t_$v.log 2>&1 || { tail -30 gpurun_out/r03af/t_$v.log; exit 3; }
  echo "$v: $(tail -1 gpurun_out/r03af/t_$v.log)"
done
bash tools/ab_kbench.sh "tp_fwd" main nph6 nph12 acc48
bash tools/gpu_bench_ab.sh r03af_ab "EELG_LIB=$R/variants/libeelg_nph6.so" "EELG_LIB=$R/variants/libeelg_nph12.so" "EELG_LIB=$R/variants/libeelg_acc48.so"
