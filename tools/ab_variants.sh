#!/bin/bash
# A/B of kernel variants built by tools/build_variant.sh (variants/libeelg_<tag>.so, loaded via
# EELG_LIB; "main" = the in-tree library): TP parity tests, then tools/kbench.py timings.
# usage (GPU box): bash tools/ab_variants.sh main <tag> [<tag> ...]
set -e
mkdir -p gpurun_out/var
for v in "$@"; do
  if [ "$v" = main ]; then L=""; else L=$PWD/variants/libeelg_$v.so; fi
  EELG_LIB=$L timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bf16.py -x -q --timeout 120 --timeout-method thread -k "interaction or model or tp" > gpurun_out/var/t_$v.log 2>&1 || { echo "$v TESTS FAILED"; tail -20 gpurun_out/var/t_$v.log; exit 1; }
  EELG_LIB=$L timeout -k 10 200 python tools/kbench.py --reps 20 --only "tp_fwd" > gpurun_out/var/k_$v.txt 2>&1
  echo "== $v $(tail -1 gpurun_out/var/t_$v.log)"; grep " ms" gpurun_out/var/k_$v.txt | cut -c1-70
done
