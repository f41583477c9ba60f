#!/bin/bash
# Nontemporal TP-weight loads (wnt1: tp_fwd, wnt2: tp_bwd, wnt3: both): parity, kbench, bench A/B;
# the round's isolated kbench of every kernel; an in-line (EELG_OVERLAP=0) kernel trace of the step
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"; mkdir -p gpurun_out/r03ab
EELG_LIB=$R/variants/libeelg_wnt3.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
    -k "interaction or model_forward_backward_matches_oracle and 4" > gpurun_out/r03ab/t_wnt3.log 2>&1 || { tail -30 gpurun_out/r03ab/t_wnt3.log; exit 3; }
echo "wnt3: $(tail -1 gpurun_out/r03ab/t_wnt3.log)"
bash tools/ab_kbench.sh "tp_" main wnt1 wnt2 wnt3
bash tools/gpu_bench_ab.sh r03ab_ab "EELG_LIB=$R/variants/libeelg_wnt1.so" "EELG_LIB=$R/variants/libeelg_wnt2.so" "EELG_LIB=$R/variants/libeelg_wnt3.so"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 "$R/tools/kbench.py" --reps 20 > "$R/gpurun_out/r03ab/kbench.txt" 2>&1
EELG_OVERLAP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/r03ab/inline" -o run \
    -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$R/gpurun_out/r03ab/inline.log" 2>&1
echo done
