#!/bin/bash
# Round-4: sum_rows on 256-thread blocks -- its test, then a kernel trace of the bench command
# (sum_rows' duration beside the step's large kernels) and a bench line.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/r04v; mkdir -p "$O"
cd "$R"
timeout -k 10 300 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_reduce.py > "$O/t_red.log" 2>&1
rc=$?; echo "t_red rc=$rc $(tail -1 "$O/t_red.log")"; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 bench.py --no-cpu-baseline > "$O/bench.json" 2>&1 || exit 3
python3 -c "import json; l=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print('bench', l['value'], l['ms_per_step'], l['roofline']['frac'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o run -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$O/trace.log" 2>&1 || exit 4
grep -i "sum_rows\|reduce_kernel" "$O/trace/run_kernel_stats.csv" | cut -c1-200
echo done > "$O/ok"
