#!/bin/bash
# Round-4: radial output-weight gradient grid (EELG_RAD_WO_WG) sweep: kbench of the radial MLP
# and the step.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/r04ag; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for wg in 1024 512 2048 4096; do
  timeout -k 10 200 env EELG_RAD_WO_WG=$wg python3 "$R/tools/kbench.py" --reps 20 --only "radial" > "$O/k_$wg.txt" 2>&1 || exit 3
  echo "== WO_WG $wg"; grep "HIP" "$O/k_$wg.txt" | cut -c1-100
done
cd "$R"
for wg in 1024 2048 4096 1024; do
  timeout -k 10 300 env EELG_RAD_WO_WG=$wg python3 bench.py --no-cpu-baseline > "$O/b_$wg.json" 2>&1 || exit 4
  python3 -c "import json; l=json.loads(open('$O/b_$wg.json').read().strip().splitlines()[-1]); print('$wg', l['value'], l['ms_per_step'], l['roofline']['frac'])"
done
echo done > "$O/ok"
