#!/bin/bash
# Round-4: grad-W grid size (node slices x weight tiles): LINW_WG / LINW_MAX_SLICES sweep,
# kbench of the linears and the step.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/r04ac; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for v in 1024:64 2048:64 4096:128 8192:256; do
  wg=${v%:*}; ms=${v#*:}
  timeout -k 10 200 env EELG_LINW_WG=$wg EELG_LINW_MAX_SLICES=$ms python3 "$R/tools/kbench.py" --reps 20 --only "lin" > "$O/k_$wg.txt" 2>&1 || exit 3
  echo "== WG $wg MAXS $ms"; grep "bwd_w" "$O/k_$wg.txt" | cut -c1-100
done
cd "$R"
for v in 1024:64 4096:128 8192:256 1024:64; do
  wg=${v%:*}; ms=${v#*:}
  timeout -k 10 300 env EELG_LINW_WG=$wg EELG_LINW_MAX_SLICES=$ms python3 bench.py --no-cpu-baseline > "$O/b_$wg.json" 2>&1 || exit 4
  python3 -c "import json; l=json.loads(open('$O/b_$wg.json').read().strip().splitlines()[-1]); print('$wg', l['value'], l['ms_per_step'], l['roofline']['frac'])"
done
echo done > "$O/ok"
