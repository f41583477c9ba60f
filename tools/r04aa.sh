#!/bin/bash
# Round-4: collate-time Morton node order (config 5 and config 2 step A/B; the loss must agree).
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/r04aa; mkdir -p "$O"
cd "$R"
b() { local tag=$1; shift; timeout -k 10 300 python3 bench.py --no-cpu-baseline "$@" > "$O/$tag.json" 2>&1 || exit 3
  python3 -c "import json; l=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print('$tag', l['value'], l['ms_per_step'], l['roofline']['frac'], l['roofline']['mean_ms'], l['loss'], l.get('peak_hbm_gb'))"; }
b c5_morton --config 5 --node-order morton
sleep 30; rocm-smi --showmeminfo vram > "$O/smi1.txt" 2>&1 || true
b c5_none --config 5 --node-order none
sleep 30; rocm-smi --showmeminfo vram > "$O/smi2.txt" 2>&1 || true
sleep 30
b c5_morton2 --config 5 --node-order morton
b c5_none2 --config 5 --node-order none
echo done > "$O/ok"
