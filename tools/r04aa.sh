#!/bin/bash
# Round-4: collate-time Morton node order (config 5 and config 2 step A/B; the loss must agree).
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/r04aa; mkdir -p "$O"
cd "$R"
b() { local tag=$1; shift; timeout -k 10 300 python3 bench.py --no-cpu-baseline "$@" > "$O/$tag.json" 2>&1 || exit 3
  python3 -c "import json; l=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print('$tag', l['value'], l['ms_per_step'], l['roofline']['frac'], l['roofline']['mean_ms'], l['loss'])"; }
b c5_none --config 5 --node-order none
b c5_morton --config 5 --node-order morton
b c5_none2 --config 5 --node-order none
b c5_morton2 --config 5 --node-order morton
b c2_none --node-order none
b c2_morton --node-order morton
echo done > "$O/ok"
