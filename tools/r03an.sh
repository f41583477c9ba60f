#!/bin/bash
# bench lines of BASELINE configs 5 and 4 on the closing build
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p "$R/gpurun_out/r03an"; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 "$R/bench.py" --config 5 --no-cpu-baseline > "$R/gpurun_out/r03an/config5.json" 2> "$R/gpurun_out/r03an/config5.err"
for m in cgc_modified cgc_vanilla; do
  timeout -k 10 300 python3 "$R/bench.py" --model $m --batch 256 --no-cpu-baseline > "$R/gpurun_out/r03an/$m.json" 2> "$R/gpurun_out/r03an/$m.err"
done
for f in config5 cgc_modified cgc_vanilla; do python3 -c "import json; d=json.load(open('$R/gpurun_out/r03an/$f.json')); print('$f', d['value'], d['ms_per_step'], (d['roofline'] or {}).get('frac'))"; done
