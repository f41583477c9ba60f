#!/bin/bash
# Bench A/B on one box: the default bench line, then the same with each env setting given
# (e.g. "EELG_OVERLAP=0"), alternating twice.  usage: bash tools/gpu_bench_ab.sh <tag> [ENV=VAL ...]
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$1; shift; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for rep in 1 2; do
  timeout -k 10 200 python3 "$R/bench.py" --no-cpu-baseline > "$O/base_$rep.json" 2> "$O/base_$rep.err"
  echo "base $rep: $(python3 -c "import json,sys; d=json.load(open('$O/base_$rep.json')); print(d['value'], d['ms_per_step'], d['roofline']['mean_ms'])")"
  i=0
  for kv in "$@"; do
    i=$((i+1))
    env $kv timeout -k 10 200 python3 "$R/bench.py" --no-cpu-baseline > "$O/v${i}_$rep.json" 2> "$O/v${i}_$rep.err"
    echo "$kv $rep: $(python3 -c "import json,sys; d=json.load(open('$O/v${i}_$rep.json')); print(d['value'], d['ms_per_step'], d['roofline']['mean_ms'])")"
  done
done
