#!/bin/bash
# Headline-roofline reproducibility probe: the tp_fwd launch time by HIP
# events (untraced) and by rocprofv3 kernel trace, for the overlapped step and for the in-line
# step (EELG_OVERLAP=0) with the layer's radial MLP issued before (EELG_RADIAL_FIRST=1) or
# after (=0) linear_up.  Each GPU step has its own time limit; the first failure ends the script.
# usage (GPU box): bash tools/frac_probe.sh <tag> [modes...]   modes: ovl inl_rf inl_old (default all)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$1; shift; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
run() { local log=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?
        echo "[$log] rc=$rc $(tail -1 "$O/$log" | cut -c1-160)"; [ $rc -eq 0 ] || exit $rc; }
B="$R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --kernel-summary"
modes=${*:-ovl inl_rf inl_old}
for m in $modes; do
  case $m in
    ovl)     E="EELG_OVERLAP=1" ;;
    inl_rf)  E="EELG_OVERLAP=0 EELG_RADIAL_FIRST=1" ;;
    inl_old) E="EELG_OVERLAP=0 EELG_RADIAL_FIRST=0" ;;
  esac
  run "b_$m.json" 240 env $E python3 $B
  run "t_$m.log" 300 env $E rocprofv3 --kernel-trace --stats --output-format csv -d "$O/t_$m" -o run -- python3 $B
done
echo done > "$O/ok"
