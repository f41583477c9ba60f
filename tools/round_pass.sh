#!/bin/bash
# One GPU-box pass of named steps, each under its own time limit, writing under gpurun_out/<tag>/.
# Replaces the per-run scripts of round 4 (tools/r04*.sh).  rc 0 / 1 of a step (pass / test
# failures) lets the pass continue; anything else (fault, abort, time limit) ends it.
#
# usage (GPU box): bash tools/round_pass.sh <tag> <step> [<step> ...]
#   tests                 the whole `pytest -m gpu` suite (EELG_PARITY_OUT -> parity.json)
#   pytest:<files>[:<k>]  pytest -m gpu over <files> ('+' between files), -k <k> ('+' for spaces)
#   smoke                 __graft_entry__.smoke()
#   bench[:<args>]        bench.py line (args with '+' for spaces, e.g. bench:--config+5)
#   prof:<name>[:<args>]  tools/profile_round.sh for a workload (bench args as above)
#   inline                EELG_OVERLAP=0 rocprofv3 kernel trace of the default bench command
#   kbench[:<regex>]      tools/kbench.py --reps 20 [--only regex]
#   pmc:<regex>           tools/pmc_passes.sh counter groups over kbench's kernels matching regex
#   var:<name>:<regex>    kbench of variants/libeelg_<name>.so (tools/build_variant.sh)
#   cmd:<log>:<command>   any command ('+' for spaces), e.g. cmd:pk.txt:tools/proto/pkfma_bench
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; shift
O=$R/gpurun_out/$TAG; mkdir -p "$O"
export TMPDIR=/tmp
cd "$R"
PYT="python -u -m pytest -q --timeout 400 --timeout-method thread"
step() {   # step <log> <timeout> <cmd...>
  local log=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?
  echo "[$log] rc=$rc $(tail -1 "$O/$log" | cut -c1-200)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; tail -20 "$O/$log"; exit $rc; fi
}
sp() { echo "${1//+/ }"; }
for s in "$@"; do
  case "$s" in
    tests)     step tests.log 900 env EELG_PARITY_OUT="$O/parity.json" $PYT tests -m gpu
               grep -E "FAILED|passed|failed" "$O/tests.log" | tail -5 ;;
    pytest:*)  r=${s#pytest:}; f=$(sp "${r%%:*}"); k=""; [ "$r" != "${r%%:*}" ] && k=$(sp "${r#*:}")
               n=$(echo "$r" | tr -c 'a-zA-Z0-9_' '_' | cut -c1-40)
               if [ -n "$k" ]; then step "t_$n.log" 600 env EELG_PARITY_OUT="$O/parity_$n.json" $PYT -m gpu $f -k "$k"
               else step "t_$n.log" 600 env EELG_PARITY_OUT="$O/parity_$n.json" $PYT -m gpu $f; fi ;;
    smoke)     step smoke.log 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)     step bench.json 400 python3 bench.py ;;
    bench:*)   a=$(sp "${s#bench:}"); n=$(echo "${s#bench:}" | tr -c 'a-zA-Z0-9_' '_' | cut -c1-40)
               step "bench_$n.json" 400 python3 bench.py $a ;;
    prof:*)    r=${s#prof:}; n=${r%%:*}; a=""; [ "$r" != "$n" ] && a=$(sp "${r#*:}")
               step "prof_$n.log" 900 env BENCH_ARGS="$a" bash tools/profile_round.sh "gpurun_out/$TAG/$n" ;;
    inline)    step inline.log 300 env EELG_OVERLAP=0 rocprofv3 --kernel-trace --stats --output-format csv \
                   -d "$O/inline" -o run -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline ;;
    kbench)    step kbench.txt 300 python3 "$R/tools/kbench.py" --reps 20 ;;
    kbench:*)  step "kbench_$(echo "${s#kbench:}" | tr -c 'a-zA-Z0-9_' '_' | cut -c1-30).txt" 300 \
                   python3 "$R/tools/kbench.py" --reps 20 --only "${s#kbench:}" ;;
    pmc:*)     step pmc.log 900 bash tools/pmc_passes.sh "$TAG" "${s#pmc:}" ;;
    var:*)     r=${s#var:}; n=${r%%:*}; x=${r#*:}
               step "k_$n.txt" 300 env EELG_LIB="$R/variants/libeelg_$n.so" python3 "$R/tools/kbench.py" --reps 20 --only "$x" ;;
    cmd:*)     r=${s#cmd:}; n=${r%%:*}; c=$(sp "${r#*:}")
               step "$n" 300 $c ;;
    *)         echo "unknown step $s"; exit 2 ;;
  esac
done
echo done > "$O/ok"
