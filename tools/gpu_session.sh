#!/bin/bash
# One GPU session on the gpurun box, parameterised (replaces the round-2 one-off scripts).
#   bash tools/gpu_session.sh TAG [STEP ...]
# STEPs (run in order, each under its own time limit, stop at the first failure):
#   tests[=PYTEST_ARGS]  pytest -m gpu (default: all of tests/; e.g. tests=tests/test_gpu_demc.py)
#   smoke                __graft_entry__.smoke()
#   bench[=ARGS]         python bench.py ARGS            -> $OUT/bench*.json
#   bench20              the driver's command: bench.py --gpus 1 --steps 20 --warmup 5
#   stats[=ARGS]         rocprofv3 --kernel-trace --stats of bench.py ARGS -> $OUT/stats*/
#   probe=SCRIPT[:ARGS]  python tools/SCRIPT ARGS         -> $OUT/probe*.json
#   sh=COMMAND           bash -c COMMAND (a GPU command of its own, e.g. an env-var A/B) -> $OUT/sh*.log
# Outputs under gpurun_out/TAG/; steps.log records each step and its exit status.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:?usage: gpu_session.sh TAG STEP...}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
REPO=$(pwd)
n=0
log() { echo "$*" >> $OUT/steps.log; echo "$*"; }
for st in "$@"; do
  n=$((n+1))
  name=${st%%=*}; arg=""; [ "$name" != "$st" ] && arg=${st#*=}
  log "== $n $st"
  case $name in
    tests)
      timeout -k 10 1500 python -u -m pytest ${arg:-tests} -m gpu -x -v --timeout 300 --timeout-method thread \
        -p no:cacheprovider > $OUT/tests$n.log 2>&1; rc=$?
      tail -3 $OUT/tests$n.log ;;
    smoke)
      timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$? ;;
    bench)
      timeout -k 10 400 python bench.py $arg > $OUT/bench$n.json 2> $OUT/bench$n.err; rc=$?
      head -c 600 $OUT/bench$n.json; echo ;;
    bench20)
      timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench20.json 2> $OUT/bench20.err; rc=$?
      head -c 600 $OUT/bench20.json; echo ;;
    stats)
      (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $REPO/$OUT/stats$n -o stats \
        -- python3 $REPO/bench.py ${arg:---no-cpu-baseline --no-exact} > $REPO/$OUT/stats$n.json 2> $REPO/$OUT/stats$n.err); rc=$? ;;
    probe)
      scr=${arg%%:*}; pa=""; [ "$scr" != "$arg" ] && pa=${arg#*:}
      timeout -k 10 400 python tools/$scr $pa > $OUT/probe$n.json 2> $OUT/probe$n.err; rc=$?
      head -c 1500 $OUT/probe$n.json; echo ;;
    sh)
      timeout -k 10 900 bash -c "$arg" > $OUT/sh$n.log 2>&1; rc=$?
      tail -5 $OUT/sh$n.log ;;
    *) log "unknown step $name"; exit 2 ;;
  esac
  log "rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
