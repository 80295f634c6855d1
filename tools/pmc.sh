#!/bin/bash
# PMC passes (one counter group per rocprofv3 run; never combined with trace domains)
# over a short bench run.  Usage: bash tools/pmc.sh TAG "CTR1 CTR2 ..." ["CTR ..."] ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $OUT/p$i -o p$i -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > /dev/null 2> $OUT/p$i.err || { echo "pass $i failed rc=$?" >> $OUT/steps.log; exit 1; }
  echo "pass $i ok: $grp" >> $OUT/steps.log
done
