#!/bin/bash
# Iteration session: GPU tests, section probe, kernel-variant timing, short bench.
# Usage: bash tools/gpu_iter.sh TAG [extra]   (extra = "avail" also lists the PMC counters)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-iter}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
timeout -k 10 300 python tools/section_probe.py > $OUT/section.json 2> $OUT/section.err || { echo "probe failed"; exit 1; }
cat $OUT/section.json
for v in rtd_only rtd_bare; do
  timeout -k 10 300 python tools/section_probe.py --variant $v > $OUT/section_$v.json 2>> $OUT/section.err || { echo "probe $v failed"; exit 1; }
done
timeout -k 10 300 python tools/kernel_timing.py --steps 50 > $OUT/variants.log 2>&1 || { echo "variants failed"; exit 1; }
cat $OUT/variants.log
timeout -k 10 300 python bench.py --steps 400 --warmup 40 --cpu-seconds 5 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; exit 1; }
cat $OUT/bench.json
if [ "$2" = "avail" ]; then
  timeout -k 10 120 rocprofv3 --list-avail > $OUT/avail.txt 2>&1 || echo "list-avail rc=$?"
fi
exit 0
