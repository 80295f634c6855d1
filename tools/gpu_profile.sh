#!/bin/bash
# One GPU session: parity tests, bench, rocprofv3 kernel stats, PMC passes (FETCH_SIZE,
# WRITE_SIZE) for the HBM traffic of the RTD kernel.  Outputs under gpurun_out/$TAG/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
step() { echo "== $*" >> $OUT/steps.log; }
step tests
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > $OUT/tests.log 2>&1
echo "pytest rc=$?" >> $OUT/steps.log
step bench
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --cpu-seconds 10 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed rc=$?" >> $OUT/steps.log; exit 1; }
step rocprof-stats
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o stats -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline > $OUT/prof_bench.json 2> $OUT/prof.err || { echo "rocprof failed rc=$?" >> $OUT/steps.log; exit 1; }
step pmc-fetch
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o fetch -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > /dev/null 2> $OUT/pmc_fetch.err || { echo "pmc fetch failed rc=$?" >> $OUT/steps.log; exit 1; }
step pmc-write
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o write -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > /dev/null 2> $OUT/pmc_write.err || { echo "pmc write failed rc=$?" >> $OUT/steps.log; exit 1; }
step done
