#!/bin/bash
# One GPU session: parity tests, bench, rocprofv3 kernel stats of the bench command, PMC
# passes (FETCH_SIZE, WRITE_SIZE, SQ busy/MFMA counters -- each in its own pass, never with
# a trace domain).  Outputs under gpurun_out/$TAG/; tools/profile_summary.py condenses them.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
step() { echo "== $*" >> $OUT/steps.log; }
step tests
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > $OUT/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/steps.log; [ $rc -eq 0 ] || exit $rc
step bench
timeout -k 10 300 python bench.py --steps 400 --warmup 40 --cpu-seconds 15 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed rc=$?" >> $OUT/steps.log; exit 1; }
step rocprof-stats
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o stats -- python3 bench.py --steps 400 --warmup 40 --no-cpu-baseline > $OUT/prof_bench.json 2> $OUT/prof.err || { echo "rocprof failed rc=$?" >> $OUT/steps.log; exit 1; }
step pmc-fetch
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o fetch -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > /dev/null 2> $OUT/pmc_fetch.err || { echo "pmc fetch failed rc=$?" >> $OUT/steps.log; exit 1; }
step pmc-write
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o write -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > /dev/null 2> $OUT/pmc_write.err || { echo "pmc write failed rc=$?" >> $OUT/steps.log; exit 1; }
step pmc-sq
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc_sq -o sq -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > /dev/null 2> $OUT/pmc_sq.err || { echo "pmc sq failed rc=$?" >> $OUT/steps.log; exit 1; }
step done
