#!/bin/bash
# DZ proposal rows through LDS: bitwise DZ tests, then the step probe with and without
# (NGRTD_DZ_PROP_GLOBAL=1), natural and transformed, and the sampler bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-dzlds}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_demc.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/demc_tests.log 2>&1
rc=$?; tail -3 $OUT/demc_tests.log; [ $rc -eq 0 ] || exit $rc
for j in "" 1; do
  DZ_JAC=$j timeout -k 10 120 python tools/dz_probe.py >> $OUT/probe.jsonl 2>> $OUT/probe.err || exit 1
  NGRTD_DZ_PROP_GLOBAL=1 DZ_JAC=$j timeout -k 10 120 python tools/dz_probe.py >> $OUT/probe.jsonl 2>> $OUT/probe.err || exit 1
done
cat $OUT/probe.jsonl
timeout -k 10 300 python tools/sampler_bench.py --steps 400 > $OUT/sampler.json 2> $OUT/sampler.err || exit 1
cat $OUT/sampler.json
