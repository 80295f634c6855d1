#!/bin/bash
# Walker-major multi-step DEMetropolisZ: DZ bitwise tests, step probe, sampler bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-dzwm}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_demc.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/demc_tests.log 2>&1
rc=$?; tail -3 $OUT/demc_tests.log; [ $rc -eq 0 ] || exit $rc
for j in "" 1; do for d in 0 16; do
  DZ_JAC=$j NGRTD_DZ_DIAG=$d timeout -k 10 120 python tools/dz_probe.py >> $OUT/probe.jsonl 2>> $OUT/probe.err || exit 1
done; done
cat $OUT/probe.jsonl
timeout -k 10 300 python tools/sampler_bench.py --steps 400 > $OUT/sampler.json 2> $OUT/sampler.err || exit 1
cat $OUT/sampler.json
