#!/bin/bash
# Single-launch DEMetropolisZ step: bitwise DEMZ tests, then the sampler bench (fused and,
# for the A/B, the proposal + log-prob pair via NGRTD_DZ_MODE=pair).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r02g}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_demc.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/sampler_bench.py --steps 200 > $OUT/sampler.json 2> $OUT/sampler.err || exit 1
cat $OUT/sampler.json
NGRTD_DZ_MODE=pair timeout -k 10 300 python tools/sampler_bench.py --steps 200 > $OUT/sampler_pair.json 2> $OUT/sampler_pair.err || exit 1
cat $OUT/sampler_pair.json
