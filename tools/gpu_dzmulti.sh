#!/bin/bash
# Multi-step DEMetropolisZ launch: the DZ bitwise tests first, then the sampler bench and its
# rocprofv3 kernel stats (one launch = up to 256 steps), then the rest of the GPU tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-dzmulti}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_demc.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/demc_tests.log 2>&1
rc=$?; tail -3 $OUT/demc_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/sampler_bench.py --steps 400 > $OUT/sampler.json 2> $OUT/sampler.err || exit 1
cat $OUT/sampler.json
NGRTD_DZ_CHUNK=1 timeout -k 10 300 python tools/sampler_bench.py --steps 200 > $OUT/sampler_chunk1.json 2> $OUT/sampler_chunk1.err || exit 1
cat $OUT/sampler_chunk1.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/sprof -o sampler -- python3 $GRAFT_REPO_ROOT/tools/sampler_bench.py --steps 200 > $GRAFT_REPO_ROOT/$OUT/sprof.json 2> $GRAFT_REPO_ROOT/$OUT/sprof.err || exit 1
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider --deselect tests/test_gpu_demc.py > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; exit $rc
