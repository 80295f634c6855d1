#!/bin/bash
# Round-2 sampler check: DEMetropolisZ GPU tests, the sampler bench and its kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r02c
timeout -k 10 600 python -u -m pytest tests/test_gpu_demc.py tests/test_gpu_dropin.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r02c/tests.log 2>&1
rc=$?; tail -25 gpurun_out/r02c/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/sampler_bench.py --steps 200 > gpurun_out/r02c/sampler.json 2> gpurun_out/r02c/sampler.err || exit 1
cat gpurun_out/r02c/sampler.json
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r02c/prof -o sampler -- python3 $GRAFT_REPO_ROOT/tools/sampler_bench.py --steps 100 > $GRAFT_REPO_ROOT/gpurun_out/r02c/prof.log 2>&1 || exit 1
find $GRAFT_REPO_ROOT/gpurun_out/r02c/prof -name "*kernel_stats.csv" | head -3
