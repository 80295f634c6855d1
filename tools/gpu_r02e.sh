#!/bin/bash
# Jacobian-plan parity at c4 shape, sampler tests, then the sampler bench + its profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r02e
timeout -k 10 600 python -u -m pytest tests/test_gpu_demc.py tests/test_gpu_dropin.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r02e/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r02e/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/sampler_bench.py --steps 200 > gpurun_out/r02e/sampler.json 2> gpurun_out/r02e/sampler.err || exit 1
cat gpurun_out/r02e/sampler.json
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r02e/prof -o sampler -- python3 $GRAFT_REPO_ROOT/tools/sampler_bench.py --steps 100 > $GRAFT_REPO_ROOT/gpurun_out/r02e/prof.log 2>&1 || exit 1
find $GRAFT_REPO_ROOT/gpurun_out/r02e/prof -name "*kernel_stats.csv"
