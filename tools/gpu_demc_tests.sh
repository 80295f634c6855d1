#!/bin/bash
# The device DEMetropolisZ GPU tests alone.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-demc_tests}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_demc.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/demc_tests.log 2>&1
rc=$?; tail -4 $OUT/demc_tests.log; exit $rc
