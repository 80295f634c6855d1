#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r02n}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_demc.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for d in ${DIAGS:-0 1 8}; do
  NGRTD_DZ_DIAG=$d timeout -k 10 120 python tools/dz_probe.py >> $OUT/nat.json 2>/dev/null || exit 1
  DZ_JAC=1 NGRTD_DZ_DIAG=$d timeout -k 10 120 python tools/dz_probe.py >> $OUT/jac.json 2>/dev/null || exit 1
done
cat $OUT/nat.json $OUT/jac.json
