#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r02r}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_demc.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for m in fused pair; do
  NGRTD_DZ_MODE=$m timeout -k 10 300 python tools/sampler_bench.py --steps 200 > $OUT/sampler_$m.json 2> $OUT/sampler_$m.err || exit 1
  python3 -c "import json;d=json.load(open('$OUT/sampler_$m.json'));print('$m', d['device_demcz_natural']['us_per_step'], d['device_demcz_transformed']['us_per_step'])"
done
