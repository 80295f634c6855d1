#!/bin/bash
# DZ step: bitwise DEMZ tests, step timing probe (fused vs pair), section probe
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r02k}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_demc.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/dz_probe.py > $OUT/dz.json 2>&1 || exit 1
DZ_JAC=1 timeout -k 10 200 python tools/dz_probe.py > $OUT/dz_jac.json 2>&1 || exit 1
timeout -k 10 200 python tools/section_probe.py --variant dz > $OUT/sect_dz.json 2>&1 || exit 1
cat $OUT/dz.json $OUT/dz_jac.json
python -c "import json;d=json.load(open('$OUT/sect_dz.json'));print(d['kernel_us_event'],d['theta_role'],d['rtd_role'])"
