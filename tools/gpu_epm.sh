#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-epm}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dropin.py tests/test_gpu_demc.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/epm_probe.py > $OUT/probe.json 2> $OUT/probe.err || exit 1
python3 -c "
import json;d=json.load(open('$OUT/probe.json'));print({k:v for k,v in d.items() if not k.endswith('_info')})"
