#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r02o}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "c4_full_size" > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-exact > $OUT/bench20.json 2> $OUT/bench20.err || exit 1
timeout -k 10 300 python bench.py --no-exact --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || exit 1
python3 -c "
import json
for f in ('$OUT/bench20.json','$OUT/bench.json'):
    d=json.load(open(f)); print(f, d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
