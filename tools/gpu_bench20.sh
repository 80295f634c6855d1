#!/bin/bash
# The driver-shaped headline bench (20 steps, 5 warm-up) five times, and the default bench once.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-bench20}
mkdir -p $OUT
for i in 1 2 3 4 5; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-exact >> $OUT/bench20.jsonl 2>> $OUT/bench20.err || exit 1
done
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
python3 -c "
import json
for l in open('$OUT/bench20.jsonl'):
    d=json.loads(l); print(round(d['value']/1e6,1), round(d['ms_per_step']*1e3,2), round(d['roofline']['kernel_ms']*1e3,2))
d=json.load(open('$OUT/bench.json')); print('default', round(d['value']/1e6,1), round(d['ms_per_step']*1e3,2))
"
