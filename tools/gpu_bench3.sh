#!/bin/bash
# three short bench runs (kernel time per launch) -- quick A/B of a kernel change
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/b3
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/b3/tests.log 2>&1 || { tail -20 gpurun_out/b3/tests.log; exit 1; }
tail -1 gpurun_out/b3/tests.log
for i in 1 2 3; do timeout -k 10 120 python bench.py --steps 400 --warmup 40 --no-cpu-baseline > gpurun_out/b3/b$i.json 2>/dev/null || exit 1; python -c "import json;d=json.load(open('gpurun_out/b3/b$i.json'));print(d['value'],d['roofline']['kernel_ms'])"; done
