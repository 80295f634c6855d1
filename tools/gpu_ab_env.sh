#!/bin/bash
# A/B of a plan-time switch: parity tests, then 3 alternating bench runs with and without
# the environment variable $1 set (kernel time per launch).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
V=$1
mkdir -p gpurun_out/ab
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ab/tests.log 2>&1 || { tail -20 gpurun_out/ab/tests.log; exit 1; }
tail -1 gpurun_out/ab/tests.log
for i in 1 2 3; do
  timeout -k 10 120 python bench.py --steps 400 --warmup 40 --no-cpu-baseline > gpurun_out/ab/a$i.json 2>/dev/null || exit 1
  timeout -k 10 120 env $V=1 python bench.py --steps 400 --warmup 40 --no-cpu-baseline > gpurun_out/ab/b$i.json 2>/dev/null || exit 1
  python -c "import json;a=json.load(open('gpurun_out/ab/a$i.json'));b=json.load(open('gpurun_out/ab/b$i.json'));print('default',a['value'],a['roofline']['kernel_ms'],' $V',b['value'],b['roofline']['kernel_ms'])"
done
