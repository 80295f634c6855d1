#!/bin/bash
# Quick GPU iteration: headline parity tests, 3 bench runs, section probe.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/q
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_demc.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/q/tests.log 2>&1 || { tail -30 gpurun_out/q/tests.log; exit 1; }
tail -1 gpurun_out/q/tests.log
for i in 1 2 3; do timeout -k 10 120 python bench.py --steps 400 --warmup 40 --no-cpu-baseline > gpurun_out/q/b$i.json 2>/dev/null || exit 1; python -c "import json;d=json.load(open('gpurun_out/q/b$i.json'));print(d['value'],d['roofline']['kernel_ms'])"; done
timeout -k 10 120 python tools/section_probe.py > gpurun_out/q/probe.json 2>/dev/null && python -c "import json;d=json.load(open('gpurun_out/q/probe.json'));print(d['theta_role'],d['rtd_role'])"
