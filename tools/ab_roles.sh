set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_demc.py tests/test_gpu_dropin.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ab/tests.log 2>&1 || { tail -30 gpurun_out/ab/tests.log; exit 1; }
tail -2 gpurun_out/ab/tests.log
for r in 1 2 1 2; do NGRTD_FUSED_ROLES=$r timeout -k 10 120 python bench.py --steps 400 --warmup 40 --no-cpu-baseline > gpurun_out/ab/b$r.json 2>/dev/null || exit 1; python -c "import json;d=json.load(open('gpurun_out/ab/b$r.json'));print('roles',$r,d['value'],d['roofline']['kernel_ms'])"; done
