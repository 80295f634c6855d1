set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/t2.log 2>&1; echo "pytest rc=$?" >> gpurun_out/t2.log
timeout -k 10 300 python bench.py --steps 50 --warmup 10 --cpu-seconds 5 > gpurun_out/b2.json 2> gpurun_out/b2.err
echo "bench rc=$?" >> gpurun_out/t2.log
