# GPU check: parity tests then a short bench.  Usage: bash tools/gpu_check.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-chk}
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/$TAG.test.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/$TAG.test.log
tail -5 gpurun_out/$TAG.test.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --cpu-seconds 5 > gpurun_out/$TAG.bench.json 2> gpurun_out/$TAG.bench.err
rc=$?
echo "bench rc=$rc"
cat gpurun_out/$TAG.bench.json
exit $rc
