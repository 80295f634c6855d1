#!/bin/bash
# Round-2 re-check at HEAD (multi-step DEMetropolisZ): all GPU tests, smoke(), the headline bench
# (default and driver-shaped), its rocprofv3 kernel stats, the sampler bench and its kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r02final2}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench20.json 2> $OUT/bench20.err || exit 1
timeout -k 10 300 python tools/sampler_bench.py --steps 400 > $OUT/sampler.json 2> $OUT/sampler.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof -o bench -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-exact > $GRAFT_REPO_ROOT/$OUT/prof_bench.json 2> $GRAFT_REPO_ROOT/$OUT/prof_bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/sprof -o sampler -- python3 $GRAFT_REPO_ROOT/tools/sampler_bench.py --steps 200 > $GRAFT_REPO_ROOT/$OUT/sprof.json 2> $GRAFT_REPO_ROOT/$OUT/sprof.err || exit 1
cd $GRAFT_REPO_ROOT
cat $OUT/smoke.log; cat $OUT/bench.json; cat $OUT/bench20.json; cat $OUT/sampler.json
bash tools/gpu_dzpmc.sh ${1:-r02final2}_pmc > /dev/null || exit 1
