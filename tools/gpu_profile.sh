#!/bin/bash
# One GPU session: parity tests, PMC passes over a short bench (each counter group in its
# own rocprofv3 run, never combined with a trace domain), their summary, then the bench
# (reading that summary for the FP64 FLOPs and HBM traffic of its kernel) and rocprofv3
# --kernel-trace --stats of the same bench command.  Outputs under gpurun_out/$TAG/;
# copy with:  python tools/profile_summary.py gpurun_out/$TAG profiles/rNN
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-run}
# BENCH_ARGS: extra bench.py flags (e.g. "--mod-type1 exp_pist_flow"); SKIP_TESTS=1 skips pytest
BA=${BENCH_ARGS:-}
# PMC_ARGS: extra flags of the PMC passes only (default: no side legs -- the headline kernel's
# counters; every counter pass serialises each dispatch, and the side legs' sampling runs
# dispatch hundreds of thousands of kernels)
PA=${PMC_ARGS:---no-models --no-reference-runs --no-sampler}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
step() { echo "== $*" >> $OUT/steps.log; }
if [ -z "$SKIP_TESTS" ]; then
step tests
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > $OUT/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/steps.log; [ $rc -eq 0 ] || exit $rc
fi
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" \
           "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64" \
           "SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FLOPS_FP64_TRANS SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64" \
           "SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY" \
           "SQ_INSTS_MFMA SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_CVT" \
           "GRBM_GUI_ACTIVE SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT"; do
  i=$((i+1))
  step "pmc$i $grp"
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $OUT/pmc$i -o pmc$i -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-exact $PA $BA > $OUT/pmc_bench.json 2> $OUT/pmc$i.err || { echo "pmc$i failed rc=$?" >> $OUT/steps.log; exit 1; }
done
step summary
python tools/profile_summary.py $OUT $OUT/summ > /dev/null || { echo "summary failed" >> $OUT/steps.log; exit 1; }
step bench
NGRTD_PMC_SUMMARY=$OUT/summ_pmc.json timeout -k 10 300 python bench.py --steps 400 --warmup 40 --cpu-seconds 15 $BA > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed rc=$?" >> $OUT/steps.log; exit 1; }
step rocprof-stats
NGRTD_PMC_SUMMARY=$OUT/summ_pmc.json timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o stats -- python3 bench.py --steps 400 --warmup 40 --no-cpu-baseline --no-exact $BA > $OUT/prof_bench.json 2> $OUT/prof.err || { echo "rocprof failed rc=$?" >> $OUT/steps.log; exit 1; }
step done
