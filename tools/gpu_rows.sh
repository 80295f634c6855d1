#!/bin/bash
# GPU session for the §8f rows (prep ensemble propagation, frac_inf_diff, DE-MC sampler,
# tau sweep): their parity tests, one FP64-FLOP PMC pass of the frac bench (its own
# rocprofv3 run, no trace domains), the benches (frac reads that PMC pass for its
# roofline), and rocprofv3 --kernel-trace --stats of the frac and prep benches.
# Outputs under gpurun_out/$TAG/.   Usage: bash tools/gpu_rows.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-rows}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
step() { echo "== $*" >> $OUT/steps.log; }
step tests
timeout -k 10 400 python -u -m pytest tests/test_gpu_prep.py tests/test_gpu_frac.py -x -v -s --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { echo "tests failed" >> $OUT/steps.log; exit 1; }
step frac-pmc
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU SQ_WAVES SQ_INSTS_VALU_TRANS_F64 --output-format csv -d $OUT/pmc1 -o pmc1 -- python3 tools/frac_bench.py --reps 2 --cpu-seconds 0.5 > $OUT/pmc_bench.json 2> $OUT/pmc1.err || { echo "pmc failed" >> $OUT/steps.log; exit 1; }
step frac-bench
timeout -k 10 300 python tools/frac_bench.py --pmc-dir $OUT/pmc1 > $OUT/frac_bench.json 2> $OUT/frac_bench.err || { echo "frac bench failed" >> $OUT/steps.log; exit 1; }
step prep-bench
timeout -k 10 300 python tools/prep_bench.py > $OUT/prep_bench.json 2> $OUT/prep_bench.err || { echo "prep bench failed" >> $OUT/steps.log; exit 1; }
step rows-stats
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o stats -- python3 tools/frac_bench.py --reps 5 --cpu-seconds 0.5 > $OUT/prof_frac.json 2> $OUT/prof.err || { echo "stats failed" >> $OUT/steps.log; exit 1; }
step prep-stats
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_prep -o stats -- python3 tools/prep_bench.py > $OUT/prof_prep.json 2> $OUT/prof_prep.err || { echo "prep stats failed" >> $OUT/steps.log; exit 1; }
step sampler-sweep
timeout -k 10 300 python tools/sampler_bench.py > $OUT/sampler_bench.json 2> $OUT/sampler.err || { echo "sampler bench failed" >> $OUT/steps.log; exit 1; }
timeout -k 10 300 python tools/sweep_bench.py > $OUT/sweep_bench.json 2> $OUT/sweep.err || { echo "sweep bench failed" >> $OUT/steps.log; exit 1; }
step sampler-stats
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_sampler -o stats -- python3 tools/sampler_bench.py > $OUT/prof_sampler.json 2> $OUT/prof_sampler.err || { echo "sampler stats failed" >> $OUT/steps.log; exit 1; }
step done
