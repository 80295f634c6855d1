#!/bin/bash
# PMC passes per model (tools/model_pmc.py: one plan per process, so each kernel instance's
# counters belong to that model only), each counter group in its own rocprofv3 run (never
# combined with a trace domain).  Usage (on the GPU box):
#   bash tools/gpu_model_pmc.sh TAG "model:sv@N[^tau2hi]" ...
# then:  python tools/model_pmc_summary.py gpurun_out/TAG profiles/rNN_model_pmc.json
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
for spec in "$@"; do
  m=${spec%%@*}; rest=${spec#*@}; n=${rest%%^*}; t2=""; [ "$rest" != "$n" ] && t2="--tau2-hi ${rest#*^}"
  key=$(echo "$spec" | tr ':@^' '__-')
  mkdir -p $OUT/$key
  i=0
  for grp in "FETCH_SIZE" "WRITE_SIZE" \
             "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FLOPS_FP64_TRANS SQ_INSTS_LDS" \
             "SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_WAVE_CYCLES"; do
    i=$((i+1))
    d=$OUT/$key/p$i
    timeout -k 10 240 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $d -o p$i -- \
      python3 tools/model_pmc.py --model $m --ages $n $t2 > $OUT/$key/run$i.json 2> $OUT/$key/p$i.err \
      || { echo "$spec pass $i failed rc=$?" >> $OUT/steps.log; exit 1; }
  done
  echo "$spec ok" >> $OUT/steps.log
done
