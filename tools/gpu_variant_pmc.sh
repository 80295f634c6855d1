#!/bin/bash
# Dynamic instruction counts per workload variant (one PMC group per rocprofv3 run).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-vpmc}
mkdir -p $OUT
export TMPDIR=/tmp
for v in joint noprior prioronly rtd_only rtd_bare; do
  i=0
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" \
             "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64"; do
    i=$((i+1))
    timeout -k 10 200 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $OUT/$v/p$i -o p$i -- python3 tools/variant_run.py $v 10 > /dev/null 2> $OUT/$v.p$i.err || { echo "$v p$i failed"; exit 1; }
  done
done
echo done
