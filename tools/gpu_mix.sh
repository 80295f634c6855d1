#!/bin/bash
# Instruction mix of the headline kernel (two PMC passes, each its own rocprofv3 run,
# kernel-trace only) for the product library and each variant library given (NGRTD_LIB).
#   bash tools/gpu_mix.sh [variant.so ...]   -> gpurun_out/mix/<name>_pmc{1,2}/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/mix
run() {  # name lib
  local n=$1 lib=$2 i=0
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES" \
             "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT"; do
    i=$((i+1))
    NGRTD_LIB=$lib timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d gpurun_out/mix/${n}_pmc$i -o p -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > /dev/null 2> gpurun_out/mix/${n}_pmc$i.err || { echo "$n pass $i failed"; return 1; }
  done
}
run default "" || exit 1
for v in "$@"; do run $(basename $v .so) $PWD/$v || exit 1; done
python3 tools/mix_summary.py gpurun_out/mix
