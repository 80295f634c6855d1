#!/bin/bash
# PMC instruction counts of the single-launch DEMetropolisZ step, natural and transformed
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-dzpmc}
mkdir -p $OUT
export TMPDIR=/tmp
G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH"
G2="SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU_FLOPS_FP64 SQ_ACTIVE_INST_VALU SQ_INSTS_FLAT"
G3="FETCH_SIZE"
G4="WRITE_SIZE"
for jac in 0 1; do
  i=0
  for grp in "$G1" "$G2" "$G3" "$G4"; do
    i=$((i+1))
    if [ $jac = 1 ]; then export DZ_JAC=1; else unset DZ_JAC; fi
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $OUT/j${jac}p$i -o p -- python3 tools/dz_probe.py > /dev/null 2> $OUT/j${jac}p$i.err || { echo "pass $jac $i failed"; exit 1; }
  done
  python3 tools/pmc_summary.py $OUT/j${jac}p1 $OUT/j${jac}p2 $OUT/j${jac}p3 $OUT/j${jac}p4 > $OUT/summ_j$jac.txt
done
cat $OUT/summ_j0.txt $OUT/summ_j1.txt
