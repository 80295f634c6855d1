#!/bin/bash
# A/B of the dispersion exponential table (library variants named on the command line against
# the product library): c4 log-prob launches at N = 1200 and N = 25 256 (tools/model_probe.py),
# the reference-shape dispersion step (tools/disp_step_probe.py), 2 interleaved rounds; then the
# LDS counters of the product library's N = 25 256 launch (one rocprofv3 --pmc pass).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/abdt
mkdir -p $OUT
for i in 1 2; do
  for v in noblegas_rtd_mcmc_amd/libngrtd.so "$@"; do
    n=$(basename $v .so)
    a=$(NGRTD_LIB=$PWD/$v timeout -k 10 120 python tools/model_probe.py --models dispersion:0,dispersion:123,dispersion-piston:0 --rounds 1) || exit 1
    b=$(NGRTD_LIB=$PWD/$v timeout -k 10 180 python tools/model_probe.py --models dispersion:123 --ages 25256 --steps 10 --rounds 1) || exit 1
    c=$(NGRTD_LIB=$PWD/$v timeout -k 10 120 python tools/disp_step_probe.py) || exit 1
    echo "round $i $n N1200 $a N25256 $b step $c" >> $OUT/ab.txt
  done
done
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_WAVES --output-format csv -d $OUT/pmc -o p -- python3 tools/model_probe.py --models dispersion:123 --ages 25256 --steps 5 --rounds 1 > $OUT/pmc.out 2> $OUT/pmc.err
