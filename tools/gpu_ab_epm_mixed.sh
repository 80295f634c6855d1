#!/bin/bash
# A/B: all-double EPM tail pieces for the plain plans (product) vs mixed pieces with 5 / 10 / 15
# chunks loaded ahead (NGRTD_EPM_MIXED_ALL builds), 2 interleaved rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for i in 1 2; do
  for v in ${VARS:-default mix5 mix10 mix15}; do
    if [ $v = default ]; then L=""; else L="NGRTD_LIB=$PWD/noblegas_rtd_mcmc_amd/libngrtd_$v.so"; fi
    echo -n "$v "; env $L timeout -k 10 120 python tools/model_probe.py --models exp_pist_flow:0,exp_pist_flow-piston:0,exp_pist_flow:123 --steps 200 --rounds 1 2>/dev/null | grep '^{' || exit 1
  done
done
