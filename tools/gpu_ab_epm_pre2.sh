#!/bin/bash
# A/B of the LW / DZ exp_pist_flow tail prefetch depths with the mixed pieces: the LW log-prob
# (model_probe) and the lane-chain EPM step + joint steps (gpu_ab_sampler.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for i in 1 2; do
  for v in default lw5 lw10 dz5; do
    if [ $v = default ]; then L=""; else L="NGRTD_LIB=$PWD/noblegas_rtd_mcmc_amd/libngrtd_$v.so"; fi
    echo -n "$v "; env $L timeout -k 10 120 python tools/model_probe.py --models exp_pist_flow:123,exp_pist_flow-piston:123 --steps 200 --rounds 1 2>/dev/null | grep '^{' || exit 1
  done
done
