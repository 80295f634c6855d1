#!/bin/bash
# A/B of the lane-chain exp_pist_flow step (bench sampler line rtd_4tracer_123_exp_pist_flow):
# the product library vs libngrtd_tpd14.so (tools/build_variant.py tpd14 -DNGRTD_EPM_TAIL_PRE_DZ=14).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04zd
mkdir -p $OUT
for i in 1 2 3; do
  line="round $i:"
  for cfg in "default:" "tpd14:NGRTD_LIB=noblegas_rtd_mcmc_amd/libngrtd_tpd14.so"; do
    n=${cfg%%:*}; ev=${cfg#*:}
    timeout -k 10 180 env ${ev} python bench.py --full-line --steps 50 --warmup 5 --no-cpu-baseline --no-models --no-exact \
      > $OUT/$n.$i.json 2> $OUT/$n.$i.err || { echo "$n failed"; exit 1; }
    line="$line | $n $(python -c "import json;d=json.load(open('$OUT/$n.$i.json'));s=d['sampler'];print('%.2f/%.2f' % (s['rtd_4tracer_123_exp_pist_flow']['us_per_step'], s['rtd_4tracer_123']['us_per_step']))")"
  done
  echo "$line"
done
