#!/bin/bash
# A/B of the device DEMetropolisZ step: 3 rounds of bench.py's sampler line (no headline side
# lines) over configurations given as "NAME:ENV=VAL[,ENV=VAL]" (or "NAME:" for the default;
# NGRTD_LIB=<path> selects a variant library) -> us per step transformed / natural / joint, then the lane-chain shapes (RTD 4 tracers 123,
# its exp_pist_flow, RTD 1 tracer, CE-only).
#   bash tools/gpu_ab_sampler.sh TAG "default:" "write:NGRTD_DZ_PROP_WRITE=1" ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
for i in 1 2 3; do
  line="round $i:"
  for cfg in "$@"; do
    n=${cfg%%:*}; ev=${cfg#*:}
    timeout -k 10 240 env ${ev//,/ } python bench.py --full-line --steps 200 --warmup 20 --no-cpu-baseline --no-models --no-exact \
      --no-reference-runs \
      > $OUT/$n.$i.json 2> $OUT/$n.$i.err || { echo "$n failed"; exit 1; }
    line="$line | $n $(python -c "import json;d=json.load(open('$OUT/$n.$i.json'));s=d['sampler'];print('%.2f/%.2f/%.2f lane %.2f/%.2f/%.2f/%.2f' % (s['transformed']['us_per_step'], s['natural']['us_per_step'], s['transformed_joint']['us_per_step'], *[s[k]['us_per_step'] for k in ('rtd_4tracer_123', 'rtd_4tracer_123_exp_pist_flow', 'rtd_1tracer', 'ce_only')]))")"
  done
  echo "$line"
done
