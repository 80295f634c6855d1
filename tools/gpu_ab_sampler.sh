#!/bin/bash
# A/B of the device DEMetropolisZ step: 3 rounds of bench.py's sampler line (no headline side
# lines) over configurations given as "NAME:ENV=VAL[,ENV=VAL]" (or "NAME:" for the default;
# NGRTD_LIB=<path> selects a variant library) -> us per step transformed / natural / joint.
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
    timeout -k 10 180 env ${ev//,/ } python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-models --no-exact \
      > $OUT/$n.$i.json 2> $OUT/$n.$i.err || { echo "$n failed"; exit 1; }
    line="$line | $n $(python -c "import json;d=json.load(open('$OUT/$n.$i.json'));s=d['sampler'];print('%.2f/%.2f/%.2f' % (s['transformed']['us_per_step'], s['natural']['us_per_step'], s['transformed_joint']['us_per_step']))")"
  done
  echo "$line"
done
