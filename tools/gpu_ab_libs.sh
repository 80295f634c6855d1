#!/bin/bash
# A/B of library builds: 3 rounds of bench runs, each round over the product library and
# every variant named on the command line (NGRTD_LIB=<path>): headline kernel ms / exp_pist_flow
# kernel ms / sampler us per step (tools/build_variant.py builds variants).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/abl
for i in 1 2 3; do
  line="round $i: default"
  timeout -k 10 120 python bench.py --full-line --steps 400 --warmup 40 --no-cpu-baseline > gpurun_out/abl/d$i.json 2>/dev/null || exit 1
  line="$line $(python -c "import json;d=json.load(open('gpurun_out/abl/d$i.json'));m=d.get('models',{});s=d.get('sampler',{});print('%.5f/%.5f/%.2f' % (d['roofline']['kernel_ms'], m.get('exp_pist_flow',{}).get('kernel_ms',0), s.get('us_per_step',0)))")"
  for v in "$@"; do
    n=$(basename $v .so)
    timeout -k 10 120 env NGRTD_LIB=$PWD/$v python bench.py --full-line --steps 400 --warmup 40 --no-cpu-baseline > gpurun_out/abl/$n.$i.json 2>/dev/null || exit 1
    line="$line | $n $(python -c "import json;d=json.load(open('gpurun_out/abl/$n.$i.json'));m=d.get('models',{});s=d.get('sampler',{});print('%.5f/%.5f/%.2f' % (d['roofline']['kernel_ms'], m.get('exp_pist_flow',{}).get('kernel_ms',0), s.get('us_per_step',0)))")"
  done
  echo "$line"
done
