#!/bin/bash
# A/B of library builds: 3 rounds of bench runs, each round over the product library and
# every variant named on the command line (NGRTD_LIB=<path>), kernel time per launch.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/abl
for i in 1 2 3; do
  line="round $i: default"
  timeout -k 10 120 python bench.py --steps 400 --warmup 40 --no-cpu-baseline > gpurun_out/abl/d$i.json 2>/dev/null || exit 1
  line="$line $(python -c "import json;d=json.load(open('gpurun_out/abl/d$i.json'));print(d['roofline']['kernel_ms'])")"
  for v in "$@"; do
    n=$(basename $v .so)
    timeout -k 10 120 env NGRTD_LIB=$PWD/$v python bench.py --steps 400 --warmup 40 --no-cpu-baseline > gpurun_out/abl/$n.$i.json 2>/dev/null || exit 1
    line="$line | $n $(python -c "import json;d=json.load(open('gpurun_out/abl/$n.$i.json'));print(d['roofline']['kernel_ms'])")"
  done
  echo "$line"
done
