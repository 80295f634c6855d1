#!/bin/bash
# A/B of library builds on the sampler legs (bench `sampler`: 2048 walkers x 64 wells) and the
# reference's own runs (bench `reference_runs`: 1 well x 3 chains): 2 interleaved rounds over
# the product library and every variant named (NGRTD_LIB=<path>), full records under
# gpurun_out/absr/, one summary line per run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/absr
summ() {
  python - "$1" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
s = d.get("sampler", {})
r = d.get("reference_runs", {}).get("runs", [])
sm = {k: round(v["us_per_step"], 2) for k, v in s.items() if isinstance(v, dict) and "us_per_step" in v}
rr = {x["run"]: round(x["wall_s"], 3) for x in r if isinstance(x, dict) and "wall_s" in x}
print(json.dumps({"sampler_us": sm, "ref_wall_s": rr}))
PY
}
for i in 1 2; do
  for v in noblegas_rtd_mcmc_amd/libngrtd.so "$@"; do
    n=$(basename $v .so)
    timeout -k 10 300 env NGRTD_LIB=$PWD/$v python bench.py --full-line --steps 20 --warmup 5 --no-cpu-baseline --no-models > gpurun_out/absr/$n.$i.json 2> gpurun_out/absr/$n.$i.err || exit 1
    echo "round $i $n $(summ gpurun_out/absr/$n.$i.json)" >> gpurun_out/absr/summary.txt
  done
done
