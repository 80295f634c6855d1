#!/bin/bash
# Round-2 check: all GPU tests, then the bench variants (headline, strong c5 shard, published models).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r02b
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r02b/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r02b/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r02b/b20.json 2> gpurun_out/r02b/b20.err || exit 1
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/r02b/b200.json 2>/dev/null || exit 1
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --walkers 256 --scaling strong > gpurun_out/r02b/b256.json 2>/dev/null || exit 1
for m in "exp_pist_flow" "exponential --mod-type2 piston" "exp_pist_flow --mod-type2 piston"; do
  tag=$(echo $m | tr -d ' -')
  timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --mod-type1 $m > gpurun_out/r02b/m_$tag.json 2>/dev/null || exit 1
done
python - <<'PY'
import json,glob
for f in sorted(glob.glob("gpurun_out/r02b/*.json")):
    d=json.load(open(f)); r=d["roofline"]
    print(f, "%.4g"%d["value"], "ms/step %.4f"%d["ms_per_step"], "kern %.4f"%r["kernel_ms"], r["bound"], "frac %.3f"%r["frac"],
          "exact", d.get("exact_value"), "plan_ms %.1f"%d["plan_build_ms"], "cpu", (d.get("cpu_baseline") or {}).get("variants"))
PY
