#!/bin/bash
# Round-2: full GPU tests + published-model bench lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r02d
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r02d/tests.log 2>&1
rc=$?; tail -15 gpurun_out/r02d/tests.log; [ $rc -eq 0 ] || exit $rc
for m in "exp_pist_flow" "exponential --mod-type2 piston" "exp_pist_flow --mod-type2 piston"; do
  tag=$(echo $m | tr -d ' -')
  timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --mod-type1 $m > gpurun_out/r02d/m_$tag.json 2>/dev/null || exit 1
done
python - <<'PY'
import json,glob
for f in sorted(glob.glob("gpurun_out/r02d/*.json")):
    d=json.load(open(f)); r=d["roofline"]
    print(f, "%.4g"%d["value"], "ms/step %.4f"%d["ms_per_step"], "kern %.4f"%r["kernel_ms"], r["kernel"], r["bound"], "frac %.3f"%r["frac"], d["kernels_ms"])
PY
