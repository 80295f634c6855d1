#!/usr/bin/env python3
"""Summarise tools/gpu_model_pmc.sh: per model (key "model[.savenum]@N"), the per-launch PMC
averages of its log-prob kernel and the derived FP64 FLOPs per unit and HBM bytes per launch
(FETCH_SIZE doubled per MI355X_MICROARCH.md 'HBM' -- tools/fetch_calib.hip -- + WRITE_SIZE, both
KiB), merged into OUT.json (bench.py's model lines read it):

    python tools/model_pmc_summary.py gpurun_out/TAG profiles/r05_model_pmc.json"""
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import summarize  # noqa: E402


def main(src, dst):
    out = json.load(open(dst)) if os.path.exists(dst) else {}
    for d in sorted(glob.glob(os.path.join(src, "*", ""))):
        runs = [json.loads(open(f).read().strip().splitlines()[-1]) for f in sorted(glob.glob(os.path.join(d, "run*.json")))
                if os.path.getsize(f)]
        if not runs:
            continue
        r0 = runs[0]
        res = summarize(sorted(glob.glob(os.path.join(d, "p*"))))
        ks = [k for k in res if "logp_fused_kernel" in k]
        if len(ks) != 1:
            continue
        c = res[ks[0]]
        mod, _, sv = r0["model"].partition(":")
        key = mod + ("." + sv if sv and sv != "0" else "") + "@N%d" % r0["ages"]
        e = {k: v for k, v in c.items() if not k.startswith("dur")}
        e["us_per_launch_pmc_runs"] = [r["us_per_launch"] for r in runs]
        e["kernel"] = r0["kernel"]
        e["units"] = r0["units"]
        e["finite_frac"] = r0["finite_frac"]
        if r0.get("tau2_hi") is not None:
            e["tau2_hi"] = r0["tau2_hi"]
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            e["hbm_bytes_per_launch"] = (2.0 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024.0
        if "SQ_INSTS_VALU_FLOPS_FP64" in c:
            fl = 64.0 * (c["SQ_INSTS_VALU_FLOPS_FP64"] + c.get("SQ_INSTS_VALU_FLOPS_FP64_TRANS", 0.0)) \
                + 512.0 * c.get("SQ_INSTS_VALU_MFMA_MOPS_F64", 0.0)
            e["fp64_flop_per_launch"] = fl
            e["fp64_flop_per_unit"] = fl / r0["units"]
        out[key] = e
    with open(dst, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print(json.dumps({k: {c: round(v, 2) for c, v in e.items() if isinstance(v, float)} for k, e in out.items()},
                     indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
