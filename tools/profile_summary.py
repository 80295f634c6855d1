#!/usr/bin/env python3
"""Condense a tools/gpu_profile.sh run into the files committed under profiles/:

    python tools/profile_summary.py gpurun_out/TAG profiles/rNN

writes rNN_kernel_stats.csv (rocprofv3 --stats of the bench command), rNN_pmc.json (per
launch averages of every PMC counter for the ngrtd kernels, plus HBM bytes per launch:
FETCH_SIZE doubled per MI355X_MICROARCH.md 'HBM' + WRITE_SIZE, both KiB counters) and
rNN_bench.json (the bench line)."""
import json
import os
import shutil
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import summarize  # noqa: E402


def main(src, prefix):
    os.makedirs(os.path.dirname(prefix) or ".", exist_ok=True)
    stats = os.path.join(src, "prof", "stats_kernel_stats.csv")
    if os.path.exists(stats):
        shutil.copy(stats, prefix + "_kernel_stats.csv")
    if os.path.exists(os.path.join(src, "bench.json")):
        shutil.copy(os.path.join(src, "bench.json"), prefix + "_bench.json")
    import glob
    res = summarize(sorted(glob.glob(os.path.join(src, "pmc*"))))
    units = None
    for name in ("bench.json", "prof_bench.json", "pmc_bench.json"):
        try:
            with open(os.path.join(src, name)) as f:
                units = json.loads(f.read().strip().splitlines()[-1])["geometry"]["units"]
            break
        except Exception:
            pass
    out = {}
    for k, d in res.items():
        if "ngrtd" not in k:
            continue
        e = {c: v for c, v in d.items()}
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            # FETCH_SIZE reports half the bytes for 8- and 16-byte-per-lane loads on gfx950
            # (MI355X_MICROARCH.md 'HBM'; tools/fetch_calib.hip: profiles/r01_fetch_calib.txt)
            e["hbm_bytes_per_launch"] = (2.0 * d["FETCH_SIZE"] + d["WRITE_SIZE"]) * 1024.0
        if "SQ_INSTS_VALU_FLOPS_FP64" in d:
            # FP64 FLOPs per launch.  SQ_INSTS_VALU_FLOPS_FP64 counts per wave instruction
            # (add/mul = 1, fma = 2: it equals ADD_F64 + MUL_F64 + 2 FMA_F64 of the same
            # launch), so x 64 lanes; transcendental (v_rcp/v_sqrt...) ops count 1 per lane;
            # MFMA FP64 adds MOPS x 512 (one 16x16x4 op = 2048 FLOP = 4 MOPS).
            e["fp64_flop_per_launch"] = 64.0 * (d["SQ_INSTS_VALU_FLOPS_FP64"]
                                                + d.get("SQ_INSTS_VALU_FLOPS_FP64_TRANS", 0.0)) \
                + 512.0 * d.get("SQ_INSTS_VALU_MFMA_MOPS_F64", 0.0)
        if units and "fp64_flop_per_launch" in e:
            e["units"] = units          # (walker, well) units per launch of the profiled command
            e["fp64_flop_per_unit"] = e["fp64_flop_per_launch"] / units
        out[k] = e
    # several profiled commands (one per RTD model) merge into one summary, keyed by the
    # kernel instance name (logp_fused_kernel<C, FULL, ROLES, MIX>)
    if os.path.exists(prefix + "_pmc.json"):
        with open(prefix + "_pmc.json") as f:
            prev = json.load(f)
        prev.update(out)
        out = prev
    with open(prefix + "_pmc.json", "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print(json.dumps({k[:60]: {c: round(v, 1) for c, v in e.items() if not c.startswith("dur")}
                      for k, e in out.items()}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
