#!/usr/bin/env python3
"""Per-variant instruction mix of logp_fused_kernel from tools/gpu_mix.sh passes:

    python tools/mix_summary.py gpurun_out/mix

prints, per library variant, the per-launch counter averages and the VALU issue estimate
(FP64 add/mul/fma/trans at 8 cycles per wave instruction on gfx950, every other VALU
instruction at 4), per wave."""
import collections
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import summarize  # noqa: E402


def main(root):
    groups = collections.defaultdict(list)
    for d in sorted(glob.glob(os.path.join(root, "*_pmc*"))):
        if os.path.isdir(d):
            groups[os.path.basename(d).rsplit("_pmc", 1)[0]].append(d)
    for name, dirs in groups.items():
        res = summarize(dirs)
        for k, c in res.items():
            if "logp_fused_kernel" not in k:
                continue
            waves = c.get("SQ_WAVES", 0) or 1
            f64 = sum(c.get(x, 0) for x in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64",
                                           "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_TRANS_F64"))
            valu = c.get("SQ_INSTS_VALU", 0)
            print("%-14s %s" % (name, k[:48]))
            print("   per wave: VALU %.0f (FP64 %.0f, other %.0f; int32 %.0f, int64 %.0f, cvt %.0f)  SALU %.0f  LDS %.0f"
                  % (valu / waves, f64 / waves, (valu - f64) / waves, c.get("SQ_INSTS_VALU_INT32", 0) / waves,
                     c.get("SQ_INSTS_VALU_INT64", 0) / waves, c.get("SQ_INSTS_VALU_CVT", 0) / waves,
                     c.get("SQ_INSTS_SALU", 0) / waves, c.get("SQ_INSTS_LDS", 0) / waves))
            print("   VALU issue estimate %.0f cycles/wave; WAVE_CYCLES %.0f, ACTIVE_INST_VALU %.0f, WAIT_INST_ANY %.0f"
                  " (quad-cycles per wave); dur %.2f us"
                  % ((8 * f64 + 4 * (valu - f64)) / waves, c.get("SQ_WAVE_CYCLES", 0) / waves,
                     c.get("SQ_ACTIVE_INST_VALU", 0) / waves, c.get("SQ_WAIT_INST_ANY", 0) / waves,
                     c.get("dur_us[SQ_WAVES]", 0)))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/mix")
