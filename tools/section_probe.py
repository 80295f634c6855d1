#!/usr/bin/env python3
"""Per-section shader-clock timing of logp_fused_kernel (c4 workload).

Builds noblegas_rtd_mcmc_amd/libngrtd_probe.so with -DNGRTD_SECTION_PROBE (lane 0 of each
wave stamps s_memtime at 8 points, ngrtd_kernels.hpp NGRTD_PROBE), runs the c4 log-prob,
and prints the median cycles per section for the RTD-first waves (0-3) and the CE-first
waves (4-7) of each block:

  0->1 fragment-table LDS copy + barrier     1->2 CE/prior part (CE-first waves)
  2->3 MFMA init (q powers)                   3->4 MFMA steps
  4->5 segment recombination + tile pick      5->6 conc + RTD likelihood (+ CE, RTD-first)
  6->7 barrier + per-walker sum over wells

    python tools/section_probe.py [--wells 64] [--walkers 2048]
"""
import argparse
import ctypes as C
import json
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "noblegas_rtd_mcmc_amd")
PROBE_LIB = os.path.join(PKG, "libngrtd_probe.so")


def build():
    sys.path.insert(0, REPO)
    import __graft_entry__ as g
    src = os.path.join(PKG, "csrc", "ngrtd.hip")
    if not os.path.exists(PROBE_LIB) or os.path.getmtime(PROBE_LIB) < max(os.path.getmtime(p) for p in g._deps()):
        subprocess.run(["hipcc"] + g.HIPCC_FLAGS + ["-DNGRTD_SECTION_PROBE", "-o", PROBE_LIB, src], check=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--wells", type=int, default=64)
    ap.add_argument("--walkers", type=int, default=2048)
    ap.add_argument("--build-only", action="store_true")
    ap.add_argument("--variant", default="joint", choices=["joint", "rtd_only", "rtd_bare"])
    args = ap.parse_args()
    build()
    if args.build_only:
        return
    os.environ["NGRTD_LIB"] = PROBE_LIB
    sys.path.insert(0, REPO)
    import torch
    from noblegas_rtd_mcmc_amd import _lib, workloads
    from noblegas_rtd_mcmc_amd.engine import LogProb
    spec = workloads.c4_spec(L=args.wells)
    if args.variant != "joint":
        import dataclasses
        from noblegas_rtd_mcmc_amd.spec import ModelSpec
        spec = ModelSpec(n_wells=args.wells, rtd=spec.rtd)
        if args.variant == "rtd_bare":
            spec = dataclasses.replace(spec, include_prior=False, include_like=False, roles=[])
    th = workloads.sample_prior(spec, args.walkers, np.random.default_rng(34568))
    lp = LogProb(spec, max_walkers=args.walkers)
    dev = torch.from_numpy(th).cuda()
    out = torch.empty(args.walkers, dtype=torch.float64, device="cuda")
    for _ in range(20):
        lp(dev, out=out)
    torch.cuda.synchronize()
    lp.ctx.set_profiling(True)
    lp.kernel_stats(reset=True)
    lp(dev, out=out)
    torch.cuda.synchronize()
    ks = lp.kernel_stats(reset=True)
    lib = _lib.load()
    lib.ngrtd_probe_read.argtypes = [C.c_void_p, C.c_int64]
    blocks = lp.info(args.walkers)
    nwaves = (args.walkers * args.wells + 511) // 512 * 8
    buf = np.zeros(nwaves * 8, dtype=np.uint64)
    assert lib.ngrtd_probe_read(buf.ctypes.data, buf.size) == 0
    t = buf.reshape(-1, 8).astype(np.int64)
    d = np.diff(t, axis=1)
    names = ["lds_copy", "ce_first_theta", "mfma_init", "mfma_steps", "finish_pick", "conc_like(+theta)",
             "reduce"]
    res = {"kernel_us_event": ks["fused"][0] * 1e3, "span_cycles": int(t[:, 7].max() - t[:, 0].min())}
    w = np.arange(t.shape[0]) % 8
    for grp, sel in (("rtd_first", w < 4), ("ce_first", w >= 4)):
        res[grp] = {n: float(np.median(d[sel, i])) for i, n in enumerate(names)}
        res[grp]["total"] = float(np.median(t[sel, 7] - t[sel, 0]))
    # s_memtime counters are per XCD (block b runs on XCD b % 8): spans within one XCD
    blk = np.arange(t.shape[0]) // 8
    spans, starts, ends = [], [], []
    for x in range(8):
        sel = (blk % 8) == x
        if sel.any():
            t0 = t[sel, 0].min()
            spans.append(int(t[sel, 7].max() - t0))
            starts.append(np.percentile(t[sel, 0] - t0, [50, 90, 100]).tolist())
            ends.append(np.percentile(t[sel, 7] - t0, [10, 50, 100]).tolist())
    res["xcd_span_cycles"] = spans
    res["xcd_wave_start_p50_p90_max"] = starts[0]
    res["xcd_wave_end_p10_p50_max"] = ends[0]
    del res["span_cycles"]
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
