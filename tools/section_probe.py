#!/usr/bin/env python3
"""Per-section shader-clock timing of logp_fused_kernel (c4 workload, ROLES = 2 layout).

Builds noblegas_rtd_mcmc_amd/libngrtd_probe.so with -DNGRTD_SECTION_PROBE (lane 0 of each
wave stamps s_memtime at the NGRTD_PROBE points of ngrtd_kernels.hpp), runs the c4
log-prob, and prints the median cycles per section for the theta-role waves (0-7 of each
block) and the RTD-role waves (8-15):

  0->1 prologue: table loads, LDS stores, barrier
  1->3 the role's work (RTD waves: 1->2 surrogate + likelihood, 2->3 exact fallback)
  3->6 exchange barrier (th + like)          6->7 per-walker sum over wells

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
    ap.add_argument("--variant", default="joint", choices=["joint", "rtd_only", "rtd_bare", "dz"])
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
    if args.variant == "dz":     # one single-launch DEMetropolisZ step after 10 steps
        from noblegas_rtd_mcmc_amd.sampler import DeviceDEMetropolisZ
        x, l, z = DeviceDEMetropolisZ(lp, tune=None, seed=7).start(dev, 0, 12)
        lp.demcz(x, l, 10, z)
        torch.cuda.synchronize()
    lp.ctx.set_profiling(True)
    lp.kernel_stats(reset=True)
    if args.variant == "dz":
        lp.demcz(x, l, 1, z)
    else:
        lp(dev, out=out)
    torch.cuda.synchronize()
    ks = lp.kernel_stats(reset=True)
    lib = _lib.load()
    lib.ngrtd_probe_read.argtypes = [C.c_void_p, C.c_int64]
    nwaves = (args.walkers * args.wells + 511) // 512 * 16
    buf = np.zeros(nwaves * 8, dtype=np.uint64)
    assert lib.ngrtd_probe_read(buf.ctypes.data, buf.size) == 0
    t = buf.reshape(-1, 8).astype(np.int64)
    w = np.arange(t.shape[0]) % 16
    res = {"kernel_us_event": ks["fused"][0] * 1e3}
    for grp, sel in (("theta_role", w < 8), ("rtd_role", w >= 8)):
        tt = t[sel]
        r = {"prologue": tt[:, 1] - tt[:, 0], "work": tt[:, 3] - tt[:, 1], "exchange": tt[:, 6] - tt[:, 3],
             "reduce": tt[:, 7] - tt[:, 6], "total": tt[:, 7] - tt[:, 0]}
        if grp == "theta_role" and args.variant == "dz":
            r["dz_stage"] = tt[:, 4] - tt[:, 0]
        if grp == "rtd_role":
            r["surrogate_like"] = tt[:, 2] - tt[:, 1]
            r["theta_load_piece"] = tt[:, 4] - tt[:, 1]
            r["clenshaw"] = tt[:, 5] - tt[:, 4]
            r["conc_like"] = tt[:, 2] - tt[:, 5]
        res[grp] = {k: float(np.median(v)) for k, v in r.items()}
    # s_memtime counters are per XCD (block b runs on XCD b % 8): spans within one XCD
    blk = np.arange(t.shape[0]) // 16
    sel = (blk % 8) == 0
    t0 = t[sel, 0].min()
    res["xcd0_span_cycles"] = int(t[sel, 7].max() - t0)
    res["xcd0_wave_start_p50_p90_max"] = np.percentile(t[sel, 0] - t0, [50, 90, 100]).tolist()
    res["xcd0_theta_end_p10_p50_max"] = np.percentile(t[sel & (w < 8), 3] - t0, [10, 50, 100]).tolist()
    res["xcd0_rtd_end_p10_p50_max"] = np.percentile(t[sel & (w >= 8), 3] - t0, [10, 50, 100]).tolist()
    res["xcd0_wave_end_p10_p50_max"] = np.percentile(t[sel, 7] - t0, [10, 50, 100]).tolist()
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
