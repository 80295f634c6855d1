#!/usr/bin/env python3
"""Per-section shader-clock timing of logp_fused_kernel (c4 workload, ROLES = 2 layout).

Builds noblegas_rtd_mcmc_amd/libngrtd_probe.so with -DNGRTD_SECTION_PROBE (lane 0 of each
wave stamps s_memtime at the NGRTD_PROBE points of ngrtd_kernels.hpp), runs the c4
log-prob, and prints the median cycles per section for the theta-role waves (0-7 of each
block) and the RTD-role waves (8-15):

  0->1 prologue: table loads, LDS stores, barrier
  1->3 the role's work (RTD waves: 1->2 surrogate + likelihood, 2->3 exact fallback)
  3->6 exchange barrier (th + like)          6->7 per-walker sum over wells

--variant dz: the last step of a multi-step DEMetropolisZ launch (--dz-steps, per-well /
joint chains, natural / transformed space), its sections
  8->9 staging (partners, noise, history append, proposal): 8->14 arguments and partner
  indices, 14->15 the proposal values, 15->9 the stores   9->1 staging barrier
  1->3 the role's work   3->13 the next step's partner-row loads issued (kDzPrefetch builds)
  13->6 exchange   6->10 decision   10->11 commit barrier   11->12 commit

    python tools/section_probe.py [--wells 64] [--walkers 2048] [--variant dz --pw 1 --jac 1]
                                  [--model exp_pist_flow [--model2 piston] --savenum 123]
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


def probe_lib(defines):
    return PROBE_LIB if not defines else PROBE_LIB.replace(".so", "_" + "_".join(
        d.replace("=", "").lower() for d in defines) + ".so")


def build(defines=()):
    """Both translation units with -DNGRTD_SECTION_PROBE (the DZ instances live in
    ngrtd_dz.hip, with its own probe buffer) and any --define, linked into
    libngrtd_probe[_<defines>].so."""
    sys.path.insert(0, REPO)
    import __graft_entry__ as g
    lib = probe_lib(defines)
    if not os.path.exists(lib) or os.path.getmtime(lib) < max(os.path.getmtime(p) for p in g._deps()):
        objs, procs = [], []
        for src in g._sources():          # in parallel, as __graft_entry__.build
            obj = src + ".probe%d.o" % os.getpid()
            procs.append(subprocess.Popen(["hipcc"] + g.HIPCC_FLAGS + g.EXTRA_FLAGS.get(os.path.basename(src), []) +
                                          ["-DNGRTD_SECTION_PROBE"] + ["-D" + d for d in defines] + ["-c", "-o", obj, src]))
            objs.append(obj)
        for pr in procs:
            if pr.wait() != 0:
                raise subprocess.CalledProcessError(pr.returncode, pr.args)
        subprocess.run(["hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", lib] + objs + ["-ldl"], check=True)
        for o in objs:
            os.remove(o)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--wells", type=int, default=64)
    ap.add_argument("--walkers", type=int, default=2048)
    ap.add_argument("--build-only", action="store_true")
    ap.add_argument("--variant", default="joint", choices=["joint", "rtd_only", "rtd_bare", "dz"])
    ap.add_argument("--pw", type=int, default=1)
    ap.add_argument("--jac", type=int, default=1)
    ap.add_argument("--dz-steps", type=int, default=8)
    ap.add_argument("--define", action="append", default=[], help="extra -D for the probe build (A/B)")
    ap.add_argument("--model", default="exponential", help="first RTD component (mod_type1), e.g. exp_pist_flow")
    ap.add_argument("--model2", default=None, help="second RTD component (mod_type2), e.g. piston")
    ap.add_argument("--savenum", default="", help="'123': J, thalf_cfc, lamsf6 sampled")
    args = ap.parse_args()
    build(args.define)
    if args.build_only:
        return
    os.environ["NGRTD_LIB"] = probe_lib(args.define)
    sys.path.insert(0, REPO)
    import torch
    from noblegas_rtd_mcmc_amd import _lib, workloads
    from noblegas_rtd_mcmc_amd.engine import LogProb
    spec = workloads.c4_spec(L=args.wells, mod_type1=args.model, mod_type2=args.model2,
                             par_names=workloads.model_par_names(args.model, args.model2, args.savenum))
    if args.variant == "dz" and args.jac:
        import dataclasses
        spec = dataclasses.replace(spec, jacobian=True)
    if args.variant not in ("joint", "dz"):
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
    if args.variant == "dz":     # a multi-step DEMetropolisZ launch after 50 steps
        from noblegas_rtd_mcmc_amd.sampler import DeviceDEMetropolisZ
        x, l, z = DeviceDEMetropolisZ(lp, tune=None, seed=7, per_well=bool(args.pw)).start(dev, 0, 60 + args.dz_steps)
        lp.demcz(x, l, 50, z)
        torch.cuda.synchronize()
    lp.ctx.set_profiling(True)
    lp.kernel_stats(reset=True)
    if args.variant == "dz":
        lp.demcz(x, l, args.dz_steps, z)
    else:
        lp(dev, out=out)
    torch.cuda.synchronize()
    ks = lp.kernel_stats(reset=True)
    lib = _lib.load()
    rd = lib.ngrtd_probe_read_dz if args.variant == "dz" else lib.ngrtd_probe_read
    rd.argtypes = [C.c_void_p, C.c_int64]
    nwaves = (args.walkers * args.wells + 511) // 512 * 16
    buf = np.zeros(nwaves * 16, dtype=np.uint64)
    assert rd(buf.ctypes.data, buf.size) == 0
    t = buf.reshape(-1, 16).astype(np.int64)
    w = np.arange(t.shape[0]) % 16
    res = {"kernel_us_event": ks["fused"][0] * 1e3}
    if args.variant == "dz":
        res["us_per_step_event"] = res["kernel_us_event"] / args.dz_steps
        res["per_well"], res["transformed"] = bool(args.pw), bool(args.jac)
        for grp, sel in (("theta_role", w < 8), ("rtd_role", w >= 8)):
            tt = t[sel]
            r = {"stage": tt[:, 9] - tt[:, 8], "stage_args": tt[:, 14] - tt[:, 8], "stage_values": tt[:, 15] - tt[:, 14],
                 "stage_stores": tt[:, 9] - tt[:, 15],
                 "stage_barrier": tt[:, 1] - tt[:, 9], "work": tt[:, 3] - tt[:, 1],
                 "prefetch_issue": tt[:, 13] - tt[:, 3], "exchange": tt[:, 6] - tt[:, 13],
                 "decision": tt[:, 10] - tt[:, 6],
                 "commit_barrier": tt[:, 11] - tt[:, 10], "commit": tt[:, 12] - tt[:, 11],
                 "step": tt[:, 12] - tt[:, 8]}
            res[grp] = {k: float(np.median(v)) for k, v in r.items()}
        print(json.dumps(res, indent=1))
        return
    for grp, sel in (("theta_role", w < 8), ("rtd_role", w >= 8)):
        tt = t[sel]
        r = {"prologue": tt[:, 1] - tt[:, 0], "work": tt[:, 3] - tt[:, 1], "exchange": tt[:, 6] - tt[:, 3],
             "reduce": tt[:, 7] - tt[:, 6], "total": tt[:, 7] - tt[:, 0]}
        if args.variant != "dz":   # the prologue's loads + LDS stores (0 -> 9), its barrier (9 -> 1)
            r["prologue_loads_stores"] = tt[:, 9] - tt[:, 0]
            r["prologue_barrier"] = tt[:, 1] - tt[:, 9]
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
    # wave start times within each XCD, relative to the XCD's median start (dispatch ramp)
    ramp = []
    for x in range(8):
        sx = t[(blk % 8) == x, 0].astype(np.float64)
        ramp.append((np.percentile(sx, [1, 50, 99]) - np.median(sx)).tolist())
    res["wave_start_p1_p50_p99_vs_median_per_xcd"] = ramp
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
