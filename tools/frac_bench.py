#!/usr/bin/env python3
"""frac_inf_diff RTD benchmark: the fracture / matrix-diffusion
convolution of convolution_integral_utils.py:238-266 for a batch of parameter sets on the
c3 grid (N = 1200 ages x 1000 advective-time points per age), through ngrtd_frac_conv on
device memory, timed with HIP events on the launch stream.  The CPU baseline is the
oracle's reference-faithful NumPy restatement (numba, which the reference decorates these
helpers with, is not installed here) on a bounded sample, one core.  One JSON line.

    python tools/frac_bench.py [--sets 2048] [--ages 1200] [--reps 5]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sets", type=int, default=2048)
    ap.add_argument("--ages", type=int, default=1200)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--pmc-dir", default=None, help="rocprofv3 --pmc output of this tool (SQ_INSTS_VALU_FLOPS_FP64)")
    args = ap.parse_args()
    import torch
    from noblegas_rtd_mcmc_amd import _lib, workloads
    from noblegas_rtd_mcmc_amd.convolution_integral_utils import _series_id
    from oracle import rtd as orc

    n, N = args.sets, args.ages
    rng = np.random.default_rng(5005)
    tau = rng.uniform(2.0, 800.0, n)
    D = rng.uniform(0.01, 2.0, n)
    bbar = 10 ** rng.uniform(-5, -2, n)           # aux_scripts/age_modeling_mcmc.rtd_explore.py:257-258
    Phi = rng.uniform(0.005, 0.05, n)
    s = workloads.atmos_series("H3", N)
    c_by_age = s.c_by_age[:N]
    ctx = _lib.Context.get(0)
    stream = torch.cuda.current_stream()
    ctx.set_stream(stream.cuda_stream)
    sid, _ = _series_id(ctx, np.flip(c_by_age), np.arange(N - 1, -1, -1), 0)
    d = [torch.from_numpy(a).cuda() for a in (tau, D, bbar, Phi)]
    conc = torch.empty(n, dtype=torch.float64, device="cuda")
    fm = torch.empty(n, dtype=torch.float64, device="cuda")
    p = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731

    def run():
        ctx.check(ctx.lib.ngrtd_frac_conv(ctx.h, sid, 0, *[p(t) for t in d], None, 0, None, 12.34, None, 0.0, n,
                                          p(conc), None, p(fm), _lib.MEM_DEVICE), "ngrtd_frac_conv")

    run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.reps):
        run()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / args.reps
    got = conc.cpu().numpy()
    # parity + CPU baseline: oracle on a bounded sample of the same sets
    lam = orc.thalf_2_lambda(12.34)
    t_cpu, k, worst = 0.0, 0, 0.0
    idx = np.arange(N - 1, -1, -1)
    while t_cpu < args.cpu_seconds and k < n:
        t0 = time.perf_counter()
        g, _ = orc.frac_g_tp(N, 0, 0, tau[k], D[k], bbar[k], Phi[k])
        ref = orc.convolve(np.flip(c_by_age), idx, 0, None, None, lamba=lam, g_tau=g)
        t_cpu += time.perf_counter() - t0
        worst = max(worst, abs(got[k] - ref) / abs(ref))
        k += 1
    pts = float(n) * N * 1000
    line = {"workload": "frac_inf_diff (dispersion advective RTD) + H3 convolve: %d sets x N=%d ages x 1000 "
                        "advective points" % (n, N),
            "sets": n, "ms_per_call": ms, "sets_per_s": n / (ms * 1e-3), "inner_points_per_s": pts / (ms * 1e-3),
            "cpu_baseline": {"value": k / t_cpu, "unit": "sets/s", "cores": 1, "kind": "port",
                             "sample": "%d sets, oracle/rtd.py frac_g_tp + convolve (NumPy; numba absent)" % k},
            "max_rel_err_vs_oracle": worst}
    if args.pmc_dir and os.path.isdir(args.pmc_dir):
        sys.path.insert(0, os.path.join(REPO, "tools"))
        from pmc_summary import summarize
        for kname, e in summarize([args.pmc_dir]).items():
            if "frac_inner_kernel" in kname and e.get("SQ_INSTS_VALU_FLOPS_FP64"):
                # FP64 FLOP of one inner launch: SQ_INSTS_VALU_FLOPS_FP64 x 64 lanes (fma = 2),
                # the convention of bench.py / DESIGN.md 6; time: this run's per-call time
                # (the inner kernel is 99.9 % of it, profiles/r01_frac_kernel_stats.csv)
                flop = e["SQ_INSTS_VALU_FLOPS_FP64"] * 64
                ach = flop / (ms * 1e-3)
                line["roofline"] = {"bound": "mfma", "achieved": ach / 1e12, "peak": 78.6, "unit": "TFLOP/s",
                                    "frac": ach / 78.6e12, "fp64_valu_peak_measured": 38.3,
                                    "frac_of_fp64_valu_peak": ach / 38.3e12, "flop_per_call": flop,
                                    "flop_per_point": flop / pts, "kernel": "frac_inner_kernel"}
    print(json.dumps(line), flush=True)
    assert worst <= 1e-12, worst


if __name__ == "__main__":
    main()
