#!/usr/bin/env python3
"""MCMC sampler throughput on the c4 workload (2048 chains x 64 wells): chain-steps/s of
the device-resident DEMetropolisZ (ngrtd_demcz_run: ONE launch per step -- proposal from
the state and two history partners, history append, log-prob, Metropolis decision,
tuning, commit; NGRTD_DZ_MODE=pair selects the proposal kernel + log-prob kernel pair)
in PyMC3's transformed space and in the natural space, and of the torch-op
DEMetropolisZ loop around the same log-prob kernel.  One JSON line.

    python tools/sampler_bench.py [--steps 200]
"""
import argparse
import dataclasses
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def time_device(lp, x0, steps, warm=10):
    import torch
    from noblegas_rtd_mcmc_amd.sampler import DeviceDEMetropolisZ
    s = DeviceDEMetropolisZ(lp, tune_interval=100, seed=7)
    x, l, z = s.start(x0, 50, warm + steps)
    lp.demcz(x, l, warm, z)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    lp.demcz(x, l, steps, z)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--walkers", type=int, default=2048)
    args = ap.parse_args()
    import torch
    from noblegas_rtd_mcmc_amd import workloads
    from noblegas_rtd_mcmc_amd.engine import LogProb
    from noblegas_rtd_mcmc_amd.sampler import DEMetropolisZ, Transform
    W = args.walkers
    spec = workloads.c4_spec(L=64)
    th = workloads.sample_prior(spec, W, np.random.default_rng(34568))
    x0 = torch.from_numpy(th).cuda()
    R = spec.n_params * spec.n_wells
    out = {"workload": "c4: %d chains x %d wells x 8 params (R = %d theta rows per chain)" % (W, spec.n_wells, R)}
    lpn = LogProb(spec, max_walkers=W)
    lpj = LogProb(dataclasses.replace(spec, jacobian=True), max_walkers=W)
    dn = time_device(lpn, x0, args.steps)
    dj = time_device(lpj, x0, args.steps)
    # log-prob alone (same plan) for the split of the step
    o = torch.empty(W, dtype=torch.float64, device="cuda")
    for lp_, key in ((lpn, "natural"), (lpj, "transformed")):
        run = lp_.bind(x0, o)
        for _ in range(10):
            run()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            run()
        torch.cuda.synchronize()
        out["logp_alone_us_" + key] = (time.perf_counter() - t0) / args.steps * 1e6
    # algorithmic HBM bytes of one single-launch step: state + two partner rows read,
    # history append + proposal written = 5 R W doubles (+ the accepted chains' state
    # copies, 1 or 2 R W doubles at acceptance 1)
    nb = 5 * R * W * 8
    out["device_demcz_natural"] = {"us_per_step": dn * 1e6, "chain_steps_per_s": W / dn,
                                   "algorithmic_GBps": nb / dn * 1e-9}
    out["device_demcz_transformed"] = {"us_per_step": dj * 1e6, "chain_steps_per_s": W / dj,
                                       "algorithmic_GBps": nb / dj * 1e-9}
    out["step_bytes_algorithmic"] = nb
    out["single_launch_step"] = os.environ.get("NGRTD_DZ_MODE") != "pair"
    ts = max(10, args.steps // 10)
    f = lambda t: lpj(t)  # noqa: E731
    DEMetropolisZ(f, seed=3, transform=Transform.from_spec(spec)).run(x0, 3, 0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    DEMetropolisZ(f, seed=3, transform=Transform.from_spec(spec), tune=None).run(x0, ts, 0)
    torch.cuda.synchronize()
    tt = (time.perf_counter() - t0) / ts
    out["torch_demcz_transformed"] = {"us_per_step": tt * 1e6, "chain_steps_per_s": W / tt}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
