#!/usr/bin/env python3
"""Per-step time of the device DEMetropolisZ at the reference's dispersion run shape -- RTD-only,
4 tracers, savenum 123, 1 well, 3 chains, N = 25 256, PyMC3's transformed space, per-well chains
(run_age_mcmc.py:61-70,170-178,209) -- through ngrtd_demcz_run (the proposal, wide-sum, log-prob
and accept kernels per step), after 200 tune steps.  JSON line; run it under
`rocprofv3 --kernel-trace --stats` for the kernels' share of the step.

    python tools/disp_step_probe.py [--model2 piston] [--steps 1000]"""
import argparse
import dataclasses
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model2", default=None)
    ap.add_argument("--chains", type=int, default=3)
    ap.add_argument("--steps", type=int, default=1000)
    args = ap.parse_args()
    import torch
    from noblegas_rtd_mcmc_amd import workloads as wl
    from noblegas_rtd_mcmc_amd.engine import LogProb
    from noblegas_rtd_mcmc_amd.sampler import DeviceDEMetropolisZ
    spec = wl.rtd_only_spec(L=1, N=25256, tracers=("CFC12", "SF6", "H3", "He4_ter"), mod_type1="dispersion",
                            mod_type2=args.model2, savenum="123")
    spec = dataclasses.replace(spec, jacobian=True)
    W = args.chains
    th = torch.from_numpy(wl.test_point(spec, W)).cuda()
    lp = LogProb(spec, max_walkers=W)
    n = args.steps
    s = DeviceDEMetropolisZ(lp, tune_interval=100, seed=7, transformed=True, per_well=True)
    x, l, z = s.start(th, 200, 200 + n + 1)
    lp.demcz(x, l, 200, z)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    lp.demcz(x, l, n, z)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / n
    res = {"model": "dispersion" + ("-" + args.model2 if args.model2 else ""), "chains": W,
           "geometry": lp.info(W).get("disp_wide_g"), "us_per_step": dt * 1e6}
    print(json.dumps(res))
    lp.close()


if __name__ == "__main__":
    main()
