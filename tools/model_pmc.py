#!/usr/bin/env python3
"""ONE log-prob plan launched K times back to back, for PMC passes that must count only that
model's launches (tools/gpu_model_pmc.sh; the bench's model lines read the summary):

    python tools/model_pmc.py --model exp_pist_flow:123 [--ages 25256] [--steps 50] [--tau2-hi 1000]

Model = mod_type1[-mod_type2]:savenum as bench.py's model lines (c4 shape: 2048 walkers x 64
wells, joint CE + 5 tracers); --tau2-hi draws tau2 from U(50, tau2_hi) instead of its prior
U(50, 15000) (a second exp_pist_flow component at N = 1200).  Prints one JSON line: model,
ages, units per launch, launches, us per launch, finite fraction, kernel instance."""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", required=True)
    ap.add_argument("--ages", type=int, default=1200)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--walkers", type=int, default=2048)
    ap.add_argument("--wells", type=int, default=64)
    ap.add_argument("--tau2-hi", type=float, default=None)
    args = ap.parse_args()
    import torch
    import bench
    from noblegas_rtd_mcmc_amd import workloads as wl
    from noblegas_rtd_mcmc_amd.engine import LogProb
    mod, _, sv = args.model.partition(":")
    m1, _, m2 = mod.partition("-")
    ns = argparse.Namespace(wells=args.wells, ages=args.ages, mod_type1=m1, mod_type2=m2 or None)
    spec = bench.model_spec(ns, sv if sv != "0" else "")
    th = wl.sample_prior(spec, args.walkers, np.random.default_rng(34568))
    if args.tau2_hi is not None:
        R = {r: i for i, r in enumerate(spec.roles)}
        th[R["tau2"]] = np.random.default_rng(8).uniform(50.0, args.tau2_hi, th[R["tau2"]].shape)
    th = torch.from_numpy(th).cuda()
    lp = LogProb(spec, max_walkers=args.walkers)
    out = torch.empty(args.walkers, dtype=torch.float64, device="cuda")
    run = lp.bind_n(th, out)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    run(args.steps)
    e1.record()
    torch.cuda.synchronize()
    print(json.dumps({"model": args.model, "ages": args.ages, "units": args.walkers * args.wells,
                      "launches": args.steps, "us_per_launch": e0.elapsed_time(e1) / args.steps * 1e3,
                      "finite_frac": float(torch.isfinite(out).double().mean()),
                      "kernel": bench.fused_instance(m1, m2 or None, sv if sv != "0" else ""),
                      "tau2_hi": args.tau2_hi}))
    lp.close()


if __name__ == "__main__":
    main()
