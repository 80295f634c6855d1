#!/usr/bin/env python3
"""Per-launch kernel time of c4-shape log-prob plans (A/B runs of library variants):

    python tools/model_probe.py [--models exp_pist_flow:123,exponential:0,...] [--steps 200] [--rounds 3]

Model = mod_type1[-mod_type2]:savenum (savenum digits 1 J, 2 thalf_cfc, 3 lamsf6, as bench.py).
Each round times every model once (HIP events around `steps` back-to-back launches on the
launch stream) so that variants run with NGRTD_LIB=... interleave fairly.  Prints one JSON
line: {model: [us per launch, per round]}."""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default="exp_pist_flow:0,exp_pist_flow:123")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--walkers", type=int, default=2048)
    ap.add_argument("--wells", type=int, default=64)
    ap.add_argument("--ages", type=int, default=1200, help="N (25256: the reference's full series)")
    args = ap.parse_args()
    import torch
    import bench
    from noblegas_rtd_mcmc_amd import workloads as wl
    from noblegas_rtd_mcmc_amd.engine import LogProb
    plans = []
    for m in args.models.split(","):
        mod, _, sv = m.partition(":")
        m1, _, m2 = mod.partition("-")
        ns = argparse.Namespace(wells=args.wells, ages=args.ages, mod_type1=m1, mod_type2=m2 or None)
        spec = bench.model_spec(ns, sv if sv != "0" else "")
        th = torch.from_numpy(wl.sample_prior(spec, args.walkers, np.random.default_rng(34568))).cuda()
        lp = LogProb(spec, max_walkers=args.walkers)
        out = torch.empty(args.walkers, dtype=torch.float64, device="cuda")
        plans.append((m, lp.bind_n(th, out), lp))
    res = {m: [] for m, _, _ in plans}
    for _ in range(args.rounds):
        for m, run, lp in plans:
            run(10)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            run(args.steps)
            e1.record()
            torch.cuda.synchronize()
            res[m].append(e0.elapsed_time(e1) / args.steps * 1e3)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
