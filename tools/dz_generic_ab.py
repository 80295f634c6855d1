#!/usr/bin/env python3
"""Device DEMetropolisZ per-step time for the generic model pairs at the c4 shape (2048
walkers x 64 wells, joint CE + 5 tracers, PyMC3's transformed space, per-well chains): the
single-launch step (MIX 64 | 8) against the proposal kernel + log-prob kernel pair
(NGRTD_DZ_MODE=pair), alternating in one process, --rounds times.  One JSON line per round.

    python tools/dz_generic_ab.py [--rounds 3] [--steps 256] [--tune 200]"""
import argparse
import dataclasses
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

PAIRS = (("dispersion", None, ("tau1", "D1")), ("exponential", "exponential", ("tau1", "tau2", "f1")),
         ("piston", "exponential", ("tau1", "tau2", "f1")), ("exp_pist_flow", "exponential", ("tau1", "tau2", "f1", "eta1")))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=256)
    ap.add_argument("--tune", type=int, default=200)
    args = ap.parse_args()
    import torch
    from bench import _dz_time
    from noblegas_rtd_mcmc_amd import workloads as wl
    from noblegas_rtd_mcmc_amd.engine import LogProb
    plans = []
    sel = [x for x in os.environ.get("DZ_AB_PAIRS", "").split(",") if x]   # (A/B scripts: a subset)
    modes = ("single",) if os.environ.get("DZ_AB_SINGLE") else ("single", "pair")
    for m1, m2, pn in PAIRS:
        if sel and (m1 + ("-" + m2 if m2 else "")) not in sel:
            continue
        sp = dataclasses.replace(wl.c4_spec(L=64, N=1200, mod_type1=m1, mod_type2=m2, par_names=pn), jacobian=True)
        th = torch.from_numpy(wl.sample_prior(sp, 2048, np.random.default_rng(34569))).cuda()
        plans.append((m1 + ("-" + m2 if m2 else ""), LogProb(sp, max_walkers=2048), th))
    for r in range(args.rounds):
        res = {"round": r}
        for name, lp, th in plans:
            for mode in modes:
                if mode == "pair":
                    os.environ["NGRTD_DZ_MODE"] = "pair"
                try:
                    res["%s_%s_us" % (name, mode)] = _dz_time(lp, th, True, True, args.tune, args.steps)["us_per_step"]
                finally:
                    os.environ.pop("NGRTD_DZ_MODE", None)
        print(json.dumps(res), flush=True)
    for _, lp, _ in plans:
        lp.close()


if __name__ == "__main__":
    main()
