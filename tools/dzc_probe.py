#!/usr/bin/env python3
"""Per-step time of the lane-chain DEMetropolisZ step (dz_chain_kernel) at the reference's own
run shape -- RTD-only, 1 well, 3 chains, N = 25 256, PyMC3's transformed space -- with the logs
the drop-in's sampler keeps (accepted, lp, accept stat), after 1000 tune steps; NGRTD_DZ_DIAG
selects timing-only variants of the step (wrong results; bits in ngrtd_dzc.hpp).  JSON lines.

    [NGRTD_DZ_DIAG=k] python tools/dzc_probe.py [--tracers 4|1] [--model exponential|exp_pist_flow]
        [--phase draw|tune]"""
import argparse
import dataclasses
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tracers", type=int, default=4)
    ap.add_argument("--model", default="exponential")
    ap.add_argument("--chains", type=int, default=3)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--phase", choices=("draw", "tune"), default="draw",
                    help="time draw-phase steps (after 1000 tune steps) or steps inside the tuning phase")
    args = ap.parse_args()
    import torch
    from noblegas_rtd_mcmc_amd import workloads as wl
    from noblegas_rtd_mcmc_amd.engine import LogProb
    from noblegas_rtd_mcmc_amd.sampler import DeviceDEMetropolisZ
    tr = ("CFC12", "SF6", "H3", "He4_ter") if args.tracers == 4 else ("H3",)
    sv = "123" if args.tracers == 4 else ""
    spec = dataclasses.replace(wl.rtd_only_spec(L=1, N=25256, tracers=tr, mod_type1=args.model, savenum=sv), jacobian=True)
    W = args.chains
    th = torch.from_numpy(wl.test_point(spec, W)).cuda()
    lp = LogProb(spec, max_walkers=W)
    n = args.steps
    s = DeviceDEMetropolisZ(lp, tune_interval=1000, seed=7, transformed=True, per_well=True)
    n_tune = 1000 if args.phase == "draw" else 1000 + 2 * n
    x, l, z = s.start(th, n_tune, 1000 + 2 * n + 1)
    lp.demcz(x, l, 1000, z)
    acc = torch.empty((n, W), dtype=torch.uint8, device="cuda")
    lpl = torch.empty((n, W), dtype=torch.float64, device="cuda")
    arl = torch.empty((n, W), dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    lp.demcz(x, l, n, z, accepted_log=acc, logp_log=lpl, accept_log=arl)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / n
    print(json.dumps({"diag": int(os.environ.get("NGRTD_DZ_DIAG", "0")), "tracers": args.tracers, "model": args.model,
                      "phase": args.phase, "chains": W, "us_per_step": dt * 1e6}))
    lp.close()


if __name__ == "__main__":
    main()
