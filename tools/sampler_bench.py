#!/usr/bin/env python3
"""MCMC sampler throughput on the c4 workload (2048 walkers x 64 wells): walker-steps/s of
the device-resident DE-MC (ngrtd_demc_run: 2 launches per step) and of the torch-op
DEMetropolis loop around the same log-prob kernel.  One JSON line.

    python tools/sampler_bench.py [--steps 200]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--walkers", type=int, default=2048)
    args = ap.parse_args()
    import torch
    from noblegas_rtd_mcmc_amd import workloads
    from noblegas_rtd_mcmc_amd.engine import LogProb
    from noblegas_rtd_mcmc_amd.sampler import DEMetropolis
    W = args.walkers
    spec = workloads.c4_spec(L=64)
    th = workloads.sample_prior(spec, W, np.random.default_rng(34568))
    lp = LogProb(spec, max_walkers=W)
    x = torch.from_numpy(th).cuda()
    lpv = lp(x).clone()
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    d = spec.n_params * spec.n_wells
    lamb = 2.38 / np.sqrt(2 * d)
    lp.demc(x, lpv, 10, lamb, 1e-3, 7, n_accepted=cnt)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    lp.demc(x, lpv, args.steps, lamb, 1e-3, 7, step0=10, n_accepted=cnt)
    torch.cuda.synchronize()
    dev = (time.perf_counter() - t0) / args.steps
    ts = max(20, args.steps // 5)
    DEMetropolis(lambda t: lp(t), seed=3).run(torch.from_numpy(th).cuda(), 5, 0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    DEMetropolis(lambda t: lp(t), seed=3, tune_interval=10 ** 9).run(torch.from_numpy(th).cuda(), ts, 0)
    torch.cuda.synchronize()
    tor = (time.perf_counter() - t0) / ts
    print(json.dumps({"workload": "c4: %d walkers x 64 wells (5 gases CE + 5 tracers RTD, N=1200)" % W,
                      "device_demc": {"us_per_step": dev * 1e6, "walker_steps_per_s": W / dev},
                      "torch_demetropolis": {"us_per_step": tor * 1e6, "walker_steps_per_s": W / tor},
                      "speedup": tor / dev}))


if __name__ == "__main__":
    main()
