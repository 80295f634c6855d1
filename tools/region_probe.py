#!/usr/bin/env python3
"""Where a short timed region's time goes (bench.py's N = 1 region, c4 headline plan):
host time until the native K-launch call returns, until the last event completes (spin on
query), until torch.cuda.synchronize returns, and the GPU time between the two events.
Prints one JSON line per (K, rep).
    python tools/region_probe.py [--steps 20,200] [--reps 5] [--warmup 5]"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", default="20,200")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=5)
    args = ap.parse_args()
    import torch
    from noblegas_rtd_mcmc_amd import workloads
    from noblegas_rtd_mcmc_amd.distributed import LogpStepLoop
    from noblegas_rtd_mcmc_amd.engine import LogProb
    dev = torch.device("cuda", 0)
    spec = workloads.c4_spec(L=64, N=1200)
    theta = torch.from_numpy(workloads.sample_prior(spec, 2048, np.random.default_rng(34568))).to(dev)
    lp = LogProb(spec, max_walkers=2048)
    loop = LogpStepLoop(None, 2048, dev)
    fast, fast_n = lp.bind(theta, loop.out), lp.bind_n(theta, loop.out)
    loop.evaluate = lambda out: fast()
    loop.evaluate_n = lambda out, k: fast_n(k)
    for k in [int(s) for s in args.steps.split(",")]:
        for rep in range(args.reps):
            for _ in range(args.warmup):
                loop.step()
            torch.cuda.synchronize()
            ev0 = torch.cuda.Event(enable_timing=True)
            ev1 = torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            ev0.record()
            loop.run(k)
            ev1.record()
            t_l = time.perf_counter()
            while not ev1.query():
                pass
            t_q = time.perf_counter()
            torch.cuda.synchronize()
            t_s = time.perf_counter()
            ev = ev0.elapsed_time(ev1) * 1e3
            print(json.dumps({"steps": k, "rep": rep, "launch_us": (t_l - t0) * 1e6, "spin_us": (t_q - t0) * 1e6,
                              "sync_us": (t_s - t0) * 1e6, "event_us": ev, "event_per_step_us": ev / k}),
                  flush=True)
            # the same region ending in synchronize() alone (bench.py's)
            for _ in range(args.warmup):
                loop.step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            loop.run(k)
            torch.cuda.synchronize()
            t_s = time.perf_counter()
            print(json.dumps({"steps": k, "rep": rep, "plain_sync_us": (t_s - t0) * 1e6}), flush=True)
    lp.close()


if __name__ == "__main__":
    main()
