#!/usr/bin/env python3
"""Per-kernel device time of variants of the c4 workload (GPU; HIP events on the launch
stream).  Separates the RTD matrix-core phase from the CE / likelihood / prior epilogue.

    python tools/kernel_timing.py [--steps 100]
"""
import argparse
import dataclasses
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--walkers", type=int, default=2048)
    ap.add_argument("--wells", type=int, default=64)
    args = ap.parse_args()
    import torch
    from noblegas_rtd_mcmc_amd import workloads
    from noblegas_rtd_mcmc_amd.engine import LogProb
    from noblegas_rtd_mcmc_amd.spec import ModelSpec

    W, L = args.walkers, args.wells
    base = workloads.c4_spec(L=L)
    variants = {
        "joint": base,
        "joint_noprior": dataclasses.replace(base, include_prior=False, roles=[]),
        "joint_prioronly": dataclasses.replace(base, include_like=False, roles=[]),
        "rtd_only": ModelSpec(n_wells=L, rtd=base.rtd),
        "ce_only": ModelSpec(n_wells=L, ce=base.ce),
    }
    out = {}
    for name, spec in variants.items():
        th = torch.from_numpy(workloads.sample_prior(spec, W, np.random.default_rng(1))).cuda()
        lp = LogProb(spec, max_walkers=W)
        import time
        out_t = torch.empty(W, dtype=torch.float64, device=th.device)
        for _ in range(5):
            lp(th, out=out_t)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            lp(th, out=out_t)
        torch.cuda.synchronize()
        wall_off = (time.perf_counter() - t0) / args.steps * 1e6
        lp.ctx.set_profiling(True)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            lp(th, out=out_t)
        torch.cuda.synchronize()
        wall_on = (time.perf_counter() - t0) / args.steps * 1e6
        lp.kernel_stats(reset=True)
        lp.kernel_stats(reset=True)
        for _ in range(args.steps):
            lp(th)
        torch.cuda.synchronize()
        ks = lp.kernel_stats(reset=True)
        if spec.rtd is not None:
            for _ in range(args.steps):
                lp.forward(th)
            torch.cuda.synchronize()
            kf = lp.kernel_stats(reset=True)
        else:
            kf = {}
        lp.ctx.set_profiling(False)
        out[name] = {"wall_us_events_off": wall_off, "wall_us_events_on": wall_on, "logp_us": {k: 1e3 * v[0] / max(v[1], 1) for k, v in ks.items() if v[1]},
                     "forward_us": {k: 1e3 * v[0] / max(v[1], 1) for k, v in kf.items() if v[1]}}
        lp.close()
        print(name, json.dumps(out[name]), flush=True)


if __name__ == "__main__":
    main()
