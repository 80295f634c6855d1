#!/usr/bin/env python3
"""DZ step launch sequence for a kernel trace: plain log-probs, single-step calls (no
in-kernel append) and one multi-step call, each group separated by a synchronisation."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from noblegas_rtd_mcmc_amd import workloads
    from noblegas_rtd_mcmc_amd.engine import LogProb
    from noblegas_rtd_mcmc_amd.sampler import DeviceDEMetropolisZ
    W = 2048
    spec = workloads.c4_spec(L=64)
    x0 = torch.from_numpy(workloads.sample_prior(spec, W, np.random.default_rng(34568))).cuda()
    lp = LogProb(spec, max_walkers=W)
    out = torch.empty(W, dtype=torch.float64, device="cuda")
    for _ in range(5):
        lp(x0, out=out)
    torch.cuda.synchronize()
    s = DeviceDEMetropolisZ(lp, seed=7, tune=None)
    x, l, z = s.start(x0, 0, 64)
    for _ in range(10):
        lp.demcz(x, l, 1, z)
        torch.cuda.synchronize()
    lp.demcz(x, l, 20, z)
    torch.cuda.synchronize()
    print("ok")


if __name__ == "__main__":
    main()
