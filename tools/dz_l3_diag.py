#!/usr/bin/env python3
"""Diagnostics: device DEMetropolisZ vs the torch restatement at L = 3 (170 walkers per block):
first mismatching step / chain / row of the histories, for each device schedule."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from noblegas_rtd_mcmc_amd import workloads as wl
    from noblegas_rtd_mcmc_amd.engine import LogProb
    from noblegas_rtd_mcmc_amd.sampler import DEMetropolisZ, DeviceDEMetropolisZ
    L = int(os.environ.get("DIAG_L", "3"))
    W = int(os.environ.get("DIAG_W", "200"))
    spec = wl.c4_spec(L=L, N=300)
    th0 = wl.sample_prior(spec, W, np.random.default_rng(5))
    lp = LogProb(spec, max_walkers=W)
    x0 = torch.from_numpy(th0).cuda()
    kw = dict(tune_interval=4, seed=987654321)
    ref = DEMetropolisZ(lambda t: lp(t), **kw).run(x0, tune=12, draws=8)
    for mode, ch in (("fused", "256"), ("fused", "1"), ("pair", "256")):
        os.environ["NGRTD_DZ_MODE"] = mode
        os.environ["NGRTD_DZ_CHUNK"] = ch
        dev = DeviceDEMetropolisZ(lp, **kw).run(x0, tune=12, draws=8)
        s_d, s_r = dev["samples"].cpu().numpy(), ref["samples"].cpu().numpy()
        bad = np.argwhere(~((s_d == s_r) | (np.isnan(s_d) & np.isnan(s_r))))
        lpd, lpr = dev["logp"].cpu().numpy(), ref["logp"].cpu().numpy()
        badl = np.argwhere(~((lpd == lpr) | (np.isnan(lpd) & np.isnan(lpr))))
        print(mode, ch, "sample mismatches", len(bad), bad[:5].tolist(), "logp mismatches", len(badl),
              badl[:5].tolist(), flush=True)
        if len(badl):
            d, w = badl[0]
            print("  logp dev/ref", lpd[d, w], lpr[d, w], flush=True)


if __name__ == "__main__":
    main()
