#!/usr/bin/env python3
"""EPM single-launch kernel diagnostics: per-launch time for the c4 EPM workload with the
bench's theta, with every tau' >= 1/2 (no exact-tail lanes), and for the exponential model."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(lp, th, n=50):
    import torch
    x = torch.from_numpy(th).cuda()
    o = torch.empty(th.shape[2], dtype=torch.float64, device="cuda")
    run = lp.bind(x, o)
    for _ in range(5):
        run()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        run()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e6


def main():
    from noblegas_rtd_mcmc_amd import workloads as wl
    from noblegas_rtd_mcmc_amd.engine import LogProb
    out = {}
    for name, m1, m2, pn in (("epm", "exp_pist_flow", None, ("tau1", "eta1")),
                             ("exp", "exponential", None, ("tau1",))):
        spec = wl.c4_spec(L=64, N=1200, mod_type1=m1, mod_type2=m2, par_names=pn)
        th = wl.sample_prior(spec, 2048, np.random.default_rng(34568))
        t0 = time.perf_counter()
        lp = LogProb(spec, max_walkers=2048)
        out[name + "_plan_ms"] = (time.perf_counter() - t0) * 1e3
        out[name + "_info"] = lp.info(2048)
        out[name + "_us"] = timeit(lp, th)
        if name == "epm":
            t = th.copy()
            i = spec.roles.index("tau1")
            t[i] = np.maximum(t[i], 3.0)
            out["epm_no_exact_tail_us"] = timeit(lp, t)
            t2 = th.copy()
            t2[i] = 3.0 + (t2[i] - 1.0) * 0.0   # all units the same tau: uniform head/tail rows
            out["epm_uniform_tau_us"] = timeit(lp, t2)
        lp.close()
    # NGRTD_EPM_DIAG (read at plan creation): skip the head (1), the tail surrogate (2), the
    # exact tails (4) -- wrong results, timing only
    spec = wl.c4_spec(L=64, N=1200, mod_type1="exp_pist_flow", par_names=("tau1", "eta1"))
    th = wl.sample_prior(spec, 2048, np.random.default_rng(34568))
    for d in (1, 2, 4, 3, 7):
        os.environ["NGRTD_EPM_DIAG"] = str(d)
        lp = LogProb(spec, max_walkers=2048)
        out["epm_diag%d_us" % d] = timeit(lp, th)
        lp.close()
    os.environ.pop("NGRTD_EPM_DIAG")
    print(json.dumps(out))


if __name__ == "__main__":
    main()
