#!/usr/bin/env python3
"""HIP plans against the reference's PyMC3 acceptance statistics (GPU), the numbers DESIGN.md
quotes (tests/test_gpu_pymc3_accept.py asserts <= 1e-8):

    python tools/accept_residuals.py

per shipped run: transitions, max and RMS of |logp(x_t) - logp(x_{t-1}) - log(accept[t])| for
the run's plan (PyMC3's transformed space, N = 25 256), the kernel kind the plan ran (one
launch or the multi-kernel path) and its per-launch time.  One JSON line."""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    from golden_specs import pymc3_run_spec, pymc3_runs
    from noblegas_rtd_mcmc_amd.engine import LogProb
    out = {}
    for key, e, arr in pymc3_runs():
        spec = pymc3_run_spec(e)
        n = arr["x0"].shape[0]
        lp = LogProb(spec, max_walkers=n)
        lp.ctx.set_profiling(True)
        lp.kernel_stats(reset=True)
        lp0 = lp(spec.theta_soa(arr["x0"][:, None, :]), soa=True)
        lp1 = lp(spec.theta_soa(arr["x1"][:, None, :]), soa=True)
        lp.ctx.set_profiling(False)
        ks = lp.kernel_stats(reset=True)
        lp.close()
        err = np.abs(lp1 - lp0 - arr["dlogp"])
        out[e["name"][:-7]] = {"transitions": int(n), "max_abs": float(err.max()), "rms": float(np.sqrt(np.mean(err ** 2))),
                               "single_launch": ks["fused"][1] == 2 and ks["rtd"][1] == 0,
                               "launch_ms": ks["fused"][0] / max(ks["fused"][1], 1) if ks["fused"][1] else None}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
