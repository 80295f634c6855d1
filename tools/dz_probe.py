#!/usr/bin/env python3
"""Device DEMetropolisZ step timing at c4 (2048 chains x 64 wells), per-launch HIP events:
the single-launch step (NGRTD_DZ_DIAG selects timing-only variants, wrong results), and
the plain log-prob on the state and on natural-space-noise proposals of it.  JSON line.

    [NGRTD_DZ_DIAG=k] [DZ_JAC=1] [DZ_PW=0] [DZ_MODEL=bmm|epm|epm_piston] python tools/dz_probe.py

DZ_PW=0: one chain per walker over its wells (default: per-well chains)."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def ev_time(lp, fn, n=40):
    import torch
    fn()
    torch.cuda.synchronize()
    lp.ctx.set_profiling(True)
    lp.kernel_stats(reset=True)
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    ks = lp.kernel_stats(reset=True)
    lp.ctx.set_profiling(False)
    return ks["fused"][0] * 1e3 / max(ks["fused"][1], 1)


def main():
    import dataclasses
    import torch
    from noblegas_rtd_mcmc_amd import workloads
    from noblegas_rtd_mcmc_amd.engine import LogProb
    from noblegas_rtd_mcmc_amd.sampler import DeviceDEMetropolisZ, Transform
    W = 2048
    # DZ_MODEL: the published RTD models on the same shape (exponential-piston BMM,
    # exp_pist_flow, exp_pist_flow-piston BMM); default the exponential c4 workload
    models = {"bmm": dict(mod_type1="exponential", mod_type2="piston", par_names=("tau1", "tau2", "f1")),
              "epm": dict(mod_type1="exp_pist_flow", par_names=("tau1", "eta1")),
              "epm_piston": dict(mod_type1="exp_pist_flow", mod_type2="piston",
                                 par_names=("tau1", "tau2", "f1", "eta1"))}
    model = os.environ.get("DZ_MODEL", "")
    spec = workloads.c4_spec(L=64, **models.get(model, {}))
    jac = bool(os.environ.get("DZ_JAC"))
    if jac:
        spec = dataclasses.replace(spec, jacobian=True)
    x0 = torch.from_numpy(workloads.sample_prior(spec, W, np.random.default_rng(34568))).cuda()
    lp = LogProb(spec, max_walkers=W)
    pw = os.environ.get("DZ_PW", "1") != "0"
    out = {"diag": os.environ.get("NGRTD_DZ_DIAG", "0"), "jacobian": jac, "model": model or "exponential",
           "per_well": pw}
    o = torch.empty(W, dtype=torch.float64, device="cuda")
    out["logp_state_us"] = ev_time(lp, lambda: lp(x0, out=o))
    g = torch.Generator(device="cuda").manual_seed(1)
    noise = (2 * torch.rand(x0.shape, generator=g, device="cuda", dtype=torch.float64) - 1) * 1e-3
    if jac:
        tf = Transform.from_spec(spec)
        xn = tf.backward(tf.forward(x0) + noise).contiguous()
    else:
        xn = (x0 + noise).contiguous()
    out["logp_noisy_us"] = ev_time(lp, lambda: lp(xn, out=o))
    s = DeviceDEMetropolisZ(lp, seed=7, tune=None, per_well=pw)
    x, l, z = s.start(x0, 0, 400)
    lp.demcz(x, l, 10, z)
    # one launch runs K steps (NGRTD_DZ_CHUNK caps it): per-step time = launch time / K
    K = 32
    out["dz_step_us"] = ev_time(lp, lambda: lp.demcz(x, l, K, z), n=8) / K
    print(json.dumps(out))


if __name__ == "__main__":
    main()
