#!/usr/bin/env python3
"""Batched forward sweep: the tau sweep of
age_modeling_mcmc.prep.py:735-778 -- 10 004 taus x 7 tracers x {exponential, piston}
convolutions over the full 25 256-year input series -- through the drop-in
tracer_conv_integral with array parameters (one ngrtd_conv launch per tracer and model).
Checks sampled results against the CPU oracle and times the oracle on a sample of the
same convolutions (the reference loop does one convolve() per tau).  One JSON line.

    python tools/sweep_bench.py
"""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import pandas as pd
    from noblegas_rtd_mcmc_amd import convolution_integral_utils as conv
    from noblegas_rtd_mcmc_amd import workloads
    from noblegas_rtd_mcmc_amd.spec import J_flux
    from oracle import rtd as orc

    tau_list = np.concatenate(([1], np.arange(2, 10005, 1))).astype(np.float64)      # prep.py:735-736
    tlist = ['CFC11', 'CFC12', 'CFC113', 'SF6', 'He4_ter', 'H3', 'He3']
    J = J_flux(Del=1., rho_r=2700, rho_w=1000, U=3.0, Th=10.0, phi=0.05)
    frames, kws = {}, {}
    for t in tlist:
        s = workloads.atmos_series('H3' if t in ('H3', 'He3') else t)
        vals, idx, _ = s.reference_frame()
        if t == 'He4_ter':
            vals = vals * 0.0
        frames[t] = pd.DataFrame({t: vals}, index=pd.Index(idx.astype(np.int64), name='tau'))
        kws[t] = ({'t_half': 12.34} if t == 'H3' else {'t_half': 12.34, 'rad_accum': '3He'} if t == 'He3'
                  else {'rad_accum': '4He', 'J': J} if t == 'He4_ter' else {})
    res = {}
    # warm-up: builds every series / channel table once (per-process caches)
    for t in tlist:
        c = conv.tracer_conv_integral(C_t=frames[t], t_samp=frames[t].index[-1])
        for mod in ('exponential', 'piston'):
            c.update_pars(tau=tau_list[:8], mod_type=mod, **kws[t])
            c.convolve()
    t0 = time.perf_counter()
    for t in tlist:
        c = conv.tracer_conv_integral(C_t=frames[t], t_samp=frames[t].index[-1])
        for mod in ('exponential', 'piston'):
            c.update_pars(tau=tau_list, mod_type=mod, **kws[t])
            res[(t, mod)] = np.array(c.convolve())
    gpu_s = time.perf_counter() - t0
    n_conv = len(tlist) * 2 * len(tau_list)
    # parity on a sample + CPU oracle timing of the same convolutions
    rng = np.random.default_rng(0)
    worst = 0.0
    t_cpu, n_cpu = 0.0, 0
    for t in tlist:
        f = frames[t]
        for mod in ('exponential', 'piston'):
            for i in rng.choice(len(tau_list), 6, replace=False):
                k = kws[t]
                t1 = time.perf_counter()
                ref = orc.convolve(f[t].to_numpy(), f.index.to_numpy(), f.index[-1], tau_list[i], mod,
                                   lamba=orc.thalf_2_lambda(k['t_half']) if 't_half' in k else 0.0,
                                   rad_accum=k.get('rad_accum', False), J=k.get('J', False))
                t_cpu += time.perf_counter() - t1
                n_cpu += 1
                got = res[(t, mod)][i]
                worst = max(worst, abs(got - ref) / max(abs(ref), 1e-300))
    print(json.dumps({"workload": "prep.py tau sweep: %d taus x %d tracers x {exponential, piston}, N=25256"
                                  % (len(tau_list), len(tlist)),
                      "convolutions": n_conv, "gpu_s": gpu_s, "gpu_conv_per_s": n_conv / gpu_s,
                      "cpu_oracle_conv_per_s_1core": n_cpu / t_cpu,
                      "cpu_oracle_sample": n_cpu, "max_rel_err_vs_oracle": worst}))
    assert worst <= 1e-12, worst


if __name__ == "__main__":
    main()
