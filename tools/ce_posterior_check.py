#!/usr/bin/env python3
"""CE posterior of PLM1 / PLM6 / PLM7 three ways, against the reference's summaries
(ng_interp/ng_opt<well>.csv): (1) importance sampling from the prior (exact up to Monte-Carlo
error: the posterior moments as self-normalised weighted prior moments, the weights being the
GPU log-likelihood, ngrtd_logp_units of a likelihood-only plan); (2) the device
DEMetropolisZ, per-well chains, PyMC3's transformed space; (3) the same in the natural space.
Prints one JSON object per well and method.

    python tools/ce_posterior_check.py [--is-draws 2^26] [--chains 1024] [--tune 10000] [--draws 20000]
"""
import argparse
import dataclasses
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def ref_summary(well):
    import csv
    with open(os.path.join(REPO, "tests", "golden", "ref_summaries", "ng_opt%s.csv" % well)) as f:
        rows = list(csv.reader(f))
    return {r[0]: {k: float(v) for k, v in zip(rows[0][1:], r[1:])} for r in rows[1:]}


def derived(th, c, l, xp):
    """Every summary variable of ng_opt*.csv from theta rows [6][...] of well l."""
    Emin = float(c.E_min[l])
    v = {"Ae_beta": th[0], "F_beta": th[1], "E_beta": th[2], "m": th[3], "b_beta": th[4], "nu_": th[5]}
    v["Ae"] = 10 ** (v["Ae_beta"] * (c.logA_max - c.logA_min) + c.logA_min)
    v["F"] = 10 ** (v["F_beta"] * (c.logF_max - c.logF_min) + c.logF_min)
    v["E"] = v["E_beta"] * (c.E_max - Emin) + Emin
    v["b"] = v["b_beta"] * (c.b_max - c.b_min) + c.b_min
    v["T"] = (v["E"] - v["b"]) / v["m"]
    v["nu"] = v["nu_"] * (c.nu_max - c.nu_min) + c.nu_min
    return v


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--is-draws", type=int, default=1 << 26)
    ap.add_argument("--chains", type=int, default=512)
    ap.add_argument("--tune", type=int, default=10000)
    ap.add_argument("--draws", type=int, default=50000)
    ap.add_argument("--start", choices=("test_point", "prior"), default="test_point")
    ap.add_argument("--thin", type=int, default=10)
    args = ap.parse_args()
    import torch
    from noblegas_rtd_mcmc_amd.engine import LogProb
    from noblegas_rtd_mcmc_amd.noble_gas_mcmc import CEModel
    from noblegas_rtd_mcmc_amd.sampler import sample_model
    from noblegas_rtd_mcmc_amd.workloads import field_data, sample_prior
    wells = ["PLM1", "PLM6", "PLM7"]
    m = CEModel(field_data()["obs"], wells, max_walkers=args.chains)
    spec, c = m.spec, m.spec.ce
    L = len(wells)
    out = []
    # (1) importance sampling: prior draws, weights = exp(log-likelihood)
    chunk = 1 << 21
    like = LogProb(dataclasses.replace(spec, include_prior=False), max_walkers=chunk)
    rng = np.random.default_rng(2024)
    acc = None
    t0 = time.time()
    for i in range(0, args.is_draws, chunk):
        th = torch.from_numpy(sample_prior(spec, chunk, rng)).cuda()
        ll = like.units(th)                                     # [L][chunk]
        for l in range(L):
            v = derived(th[:, l], c, l, torch)
            w = ll[l]
            if acc is None:
                acc = [dict(lmax=-np.inf, s0=0.0, s1={}, s2={}, n_eff2=0.0) for _ in range(L)]
            a = acc[l]
            lm = float(torch.nan_to_num(w, nan=-np.inf).max())
            if lm > a["lmax"]:                                   # rescale the running sums
                f = np.exp(a["lmax"] - lm) if np.isfinite(a["lmax"]) else 0.0
                a["s0"] *= f
                a["n_eff2"] *= f * f
                for k in a["s1"]:
                    a["s1"][k] *= f
                    a["s2"][k] *= f
                a["lmax"] = lm
            ww = torch.exp(torch.nan_to_num(w, nan=-np.inf) - a["lmax"])
            a["s0"] += float(ww.sum())
            a["n_eff2"] += float((ww * ww).sum())
            for k, x in v.items():
                x = torch.nan_to_num(x)
                a["s1"][k] = a["s1"].get(k, 0.0) + float((ww * x).sum())
                a["s2"][k] = a["s2"].get(k, 0.0) + float((ww * x * x).sum())
    for l, well in enumerate(wells):
        a = acc[l]
        ref = ref_summary(well)
        res = {}
        for k in ref:
            mu = a["s1"][k] / a["s0"]
            sd = np.sqrt(max(a["s2"][k] / a["s0"] - mu * mu, 0.0))
            res[k] = {"mean": mu, "sd": sd, "ref_mean": ref[k]["mean"], "ref_sd": ref[k]["sd"],
                      "ref_mcse_mean": ref[k]["mcse_mean"], "ref_mcse_sd": ref[k]["mcse_sd"]}
        out.append({"well": well, "method": "importance sampling from the prior", "draws": args.is_draws,
                    "ess": a["s0"] ** 2 / a["n_eff2"], "seconds": time.time() - t0, "vars": res})
        print(json.dumps(out[-1]), flush=True)
    like.close()
    # (2), (3) the device DEMetropolisZ, per-well chains
    for space in ("transformed", "natural"):
        if args.start == "prior":
            x0 = torch.from_numpy(sample_prior(spec, args.chains, np.random.default_rng(123423))).cuda()
        else:   # model.test_point (the prior means), every chain: PyMC3's start for DEMetropolisZ
            tp = [c.beta_Ae[0] / sum(c.beta_Ae), c.beta_F[0] / sum(c.beta_F), c.beta_E[0] / sum(c.beta_E), c.m_mu,
                  c.beta_b[0] / sum(c.beta_b), c.beta_nu[0] / sum(c.beta_nu)]
            x0 = torch.tensor(tp, dtype=torch.float64, device="cuda")[:, None, None].expand(6, L, args.chains).contiguous()
        t0 = time.time()
        r = sample_model(spec, args.chains, 0, x0, args.tune, args.draws, seed=123423, tune_interval=5000,
                         space=space)
        s = r["samples"][::args.thin]                             # [D, 6, L, W]
        for l, well in enumerate(wells):
            ref = ref_summary(well)
            v = derived(s[:, :, l].permute(1, 0, 2), c, l, torch)  # [6][D][W] -> [D][W] per var
            res = {}
            for k in ref:
                x = v[k]
                cm, cs = x.mean(0), x.std(0)
                res[k] = {"mean": float(x.mean()), "sd": float(x.std()),
                          "mcse_mean": float(cm.std()) / np.sqrt(args.chains),
                          "mcse_sd": float(cs.std()) / np.sqrt(args.chains),
                          "ref_mean": ref[k]["mean"], "ref_sd": ref[k]["sd"]}
            out.append({"well": well, "method": "device DEMetropolisZ, per-well chains, %s space, start %s"
                                                % (space, args.start),
                        "chains": args.chains, "tune": args.tune, "draws": args.draws, "thin": args.thin,
                        "accept_rate": r["accept_rate"], "seconds": time.time() - t0, "vars": res})
            print(json.dumps(out[-1]), flush=True)
        del r, s


if __name__ == "__main__":
    main()
