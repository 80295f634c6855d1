#!/usr/bin/env python3
"""The device DEMetropolisZ against the reference's own published posteriors (GPU):

    python tools/posterior_compare.py [--chains 48] [--runs SUBSTR,...]

For every shipped run (tests/golden/ref_posteriors.json: the 22 conv_traces summaries;
tests/golden/pymc3_accept_fit.json: its mu, fitted sigma and tau1 bounds) the drop-in
conv_mcmc(...).sample_mcmc() with the reference's schedule (tune 10 000, draws 10 000,
tune_interval 1000, PyMC3's transformed space) but --chains independent chains, then per
sampled variable: our mean / sd / quantiles, the z-score of the mean difference against the
two Monte-Carlo errors (ours: between our independent chains; the reference's: batch means
over its 3 chains) and the reference's between-chain spread.  One JSON line per run."""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def reference_runs():
    """{name: (fit entry, reference posterior summary)} for the shipped runs."""
    gold = os.path.join(REPO, "tests", "golden")
    fit = {e["name"]: e for e in json.load(open(os.path.join(gold, "pymc3_accept_fit.json"))).values()}
    ref = json.load(open(os.path.join(gold, "ref_posteriors.json")))
    return {name: (fit[name], ref[name]) for name in sorted(ref)}


def compare_run(e, r, chains=48, tune=10000, draws=10000, start="test_point", seed=123423, C_in=None):
    """Sample one reference run (fit entry e) with the drop-in conv_mcmc and summarise it against
    the reference's posterior summary r (see the module docstring)."""
    from noblegas_rtd_mcmc_amd import workloads as wl
    from noblegas_rtd_mcmc_amd.run_age_mcmc_utils import conv_mcmc
    C_in = C_in if C_in is not None else wl.c_in_dict()
    sv = tuple(int(c) for c in e["savenum"] if c in "123")
    perr = wl.OBS_PERR_ALT if (e["mod1"] == "exponential" and e["mod2"] == "piston") else None
    okw, ckw, pkw = wl.reference_run_kwargs(e["well"], e["tracers"], e["mod1"], e["mod2"] or False, sv or (0,),
                                            e["mu"], e["sd"], perr=perr, tau1=e["tau1"], C_in=C_in)
    mc = conv_mcmc(e["well"], list(e["tracers"]), okw, ckw, pkw, "", e["savenum"], max_walkers=chains)
    try:
        out = mc.sample_mcmc(chains=chains, tune=tune, draws=draws, seed=seed, tune_interval=1000, start=start)
    finally:
        mc._lp.close()
    res = {"run": e["name"][:-7], "chains": chains, "start": start, "accept_rate": float(out["accept_rate"]),
           "ref_accept_rate": r["accept_rate"], "sample_s": float(out["sampling_time"]), "vars": {}}
    # the tuning state each chain ends with (lambda frozen after tune steps) and its draw-phase
    # acceptance: compared with the reference's chains (tests/golden/ref_tuning.json)
    res["lambda"] = [float(x) for x in np.asarray(out["lamb"], dtype=np.float64).reshape(-1)]
    res["chain_accept"] = [float(x) for x in np.asarray(out["accepted"], dtype=np.float64).reshape(draws, -1).mean(axis=0)]
    for v, rv in r["vars"].items():
        a = np.asarray(out["posterior"][v], dtype=np.float64)       # [chain][draw]
        cm = a.mean(axis=1)
        se_ours = float(cm.std(ddof=1) / np.sqrt(cm.size))
        se = float(np.hypot(se_ours, rv["se_batch"]))
        rcm = np.array(rv["chain_means"])
        se_ref = max(rv["se_batch"], float(rcm.std(ddof=1) / np.sqrt(rcm.size)))
        res["vars"][v] = {"mean": float(a.mean()), "ref_mean": rv["mean"], "sd": float(a.std(ddof=1)), "ref_sd": rv["sd"],
                          "chain_means_q": [float(np.quantile(cm, q)) for q in (0.0, 0.5, 1.0)],
                          "z_between": float((a.mean() - rv["mean"]) / np.hypot(se_ours, se_ref)),
                          "q05": float(np.quantile(a, 0.05)), "ref_q05": rv["q05"],
                          "q95": float(np.quantile(a, 0.95)), "ref_q95": rv["q95"],
                          "se_ours": se_ours, "se_ref_batch": rv["se_batch"],
                          "ref_chain_spread": float(rcm.max() - rcm.min()),
                          "z": float((a.mean() - rv["mean"]) / se) if se > 0 else None}
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chains", type=int, default=48)
    ap.add_argument("--runs", default="")
    ap.add_argument("--tune", type=int, default=10000)
    ap.add_argument("--draws", type=int, default=10000)
    ap.add_argument("--start", default="test_point", choices=("test_point", "prior"))
    args = ap.parse_args()
    from noblegas_rtd_mcmc_amd import workloads as wl
    C_in = wl.c_in_dict()
    sel = [s for s in args.runs.split(",") if s]
    for name, (e, r) in reference_runs().items():
        if sel and not any(s in name for s in sel):
            continue
        res = compare_run(e, r, args.chains, args.tune, args.draws, args.start, C_in=C_in)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
