#!/usr/bin/env python3
"""Freeze the posterior summaries of the reference's own published runs as a fixture.

Run in the build container only (needs /root/reference):

    python tests/golden/make_ref_posteriors.py

For each of the 22 shipped traces (age_ens_runs_mcmc/conv_traces/*.netcdf: PyMC3
DEMetropolisZ, 3 chains x 10 000 draws after 10 000 tuning steps, run_age_mcmc_utils.py:407-429)
and each sampled variable (natural space, as the trace stores it): the mean, the standard
deviation, the 5 / 50 / 95 % quantiles, the per-chain means, and the Monte-Carlo standard error
of the mean by batch means (batches of 500 draws within each chain: 60 batches).  The
acceptance rate over the draws is kept too.  Output: tests/golden/ref_posteriors.json (the
sampler's statistical pin, tests/test_gpu_pymc3_accept.py)."""
import glob
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, REPO)
REF = os.environ.get("NGRTD_REFERENCE", "/root/reference")
TRACES = os.path.join(REF, "age_ens_runs_mcmc", "conv_traces")
BATCH = 500

from noblegas_rtd_mcmc_amd import trace as _trace   # noqa: E402

VARS = ("tau1", "nu_", "tau2", "f1", "eta1", "J", "thalf_cfc_", "lamsf6")


def summarise(a):
    a = np.asarray(a, dtype=np.float64)                      # [chain][draw]
    nb = a.shape[1] // BATCH
    bm = a[:, :nb * BATCH].reshape(a.shape[0], nb, BATCH).mean(axis=2).ravel()
    return {"mean": float(a.mean()), "sd": float(a.std(ddof=1)),
            "q05": float(np.quantile(a, 0.05)), "q50": float(np.quantile(a, 0.5)), "q95": float(np.quantile(a, 0.95)),
            "chain_means": [float(v) for v in a.mean(axis=1)],
            "se_batch": float(bm.std(ddof=1) / np.sqrt(bm.size)), "n_batches": int(bm.size)}


def main():
    out = {}
    for p in sorted(glob.glob(os.path.join(TRACES, "*.netcdf"))):
        t = _trace.from_netcdf(p)
        post = t["posterior"]
        acc = np.asarray(t["sample_stats"]["accepted"][1], dtype=np.float64)
        e = {"accept_rate": float(acc.mean()), "vars": {}}
        for v in VARS:
            if v in post:
                e["vars"][v] = summarise(post[v][1])
        out[os.path.basename(p)] = e
        print(os.path.basename(p), {v: round(s["mean"], 4) for v, s in e["vars"].items()})
    with open(os.path.join(HERE, "ref_posteriors.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
