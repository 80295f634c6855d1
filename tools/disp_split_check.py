#!/usr/bin/env python3
"""Dispersion age split (theta + RTD waves) vs the RTD wave alone vs the vectorised oracle, at the
c4 shape on the parity tests' 264 walkers (GPU).  Each mode runs in its own process (the library
reads NGRTD_NO_DISP_SPLIT once).  Prints one JSON line per model: max |rel| differences.

    python tools/disp_split_check.py [--models dispersion,exponential-dispersion]
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def spec_of(model):
    from noblegas_rtd_mcmc_amd import workloads as wl
    m1, _, m2 = model.partition("-")
    return wl.c4_spec(L=64, N=1200, mod_type1=m1, mod_type2=m2 or None,
                      par_names=wl.model_par_names(m1, m2 or None, ""))


def run_one(model, out):
    import torch
    from noblegas_rtd_mcmc_amd import workloads as wl
    from noblegas_rtd_mcmc_amd.engine import LogProb
    spec = spec_of(model)
    th = wl.sample_prior(spec, 2048, np.random.default_rng(34568))
    lp = LogProb(spec, max_walkers=2048)
    np.save(out, lp(torch.from_numpy(th).cuda()).cpu().numpy())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default="dispersion,exponential-dispersion")
    ap.add_argument("--one", nargs=2)
    args = ap.parse_args()
    if args.one:
        run_one(*args.one)
        return
    from noblegas_rtd_mcmc_amd import workloads as wl
    from oracle.vectorized import log_prob_vec
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from test_gpu_parity import many_walkers
    tmp = tempfile.mkdtemp()
    for model in args.models.split(","):
        res = {}
        for mode, env in (("split", {}), ("nosplit", {"NGRTD_NO_DISP_SPLIT": "1"})):
            f = os.path.join(tmp, "%s_%s.npy" % (model, mode))
            subprocess.run([sys.executable, __file__, "--one", model, f], check=True, env=dict(os.environ, **env),
                           timeout=300)
            res[mode] = np.load(f)
        spec = spec_of(model)
        th = wl.sample_prior(spec, 2048, np.random.default_rng(34568))
        sel = many_walkers(2048, seed=11)
        ref = log_prob_vec(spec, np.ascontiguousarray(th[:, :, sel]))

        def rel(x, y):
            m = np.isfinite(x) & np.isfinite(y)
            return float(np.max(np.abs(x[m] - y[m]) / np.maximum(np.abs(y[m]), 1e-300))) if m.any() else None
        print(json.dumps({"model": model, "split_vs_nosplit": rel(res["split"], res["nosplit"]),
                          "split_vs_oracle": rel(res["split"][sel], ref), "nosplit_vs_oracle": rel(res["nosplit"][sel], ref),
                          "nan_mismatch": int(np.sum(np.isnan(res["split"]) != np.isnan(res["nosplit"]))),
                          "example": [float(res["split"][0]), float(res["nosplit"][0]), float(ref[0])]}))


if __name__ == "__main__":
    main()
