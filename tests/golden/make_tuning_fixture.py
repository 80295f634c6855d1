#!/usr/bin/env python3
"""Freeze the tuning state of the reference's own PyMC3 DEMetropolisZ chains as a fixture.

Run in the build container only (needs /root/reference):

    python tests/golden/make_tuning_fixture.py

The 22 shipped traces (age_ens_runs_mcmc/conv_traces/*.netcdf, az.to_netcdf at
run_age_mcmc_utils.py:425 after mc.sample(tune=10000, draws=10000, chains=3,
step=DEMetropolisZ(tune='lambda', tune_interval=1000)), :407-417) keep the draw phase only
(discard_tuned_samples): sample_stats/lambda [chain][draw] is then constant per chain -- the
lambda PyMC3's tuning left after 10 000 steps -- and sample_stats/accepted [chain][draw]
gives each chain's draw-phase acceptance.  Read with the package's own netCDF-4 reader
(noblegas_rtd_mcmc_amd.trace.from_netcdf; no code from the files is executed).

Output: tests/golden/ref_tuning.json -- per run: the final lambda, scaling and draw-phase
acceptance of each chain, the number of draws and tuning steps (the trace attributes).
tests/test_gpu_tuning.py compares the device sampler's chains with them."""
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

from noblegas_rtd_mcmc_amd import trace as _trace   # noqa: E402


def _arr(v):
    """(dims, array) pairs of the reader -> the array."""
    return np.asarray(v[1] if isinstance(v, tuple) else v)


def main():
    out = {}
    for path in sorted(glob.glob(os.path.join(TRACES, "*.netcdf"))):
        idd = _trace.from_netcdf(path)
        ss = idd["sample_stats"]
        lam = _arr(ss["lambda"])
        acc = _arr(ss["accepted"]).astype(np.float64)
        sc = _arr(ss["scaling"])
        # lambda is frozen after tuning: one value per chain over the whole draw phase
        if not all(len(np.unique(lam[c])) == 1 for c in range(lam.shape[0])):
            raise SystemExit("%s: lambda varies within the draw phase" % path)
        out[os.path.basename(path)[:-len(".netcdf")]] = {
            "lambda": [float(lam[c, -1]) for c in range(lam.shape[0])],
            "scaling": [float(sc[c, -1]) for c in range(sc.shape[0])],
            "accept_rate": [float(acc[c].mean()) for c in range(acc.shape[0])],
            "chains": int(lam.shape[0]), "draws": int(lam.shape[1]),
            "tuning_steps": int(idd["attrs"].get("tuning_steps", 0))}
    with open(os.path.join(HERE, "ref_tuning.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print(json.dumps({k: (v["lambda"], [round(a, 3) for a in v["accept_rate"]]) for k, v in out.items()}, indent=0))


if __name__ == "__main__":
    main()
