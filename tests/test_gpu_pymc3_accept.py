"""The HIP log-prob against the reference's own PyMC3 runs (see tests/test_pymc3_accept_cpu.py
and tests/golden/make_pymc3_accept.py): for every shipped trace, the plan of that run (one
well, its tracers on the full series N = 25 256, its model and savenum, PyMC3's transformed
space: the plan adds the transform Jacobians) evaluates both states of every kept accepted
transition in one batched call each; logp(x_t) - logp(x_{t-1}) must equal the trace's
log(accept[t]) within 1e-8 for ALL of them (up to 1000 per run)."""
import numpy as np
import pytest

from golden_specs import pymc3_run_spec, pymc3_runs

pytestmark = pytest.mark.gpu
RUNS = pymc3_runs()


@pytest.mark.parametrize("key,entry,arr", RUNS, ids=[e["name"][:-7] for _, e, _ in RUNS])
def test_hip_reproduces_pymc3_accept(key, entry, arr):
    from noblegas_rtd_mcmc_amd.engine import LogProb
    spec = pymc3_run_spec(entry)
    n = arr["x0"].shape[0]
    lp = LogProb(spec, max_walkers=n)
    try:
        lp0 = lp(spec.theta_soa(arr["x0"][:, None, :]), soa=True)
        lp1 = lp(spec.theta_soa(arr["x1"][:, None, :]), soa=True)
    finally:
        lp.close()
    d = lp1 - lp0
    assert np.isfinite(d).all(), entry["name"]
    err = np.abs(d - arr["dlogp"])
    assert err.max() <= 1e-8, (entry["name"], float(err.max()), int(err.argmax()))
