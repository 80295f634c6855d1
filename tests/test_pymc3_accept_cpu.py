"""The oracle against the reference's own PyMC3 runs (tests/golden/make_pymc3_accept.py).

PyMC3 3.11.2's DEMetropolisZ records accept = exp(logp(q) - logp(q0)) for every proposal
(step_methods/metropolis.py), in the model's transformed space, and the 22 shipped traces
(age_ens_runs_mcmc/conv_traces/*.netcdf) hold it with every draw.  For an accepted step the
proposal is the next draw, so log(accept) = logp(x_t) - logp(x_{t-1}): the reference's own
transformed-space RTD log-prob differences at N = 25 256 (priors, interval / logodds / log
Jacobians, Student-t over the tracers, every convolution) for the four published models and
the 12 single-tracer runs.  The fixture holds up to 1000 such transitions per trace and one
observation sigma per tracer fitted by the generator (ens_dict.pk, from which the reference
computed it, is not shipped)."""
import numpy as np
import pytest

from golden_specs import pymc3_run_spec, pymc3_runs

RUNS = pymc3_runs()
# run_age_mcmc.py:100-114: perr 0.05 per tracer (PLM6 SF6 10.0); the commented alternative
# dict :104-108 (CFC12 / SF6 0.15, H3 / He4_ter 0.10) is what the exponential-piston run used
PERR = {"CFC12": 0.05, "SF6": 0.05, "H3": 0.05, "He4_ter": 0.05}
PERR_ALT = {"CFC12": 0.15, "SF6": 0.15, "H3": 0.10, "He4_ter": 0.10}


def test_fixture_covers_every_shipped_run():
    """22 runs: 3 wells x (4 single tracers at savenum 0 + the 4-tracer exponential /
    exp_pist_flow / exp_pist_flow-piston at 123) + PLM1's exponential-piston; >= 500 kept
    transitions each."""
    names = {e["name"] for _, e, _ in RUNS}
    assert len(names) == 22
    for w in ("PLM1", "PLM6", "PLM7"):
        for t in ("CFC12", "SF6", "H3", "He4_ter"):
            assert "%s.%s.exponential.0.netcdf" % (w, t) in names
        for m in ("exponential", "exp_pist_flow", "exp_pist_flow-piston"):
            assert "%s.CFC12.SF6.H3.He4_ter.%s.123.netcdf" % (w, m) in names
    assert "PLM1.CFC12.SF6.H3.He4_ter.exponential-piston.123.netcdf" in names
    for _, e, a in RUNS:
        assert a["x0"].shape == a["x1"].shape and a["x0"].shape[0] >= 500 and a["dlogp"].shape[0] == a["x0"].shape[0]
        assert np.isfinite(a["dlogp"]).all()
        assert e["maxres"] <= 1e-9


@pytest.mark.parametrize("key,entry,arr", RUNS, ids=[e["name"][:-7] for _, e, _ in RUNS])
def test_oracle_reproduces_pymc3_accept(key, entry, arr):
    """oracle/vectorized.py's transformed-space log-prob (spec.jacobian) at the trace's two
    states of each sampled transition: logp(x_t) - logp(x_{t-1}) == log(accept[t]) within
    1e-8 (measured ~1e-10) on 48 transitions per run."""
    from oracle.vectorized import log_prob_vec
    spec = pymc3_run_spec(entry)
    n = arr["x0"].shape[0]
    idx = np.linspace(0, n - 1, 48).astype(int)
    lp0 = log_prob_vec(spec, spec.theta_soa(arr["x0"][idx][:, None, :]))
    lp1 = log_prob_vec(spec, spec.theta_soa(arr["x1"][idx][:, None, :]))
    d = lp1 - lp0
    assert np.isfinite(d).all()
    err = np.abs(d - arr["dlogp"][idx])
    assert err.max() <= 1e-8, (entry["name"], err.max())


def test_fitted_sigma_has_the_reference_structure():
    """sigma_k = std(ens_k) + mu_k perr_k (run_age_mcmc_utils.py:353-356) with std(ens_k) a
    property of the well's observation ensemble: the independently fitted sigmas of every run
    of a well imply ONE std per tracer -- the 4-tracer exponential / exp_pist_flow /
    exp_pist_flow-piston runs and the single-tracer CFC12 / SF6 / H3 runs under perr 0.05
    (PLM6 SF6 10.0, run_age_mcmc.py:100-114), PLM1's exponential-piston run under the
    commented perr dict of :104-108 -- within 1e-6 relative, and std >= 0."""
    fit = {e["name"]: (np.array(e["mu"]), np.array(e["sd"]), e["tracers"]) for _, e, _ in RUNS}
    for w in ("PLM1", "PLM6", "PLM7"):
        ref = None
        for name, (mu, sd, trs) in fit.items():
            if not name.startswith(w + ".") or (len(trs) == 1 and trs[0] == "He4_ter"):
                continue       # the single-tracer He4_ter runs used another ensemble (their mu differs)
            alt = "exponential-piston" in name
            perr = np.array([(PERR_ALT if alt else PERR)[t] * (10.0 / 0.05 if (w == "PLM6" and t == "SF6" and not alt)
                                                              else 1.0) for t in trs])
            std = dict(zip(trs, sd - mu * perr))
            for t, v in std.items():
                assert v >= 0, (name, t, v)
                if ref is None or t not in ref:
                    ref = dict(ref or {}, **{t: v})
                else:
                    assert abs(v - ref[t]) <= 1e-6 * abs(ref[t]), (name, t, v, ref[t])
