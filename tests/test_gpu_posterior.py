"""The device DEMetropolisZ's posteriors against the reference's own (GPU).

For every one of the 22 shipped conv_traces runs (tests/golden/ref_posteriors.json: the
reference's posterior summaries from its PyMC3 runs; tests/golden/pymc3_accept_fit.json: the
run's observations, fitted sigma and tau1 bounds) the drop-in
conv_mcmc(...).sample_mcmc() is run with the reference's schedule (run_age_mcmc_utils.py:323-336:
tune 10 000, draws 10 000, tune_interval 1000, DEMetropolisZ in PyMC3's transformed space,
PyMC3's test_point start) on 48 independent chains, seed fixed, and each sampled variable is
checked three ways:

  * the pooled mean against the reference's: |z| <= 5, z = difference / hypot(se_ours, se_ref),
    se_ours from the spread of our 48 chain means (independent chains: honest under
    multimodality), se_ref = max(batch-means se over the reference's 3 chains, their
    between-chain se);
  * the median of our chain means within 0.5 reference posterior sd of the reference's mean
    (robust to the few chains that settle in the exp_pist_flow posteriors' second mode,
    eta1 ~ 4, tau1 ~ 40, which the reference's 3 chains never visited);
  * the acceptance rate within 0.12 of the reference's (3 chains, draws only).

This is a statistical check, not a parity claim: the log-prob parity is pinned to 1e-8 by
test_gpu_pymc3_accept.py.  Measured (round 5, profiles/r05_posterior_compare.json): max |z| 3.75,
max median offset 0.38 sd, max acceptance difference 0.096."""
import json
import os
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
import posterior_compare as pc  # noqa: E402

RUNS = pc.reference_runs()


@pytest.fixture(scope="module")
def c_in():
    from noblegas_rtd_mcmc_amd import workloads as wl
    return wl.c_in_dict()


# every run's comparison, kept for the pooled tuning test at the end of the module
_DONE = {}


@pytest.mark.parametrize("name", sorted(RUNS), ids=lambda n: n[:-7])
def test_posterior_matches_reference(name, c_in):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    e, r = RUNS[name]
    res = pc.compare_run(e, r, chains=48, C_in=c_in)
    _DONE[name] = res
    bad = []
    for v, s in res["vars"].items():
        if not abs(s["z_between"]) <= 5.0:
            bad.append((v, "z", s["z_between"]))
        if not abs(s["chain_means_q"][1] - s["ref_mean"]) <= 0.5 * s["ref_sd"]:
            bad.append((v, "median", s["chain_means_q"][1], s["ref_mean"], s["ref_sd"]))
    if r["accept_rate"] is not None and not abs(res["accept_rate"] - r["accept_rate"]) <= 0.12:
        bad.append(("accept", res["accept_rate"], r["accept_rate"]))
    assert not bad, json.dumps(bad)


def _frac_rank(x, sample):
    """Mid-rank of x among the sample, in [0, 1] (ties count half)."""
    import numpy as np
    a = np.asarray(sample)
    return (float((a < x).sum()) + 0.5 * float((a == x).sum())) / a.size


def test_tuning_matches_reference_chains(c_in):
    """The tuning rule against the reference's own chains (tests/golden/ref_tuning.json, made by
    tests/golden/make_tuning_fixture.py from the 22 traces' sample_stats): PyMC3's 'lambda'
    tuning (run_age_mcmc_utils.py:412-417: tune_interval 1000 over 10 000 tune steps) leaves
    every chain with lambda_0 = 2.38 / sqrt(2 ndim) times a product of PyMC3's tune() factors,
    and each reference chain is one draw of that final lambda (and of its draw-phase
    acceptance).  Pooled over the 66 reference chains, their mid-ranks among our 48 chains of
    the same run are uniform if the tuning matches: their mean lies in [0.3, 0.7], and at most
    8 of them (12 %; 2/49 = 4 % expected) fall outside our chains' [min, max] -- a wrong rule
    (no tuning, scaling tuned instead of lambda, other factors) moves whole runs out."""
    import json
    import numpy as np
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    tun = json.load(open(os.path.join(REPO, "tests", "golden", "ref_tuning.json")))
    ranks = {"lambda": [], "accept": []}
    out = {"lambda": 0, "accept": 0}
    for name in sorted(RUNS):
        res = _DONE.get(name)
        if res is None:
            e, r = RUNS[name]
            res = _DONE[name] = pc.compare_run(e, r, chains=48, C_in=c_in)
        t = tun[name[:-len(".netcdf")]]
        for key, ref, dev in (("lambda", t["lambda"], res["lambda"]), ("accept", t["accept_rate"], res["chain_accept"])):
            for x in ref:
                ranks[key].append(_frac_rank(x, dev))
                out[key] += int(x < min(dev) or x > max(dev))
    summary = {k: {"mean_rank": float(np.mean(v)), "outside": out[k], "n": len(v)} for k, v in ranks.items()}
    if os.path.isdir(os.path.join(REPO, "gpurun_out")):      # the measured ranks, for DESIGN.md §5.1
        with open(os.path.join(REPO, "gpurun_out", "tuning_ranks.json"), "w") as f:
            json.dump({"summary": summary, "ranks": ranks}, f)
    for k, v in summary.items():
        assert v["n"] == 66 and 0.3 <= v["mean_rank"] <= 0.7 and v["outside"] <= 8, summary
