"""The reference's own series length, N = 25 256 (every published run convolves the whole
C_in_dict: age_ens_runs_mcmc/run_age_mcmc.py:46,209), for the exp_pist_flow models on the
single launch.

The whole EPM channel table (1.24 MB at N = 25 256) does not fit LDS; a plan whose
exp_pist_flow component is tau1 / eta1 under their Uniform priors stages only the rows its
in-support units read (ngrtd.hip epm_window: the first unmasked age is at most
tau1_hi (1 - 1/eta1_hi)), and units outside the support box -- log-prob -inf by their priors,
NaN where the reference's weights are -- read no row past it.  Checked against the
vectorised oracle (which convolves all 25 256 ages, convolution_integral_utils.py:155-340)
with one launch asserted, and at the support's edges against the per-walker oracle with the
exact -inf / NaN pattern."""
import dataclasses

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
N_FULL = 25256


def _close(a, b, rtol=1e-12, atol=1e-9):
    both_nan = np.isnan(a) & np.isnan(b)
    same_inf = np.isinf(a) & np.isinf(b) & (np.sign(a) == np.sign(b))
    with np.errstate(invalid="ignore"):
        return both_nan | same_inf | (np.abs(a - b) <= atol + rtol * np.abs(b))


def _spec(model, variant, L):
    from noblegas_rtd_mcmc_amd import workloads as wl
    m1, _, m2 = model.partition("-")
    sv = "123" if variant.endswith("123") else ""
    if variant.startswith("rtd_only"):
        return wl.rtd_only_spec(L=L, N=N_FULL, mod_type1=m1, mod_type2=m2 or None, savenum=sv)
    spec = wl.c4_spec(L=L, N=N_FULL, mod_type1=m1, mod_type2=m2 or None, par_names=wl.model_par_names(m1, m2 or None, sv))
    return dataclasses.replace(spec, jacobian=variant.endswith("jac"))


def _one_launch(lp, dev):
    lp.ctx.set_profiling(True)
    lp.kernel_stats(reset=True)
    a = lp(dev).cpu().numpy()
    lp.ctx.set_profiling(False)
    ks = lp.kernel_stats(reset=True)
    assert ks["fused"][1] == 1 and ks["rtd"][1] == 0 and ks["unit"][1] == 0, ks
    return a


@pytest.mark.parametrize("model", ["exp_pist_flow", "exp_pist_flow-piston"])
@pytest.mark.parametrize("variant", ["rtd_only_123", "rtd_only", "joint", "joint_123", "joint_jac"])
def test_epm_full_series_single_launch_vs_oracle(model, variant):
    """The published exp_pist_flow models at N = 25 256 in ONE launch: the reference's RTD-only
    4-tracer model (savenum 123 and 0) and the joint CE + 5-tracer model (savenum 0 / 123 /
    with the Jacobians), 512 walkers x 4 wells drawn from the priors, vs the vectorised oracle
    on 96 walkers; determinism and device == host staging."""
    import torch
    from noblegas_rtd_mcmc_amd import workloads as wl
    from noblegas_rtd_mcmc_amd.engine import LogProb
    spec = _spec(model, variant, L=4)
    W = 512
    th = wl.sample_prior(spec, W, np.random.default_rng(2526))
    lp = LogProb(spec, max_walkers=W)
    dev = torch.from_numpy(th).cuda()
    a = _one_launch(lp, dev)
    assert np.array_equal(a, lp(dev).cpu().numpy()) and np.array_equal(a, lp(th, soa=True))
    sel = sorted(set(range(64)) | set(np.random.default_rng(3).choice(W, 32, replace=False).tolist()))
    from oracle.vectorized import log_prob_vec
    ref = log_prob_vec(spec, np.ascontiguousarray(th[:, :, sel]))
    ok = _close(a[sel], ref)
    assert ok.all(), (np.array(sel)[~ok], a[sel][~ok], ref[~ok])
    assert np.isfinite(a).mean() > 0.5
    lp.close()


@pytest.mark.parametrize("model", ["exp_pist_flow", "exp_pist_flow-piston"])
def test_epm_full_series_window_edges(model):
    """Units at and beyond the support box of the staged window (tau1 at 1 and 1000 and
    beyond, tau1 (1 - 1/eta1) past the series end -- every age masked, NaN --, eta1 at 1 and 5
    and beyond, tau1 or eta1 0 / negative / NaN, thalf_cfc outside [0, 1], the piston tau2
    across the table) vs the per-walker oracle: values within the parity bar and the
    oracle's -inf / NaN pattern exactly."""
    import oracle.models as om
    from noblegas_rtd_mcmc_amd import workloads as wl
    from noblegas_rtd_mcmc_amd.engine import LogProb
    spec = _spec(model, "rtd_only_123", L=1)
    R = {r: i for i, r in enumerate(spec.roles)}
    W = 64
    th = wl.sample_prior(spec, W, np.random.default_rng(9))
    tau = [1.0, 1000.0, 999.999, 1000.5, 5000.0, 40000.0, 0.5, 0.0, -3.0, np.nan, 200.0, 200.0, 200.0, 200.0,
           200.0, 200.0, 32000.0, 800.0]
    eta = [1.0, 5.0, 5.0, 5.0, 5.0, 2.0, 1.0, 2.0, 2.0, 2.0, 0.5, 6.0, 1e-3, np.nan, 5.0 - 1e-12, 1.0 + 1e-12, 1.0, 1.0]
    for w, (t, e) in enumerate(zip(tau, eta)):
        th[R["tau1"], 0, w] = t
        th[R["eta1"], 0, w] = e
    th[R["thalf_cfc_beta"], 0, 18:22] = [-0.1, 1.5, 0.0, 1.0]
    if "tau2" in R:
        th[R["tau2"], 0, 22:30] = [50.0, 400.0, 499.5, 1500.0, 15000.0, 25255.0, 30000.0, 1.0]
    lp = LogProb(spec, max_walkers=W)
    got = lp(th, soa=True)
    ref = om.log_prob(spec, th)
    ok = _close(got, ref)
    assert ok.all(), (np.nonzero(~ok)[0], got[~ok], ref[~ok])
    assert np.isnan(ref).any() and np.isneginf(ref).any() and np.isfinite(ref).sum() > 20
    lp.close()


@pytest.mark.parametrize("model", ["dispersion", "dispersion-piston", "exponential-dispersion"])
@pytest.mark.parametrize("variant", ["rtd_only_123", "joint"])
def test_dispersion_full_series_single_launch_vs_oracle(model, variant):
    """The dispersion models at N = 25 256 in ONE launch (the generic instances read the per-age
    operands with scalar loads: nothing of the series is staged in LDS, any N), 512 walkers x
    4 wells from the priors, vs the vectorised oracle on 96 walkers; determinism."""
    import torch
    from noblegas_rtd_mcmc_amd import workloads as wl
    from noblegas_rtd_mcmc_amd.engine import LogProb
    spec = _spec(model, variant, L=4)
    W = 512
    th = wl.sample_prior(spec, W, np.random.default_rng(2527))
    lp = LogProb(spec, max_walkers=W)
    dev = torch.from_numpy(th).cuda()
    a = _one_launch(lp, dev)
    assert np.array_equal(a, lp(dev).cpu().numpy())
    sel = sorted(set(range(64)) | set(np.random.default_rng(4).choice(W, 32, replace=False).tolist()))
    from oracle.vectorized import log_prob_vec
    ref = log_prob_vec(spec, np.ascontiguousarray(th[:, :, sel]))
    ok = _close(a[sel], ref)
    assert ok.all(), (np.array(sel)[~ok], a[sel][~ok], ref[~ok])
    assert np.isfinite(a).mean() > 0.5
    lp.close()
