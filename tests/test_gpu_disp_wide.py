"""Small-ensemble dispersion plans (ngrtd.hip disp_wide_plan, ngrtd_kernels.hpp disp_wide_kernel):
the dispersion component's age sum (convolution_integral_utils.py:192-196) runs across the
lanes of its own kernel -- the reference's own runs are 1 well x 3 chains at N = 25 256
(run_age_mcmc.py:209, run_age_mcmc_utils.py:412-417), where one lane per unit left the chip
idle.  Checked against the vectorised / per-walker oracle at the parity bar, against the lane
geometry (forced with ModelSpec.disp_geometry) to a few ulp, for ensemble-size independence
bit for bit, and through the device DEMetropolisZ (proposal / log-prob / accept kernels)
against the torch sampler bit for bit."""
import dataclasses

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
N_FULL = 25256
MODELS = ["dispersion", "dispersion-piston", "exponential-dispersion"]


def _close(a, b, rtol=1e-12, atol=1e-9):
    both_nan = np.isnan(a) & np.isnan(b)
    same_inf = np.isinf(a) & np.isinf(b) & (np.sign(a) == np.sign(b))
    with np.errstate(invalid="ignore"):
        return both_nan | same_inf | (np.abs(a - b) <= atol + rtol * np.abs(b))


def _same(a, b):
    import torch
    return torch.equal(a, b) or bool(((a == b) | (torch.isnan(a) & torch.isnan(b))).all())


def _spec(model, variant, L, N=N_FULL, geometry="auto"):
    from noblegas_rtd_mcmc_amd import workloads as wl
    m1, _, m2 = model.partition("-")
    sv = "123" if variant.endswith("123") else ""
    if variant.startswith("rtd_only"):
        spec = wl.rtd_only_spec(L=L, N=N, mod_type1=m1, mod_type2=m2 or None, savenum=sv)
    else:
        spec = wl.c4_spec(L=L, N=N, mod_type1=m1, mod_type2=m2 or None, par_names=wl.model_par_names(m1, m2 or None, sv))
    return dataclasses.replace(spec, jacobian=variant.endswith("jac"), disp_geometry=geometry)


@pytest.mark.parametrize("model", MODELS)
@pytest.mark.parametrize("variant", ["rtd_only_123", "rtd_only", "joint", "joint_123"])
def test_reference_shape_vs_oracle(model, variant):
    """1 well x 3 walkers at N = 25 256 (the reference's run shape): the plan takes the wide
    geometry by itself (plan_info disp_wide_g > 0), two kernels per log-prob (the sums, then
    the generic single launch), values vs the vectorised oracle at rtol 1e-12 / atol 1e-9."""
    import torch
    from noblegas_rtd_mcmc_amd import workloads as wl
    from noblegas_rtd_mcmc_amd.engine import LogProb
    from oracle.vectorized import log_prob_vec
    spec = _spec(model, variant, L=1)
    W = 3
    th = wl.sample_prior(spec, 40, np.random.default_rng(2528))[:, :, :W].copy()
    lp = LogProb(spec, max_walkers=W)
    assert lp.info(W)["disp_wide_g"] > 0
    dev = torch.from_numpy(th).cuda()
    lp.ctx.set_profiling(True)
    lp.kernel_stats(reset=True)
    a = lp(dev).cpu().numpy()
    lp.ctx.set_profiling(False)
    ks = lp.kernel_stats(reset=True)
    assert ks["rtd"][1] == 1 and ks["fused"][1] == 1 and ks["unit"][1] == 0, ks
    assert np.array_equal(a, lp(th, soa=True), equal_nan=True)
    ref = log_prob_vec(spec, th)
    ok = _close(a, ref)
    assert ok.all(), (a, ref)
    assert np.isfinite(a).any()
    lp.close()


@pytest.mark.parametrize("model", MODELS)
@pytest.mark.parametrize("variant", ["joint", "joint_123", "rtd_only_123", "joint_jac"])
def test_wide_forced_vs_lane_and_oracle(model, variant):
    """The wide geometry forced on a c4-shape plan (4 wells x 130 walkers, N = 1200) against
    the lane geometry of the same plan (summation order only: 1e-13 relative on the log-prob)
    and the vectorised oracle on 64 walkers; forward() concentrations vs the lane plan's."""
    import torch
    from noblegas_rtd_mcmc_amd import workloads as wl
    from noblegas_rtd_mcmc_amd.engine import LogProb
    from oracle.vectorized import log_prob_vec
    W = 130
    spw = _spec(model, variant, L=4, N=1200, geometry="wide")
    spl = dataclasses.replace(spw, disp_geometry="lane")
    th = wl.sample_prior(spw, W, np.random.default_rng(61))
    lw, ll = LogProb(spw, max_walkers=W), LogProb(spl, max_walkers=W)
    assert lw.info(W)["disp_wide_g"] > 0 and ll.info(W)["disp_wide_g"] == 0
    dev = torch.from_numpy(th).cuda()
    a, b = lw(dev).cpu().numpy(), ll(dev).cpu().numpy()
    assert _close(a, b, 1e-13, 1e-10).all()
    sel = list(range(0, W, 2))
    ref = log_prob_vec(spw, np.ascontiguousarray(th[:, :, sel]))
    ok = _close(a[sel], ref)
    assert ok.all(), (np.array(sel)[~ok], a[sel][~ok], ref[~ok])
    if not variant.endswith("jac"):
        _, ra = lw.forward(th, soa=True)
        _, rb = ll.forward(th, soa=True)
        assert _close(ra, rb, 1e-13, 0.0).all()
    lw.close()
    ll.close()


def test_wide_edges_vs_oracle():
    """D at its prior's ends, 0 and beyond, tau1 / tau2 at and past their priors' ends, f1 at
    0 and 1, on the wide plan of 2 wells x 64 walkers: the per-walker oracle's values and its
    -inf / NaN pattern."""
    import oracle.models as om
    from noblegas_rtd_mcmc_amd import workloads as wl
    from noblegas_rtd_mcmc_amd.engine import LogProb
    spec = _spec("dispersion-piston", "joint", L=2, N=1200)
    W = 64
    th = wl.sample_prior(spec, W, np.random.default_rng(3))
    R = {r: i for i, r in enumerate(spec.roles)}
    edits = {"tau1": [1.0, 1000.0, 0.3, 1500.0, 0.0, -2.0], "tau2": [50.0, 15000.0, 20000.0, 3.0],
             "D1": [0.01, 2.0, 0.0, 3.0, -0.5, np.nan], "f1": [0.01, 0.99, 0.0, 1.0]}
    w = 0
    for role, vals in edits.items():
        for v in vals:
            th[R[role], :, w] = v
            w += 1
    lp = LogProb(spec, max_walkers=W)
    assert lp.info(W)["disp_wide_g"] > 0
    got = lp(th, soa=True)
    ref = om.log_prob(spec, th, walkers=range(W))
    ok = _close(got, ref)
    assert ok.all(), (np.nonzero(~ok)[0], got[~ok], ref[~ok])
    assert np.isnan(ref).any() or np.isneginf(ref).any()
    lp.close()


def test_wide_independent_of_ensemble_size():
    """A walker's log-prob on a wide plan does not depend on how many walkers share the launch
    (G is fixed per plan): subsets equal the full ensemble bit for bit."""
    import torch
    from noblegas_rtd_mcmc_amd import workloads as wl
    from noblegas_rtd_mcmc_amd.engine import LogProb
    spec = _spec("dispersion", "rtd_only_123", L=2, N=N_FULL)
    W = 100
    th = wl.sample_prior(spec, W, np.random.default_rng(8))
    lp = LogProb(spec, max_walkers=W)
    assert lp.info(W)["disp_wide_g"] > 0
    full = lp(torch.from_numpy(th).cuda()).cpu().numpy()
    for lo, n in ((0, 1), (7, 3), (50, 50)):
        sub = lp(torch.from_numpy(np.ascontiguousarray(th[:, :, lo:lo + n])).cuda()).cpu().numpy()
        assert np.array_equal(sub, full[lo:lo + n], equal_nan=True), (lo, n)
    units = lp.units(torch.from_numpy(th).cuda()).cpu().numpy()
    assert np.array_equal(units.sum(axis=0), full, equal_nan=True) or _close(units.sum(axis=0), full, 1e-15, 0).all()
    lp.close()


@pytest.mark.parametrize("per_well", [True, False])
@pytest.mark.parametrize("jac", [True, False])
@pytest.mark.parametrize("model", ["dispersion", "dispersion-piston"])
def test_reference_shape_demcz_bitwise(model, jac, per_well):
    """The reference's own dispersion run shape -- RTD-only, 4 tracers, savenum 123, 1 well,
    3 chains, N = 25 256 -- through the device DEMetropolisZ (per-well chains: the proposal
    kernel, the wide sums + generic log-prob, the accept kernel per step) against the torch
    sampler over the same plan's ngrtd_logp_units, bit for bit through tuning, stop_tuning and
    the draws.  per_well False: one chain per walker, the decision in the log-prob launch's
    per-walker reduction (plan_run with the DemcAccept), on the wide plan."""
    import torch
    from noblegas_rtd_mcmc_amd import workloads as wl
    from noblegas_rtd_mcmc_amd.engine import LogProb
    from noblegas_rtd_mcmc_amd.sampler import DEMetropolisZ, DeviceDEMetropolisZ, Transform
    spec = dataclasses.replace(_spec(model, "rtd_only_123", L=1), jacobian=jac)
    W = 3
    x0 = torch.from_numpy(wl.test_point(spec, W)).cuda()
    lp = LogProb(spec, max_walkers=W)
    assert lp.info(W)["disp_wide_g"] > 0
    kw = dict(tune_interval=4, seed=1234, per_well=per_well)
    dev = DeviceDEMetropolisZ(lp, **kw).run(x0, tune=16, draws=12)
    tf = Transform.from_spec(spec) if jac else None
    f = (lambda t: lp.units(t)) if per_well else (lambda t: lp(t))
    ref = DEMetropolisZ(f, transform=tf, **kw).run(x0, tune=16, draws=12)
    for k in ("x", "lp", "samples", "logp", "accepted", "accept", "lamb", "scaling"):
        assert _same(dev[k], ref[k]), k
    assert 0 < int(dev["accepted"].sum()) < dev["accepted"].numel()
    lp.close()
