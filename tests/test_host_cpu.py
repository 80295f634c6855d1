"""CPU tests of the host-side logic: specs, layouts, workloads, sampler mechanics, and the
drop-in modules' argument handling (no device calls)."""
import numpy as np
import pandas as pd
import pytest
import torch

from noblegas_rtd_mcmc_amd import spec as S
from noblegas_rtd_mcmc_amd import workloads as wl


def test_roles_and_layout():
    spec = wl.c4_spec(L=3, N=50)
    assert spec.roles == ["Ae_beta", "F_beta", "E_beta", "m", "b_beta", "nu_ce_beta", "tau1", "nu_rtd_beta"]
    th = wl.sample_prior(spec, 5, np.random.default_rng(0))
    assert th.shape == (8, 3, 5)
    wlp = spec.theta_wlp(th)
    assert wlp.shape == (5, 3, 8)
    assert np.array_equal(spec.theta_soa(wlp), th)
    assert np.array_equal(spec.theta_soa(wlp.reshape(5, 24)), th)
    ri = spec.role_index()
    assert ri[S.ROLE_IDS["tau1"]] == 6 and ri[S.ROLE_IDS["J"]] == -1


def test_spec_validation():
    fd = wl.field_data()
    with pytest.raises(ValueError):
        S.ModelSpec(n_wells=1)
    with pytest.raises(ValueError):
        S.CEBlock(obs=np.ones((2, 3)), sd=np.ones((2, 3)), E_min=np.ones(2), gases=("Ne", "Ar"))
    t = wl.tracer("CFC12", 10)
    with pytest.raises(ValueError):
        S.RTDBlock(tracers=[t], obs=np.ones((1, 1)), sd=np.ones((1, 1)), mod_type1="frac_inf_diff")
    with pytest.raises(ValueError):
        S.RTDBlock(tracers=[t, wl.tracer("SF6", 11)], obs=np.ones((1, 2)), sd=np.ones((1, 2)))
    assert fd["well_elev"]["PLM1"] == 2786.889893


def test_bmm_roles_and_priors_sampling():
    spec = wl.c4_spec(L=2, N=40, mod_type1="exp_pist_flow", mod_type2="piston",
                      par_names=("tau1", "tau2", "f1", "eta1", "J", "thalf_cfc", "lamsf6"))
    th = wl.sample_prior(spec, 200, np.random.default_rng(1))
    r = dict(zip(spec.roles, th))
    assert (r["tau2"] >= 50).all() and (r["tau2"] <= 15000).all()
    assert (r["f1"] >= 0.01).all() and (r["lamsf6"] >= 0).all()
    assert ((r["thalf_cfc_beta"] > 0) & (r["thalf_cfc_beta"] < 1)).all()


def test_workload_shapes():
    spec, th = wl.c2(W=16)
    assert spec.n_wells == 3 and spec.ce.gases == ("He", "Ne", "Ar", "Kr", "Xe") and th.shape == (6, 3, 16)
    spec, th = wl.c3(W=16)
    assert spec.rtd.n_ages == 1200 and spec.roles == ["tau1", "nu_rtd_beta", "J"]
    spec, th = wl.c1()
    assert th.shape == (6, 1, 100)
    s = wl.atmos_series("H3", 25256)
    # C_in_dict.pk H3: 69 recent ages, then the pre-bomb fill (prep.py:168 repeats the first row)
    assert s.n == 25256 and s.c_by_age[-1] == 3.327329892219456 and s.c_by_age[0] == 5.997188929906611


def test_series_from_reference_frames():
    from noblegas_rtd_mcmc_amd.convolution_integral_utils import _series_arrays
    idx = np.arange(9, -1, -1)
    df = pd.DataFrame({"He4_ter": np.zeros(10), "other": np.ones(10)}, index=idx)
    v, i = _series_arrays(df, "4He")
    assert np.array_equal(v, np.zeros(10)) and np.array_equal(i, idx)
    with pytest.raises(ValueError):
        _series_arrays(df, False)
    v, i = _series_arrays(pd.DataFrame({"x": np.arange(10.0)}, index=idx), False)
    assert np.array_equal(v, np.arange(10.0))
    ser = S.Series.from_reference_frame(v, i, 3.7)
    assert ser.dtp == 3.0 and ser.c_by_age[0] == 9.0


def test_demcz_gaussian_moments():
    """DEMetropolisZ recovers a correlated 2-D Gaussian: the final states of 2000
    independent chains are draws from the target, so their mean and covariance must sit
    within 4 Monte-Carlo standard errors of the truth (CPU, torch)."""
    from noblegas_rtd_mcmc_amd.sampler import DEMetropolisZ
    cov = np.array([[1.0, 0.6], [0.6, 2.0]])
    P = torch.from_numpy(np.linalg.inv(cov))

    def lp(x):   # x [2, W]
        return -0.5 * torch.einsum("iw,ij,jw->w", x, P, x)
    W = 2000
    x0 = torch.from_numpy(np.random.default_rng(0).normal(size=(2, W)) * 3)
    res = DEMetropolisZ(lp, tune_interval=50, seed=1).run(x0, tune=300, draws=300)
    fin = res["x"].numpy().T                                         # [W][2]
    se_mean = np.sqrt(np.diag(cov) / W)
    assert (np.abs(fin.mean(0)) < 4 * se_mean).all(), fin.mean(0)
    c = np.cov(fin.T)
    se_cov = np.sqrt((cov ** 2 + np.outer(np.diag(cov), np.diag(cov))) / W)   # Gaussian var of sample cov
    assert (np.abs(c - cov) < 4 * se_cov).all(), c
    assert 0.1 < res["accept_rate"] < 0.9
    again = DEMetropolisZ(lp, tune_interval=50, seed=1).run(x0, tune=300, draws=300)
    assert torch.equal(again["samples"], res["samples"])


def test_demcz_rng_matches_integer_reference():
    """The torch splitmix64 (int64 tensors, wrapping) equals the integer restatement."""
    from noblegas_rtd_mcmc_amd.sampler import mix_int, mix_t, _s64, unit_t
    vals = [0, 1, 2 ** 63 - 1, 2 ** 63, 2 ** 64 - 1, 0x9E3779B97F4A7C15, 123456789123456789]
    vals += list(np.random.default_rng(3).integers(0, 2 ** 63, 50, dtype=np.int64).tolist())
    got = mix_t(torch.tensor([_s64(v) for v in vals], dtype=torch.int64)).tolist()
    assert got == [_s64(mix_int(v)) for v in vals]
    u = unit_t(torch.tensor([_s64(mix_int(v)) for v in vals], dtype=torch.int64))
    assert bool(((u > 0) & (u < 1)).all())


def test_demcz_partner_distribution_uniform():
    """iz1 != iz2, each ordered pair of distinct history entries equally likely (so the
    difference z1 - z2 is symmetric: no Hastings correction needed)."""
    from noblegas_rtd_mcmc_amd.sampler import mix_int, mix_t, _s64, _lsr, step_key, _M64
    for it in (2, 3, 5):
        counts = np.zeros((it, it))
        for s in range(40):
            key = step_key(7, s)
            w = torch.arange(4000, dtype=torch.int64)
            hp = mix_t(w + _s64(mix_int((key + 1) & _M64)))
            iz1 = (_lsr(hp, 32) * it) >> 32
            iz2 = ((hp & 0xFFFFFFFF) * (it - 1)) >> 32
            iz2 = iz2 + (iz2 >= iz1).to(torch.int64)
            np.add.at(counts, (iz1.numpy(), iz2.numpy()), 1)
        assert np.all(np.diag(counts) == 0)
        off = counts[~np.eye(it, dtype=bool)]
        expect = counts.sum() / (it * (it - 1))
        assert np.all(np.abs(off - expect) < 5 * np.sqrt(expect)), (it, counts)
        assert np.abs(counts - counts.T).max() < 5 * np.sqrt(2 * expect)


def test_pymc3_tune_schedule():
    from noblegas_rtd_mcmc_amd.sampler import pymc3_tune
    r = torch.tensor([0.0005, 0.01, 0.1, 0.3, 0.6, 0.8, 0.96], dtype=torch.float64)
    got = pymc3_tune(torch.ones(7, dtype=torch.float64), r).tolist()
    assert got == [0.1, 0.5, 0.9, 1.0, 1.1, 2.0, 10.0]


def test_demcz_tuning_and_history_drop():
    """lamb is tuned every tune_interval steps of the tuning phase only; stop_tuning drops
    the oldest 90 % of the history (proposals after it draw from the kept entries)."""
    from noblegas_rtd_mcmc_amd.sampler import DEMetropolisZ, default_lamb

    def lp(x):
        return -0.5 * (x ** 2).sum(0)
    x0 = torch.from_numpy(np.random.default_rng(1).normal(size=(3, 16)))
    res = DEMetropolisZ(lp, tune_interval=10, seed=4).run(x0, tune=35, draws=20)
    assert not torch.equal(res["lamb"], torch.full((16,), default_lamb(3), dtype=torch.float64))
    fixed = DEMetropolisZ(lp, tune=None, tune_interval=10, seed=4).run(x0, tune=35, draws=20)
    assert torch.equal(fixed["lamb"], torch.full((16,), default_lamb(3), dtype=torch.float64))
    assert res["samples"].shape == (20, 3, 16) and res["accepted"].shape == (20, 16)


def test_demcz_per_well_chains_are_independent():
    """per_well=True: every (walker, well) unit is its own chain.  A 3-well run equals three
    1-well runs (well0 = l) chain for chain, bit for bit, and each unit's decision only sees
    its own log-prob (a well whose log-prob is -inf everywhere but the start never moves,
    the others do)."""
    from noblegas_rtd_mcmc_amd.sampler import DEMetropolisZ, default_lamb
    rng = np.random.default_rng(2)
    P, L, W = 3, 3, 10
    x0 = torch.from_numpy(rng.normal(size=(P, L, W)))
    scale = torch.tensor([1.0, 2.0, 0.5], dtype=torch.float64)[:, None]

    def lpu(x):                                   # [P][L][W] -> [L][W], a different Gaussian per well
        return -0.5 * (x ** 2).sum(0) / scale ** 2
    full = DEMetropolisZ(lpu, tune_interval=5, seed=9, per_well=True).run(x0, tune=12, draws=8)
    assert tuple(full["logp"].shape) == (8, L, W) and tuple(full["lamb"].shape) == (L, W)
    for l in range(L):
        one = DEMetropolisZ(lambda x, l=l: -0.5 * (x ** 2).sum(0) / scale[l] ** 2, tune_interval=5, seed=9,
                            per_well=True, well0=l).run(x0[:, l:l + 1].clone(), tune=12, draws=8)
        assert torch.equal(one["samples"][:, :, 0], full["samples"][:, :, l])
        assert torch.equal(one["logp"][:, 0], full["logp"][:, l])
    fixed = DEMetropolisZ(lpu, tune=None, seed=9, per_well=True).run(x0, tune=4, draws=4)
    assert torch.equal(fixed["lamb"], torch.full((L, W), default_lamb(P), dtype=torch.float64))

    def stuck(x):                                 # well 1 rejects every move
        v = lpu(x)
        v[1] = torch.where(torch.isclose(x[0, 1], x0[0, 1]), v[1], torch.full_like(v[1], -np.inf))
        return v
    st = DEMetropolisZ(stuck, tune_interval=5, seed=9, per_well=True).run(x0, tune=12, draws=8)
    assert torch.equal(st["x"][:, 1], x0[:, 1]) and not torch.equal(st["x"][:, 0], x0[:, 0])
    assert int(st["accepted"][:, 1].sum()) == 0 and int(st["accepted"][:, 0].sum()) > 0


def test_ce_sampler_plumbing_with_cpu_logp():
    """c1 plumbing: DEMetropolisZ driving the CE log-prob (oracle as the CPU log-prob)."""
    import oracle.models as om
    from noblegas_rtd_mcmc_amd.sampler import DEMetropolisZ
    spec, th = wl.c1(W=12)

    def lp(x):
        return torch.from_numpy(om.log_prob(spec, x.numpy()))
    res = DEMetropolisZ(lp, tune_interval=5, seed=2).run(torch.from_numpy(th), tune=10, draws=5)
    assert res["samples"].shape == (5, 6, 1, 12) and torch.isfinite(res["logp"]).all()


def test_trace_layout_roundtrip(tmp_path):
    """ArviZ-layout trace (trace.py): posterior per PyMC3 variable name with (chain, draw)
    dims, deterministics, sample_stats, tuning_steps / sampling_time attrs; one netCDF-4
    file (h5lite), read back."""
    from noblegas_rtd_mcmc_amd import trace
    spec = wl.c4_spec(L=1, N=50, mod_type1="exponential", mod_type2="piston",
                      par_names=("tau1", "tau2", "f1", "thalf_cfc", "lamsf6"))
    from noblegas_rtd_mcmc_amd.spec import ModelSpec
    spec = ModelSpec(n_wells=1, rtd=spec.rtd)
    D, W = 7, 5
    rng = np.random.default_rng(0)
    s = np.stack([wl.sample_prior(spec, W, rng) for _ in range(D)])          # [D, P, 1, W]
    res = {"samples": torch.from_numpy(s), "logp": torch.from_numpy(rng.normal(size=(D, W))),
           "accepted": torch.from_numpy(rng.integers(0, 2, (D, W)).astype(np.uint8)),
           "lamb": torch.full((W,), 0.5, dtype=torch.float64), "scaling": torch.full((W,), 1e-3, dtype=torch.float64),
           "tuning_steps": 10000, "sampling_time": 12.5}
    idata = trace.inference_data(res, spec)
    p = idata["posterior"]
    for name in ("tau1", "tau2", "f1", "f2", "tau", "nu_", "nu", "thalf_cfc_", "thalf_cfc", "lamsf6"):
        assert p[name][0] == ("chain", "draw") and p[name][1].shape == (W, D), name
    i = spec.roles.index("tau1")
    assert np.array_equal(p["tau1"][1], s[:, i, 0, :].T)
    f1 = s[:, spec.roles.index("f1"), 0, :].T
    assert np.allclose(p["tau"][1], f1 * p["tau1"][1] + (1 - f1) * p["tau2"][1])
    out = trace.to_netcdf(idata, str(tmp_path / "PLM1.CFC12.exponential-piston.0.netcdf"))
    back = trace.from_netcdf(out)
    assert back["attrs"]["tuning_steps"] == 10000 and back["attrs"]["sampling_time"] == 12.5
    for g in ("posterior", "sample_stats"):
        for k, (dims, arr) in idata[g].items():
            assert back[g][k][0] == dims and np.array_equal(back[g][k][1], arr, equal_nan=arr.dtype.kind == "f"), (g, k)
    assert np.array_equal(back["coords"]["chain"], np.arange(W))


def test_bench_model_lines_name_the_instance_each_plan_runs():
    """bench.py's `models` lines cite the logp_fused_kernel instance of each c4 plan (MIX bits:
    1 piston second, 2 exp_pist_flow first, 32 sampled CFC12 half-life, 64 generic, 128 the
    generic instances of plans with a dispersion component -- ngrtd.hip gen_mix) and attach a
    PMC FLOP rate only to instances that run one model."""
    import bench
    inst = {(m1, m2, sv): bench.fused_instance(m1, m2, sv) for m1, m2, sv in bench.PUBLISHED_MODELS + bench.OTHER_MODELS}
    assert inst[("exponential", None, "")] == "logp_fused_kernel<5, true, 2, 0>"
    assert inst[("exp_pist_flow", "piston", "123")] == "logp_fused_kernel<5, true, 2, 35>"
    assert inst[("piston", None, "")] == "logp_fused_kernel<5, true, 2, 64>"
    assert inst[("dispersion", None, "")] == "logp_fused_kernel<5, true, 2, 192>"
    assert inst[("dispersion", None, "123")] == "logp_fused_kernel<5, true, 2, 224>"
    assert inst[("exponential", "dispersion", "")] == "logp_fused_kernel<5, true, 2, 192>"
    # the specialised instances are one per published model and savenum
    spec_inst = [v for (m1, m2, sv), v in inst.items() if not int(v.rsplit(", ", 1)[1].rstrip(">")) & 64]
    assert len(spec_inst) == len(set(spec_inst)) == len(bench.PUBLISHED_MODELS)
