"""Deterministic builders for the BASELINE.json configurations c1..c5.

All inputs are synthetic or come from the small data tables under ``data/``, extracted
from the reference's shipped files by tools/make_package_data.py: the noble-gas obs of
Field_Data/PLM_noblegas_2021.xlsx, the input series of age_ens_runs_mcmc/C_in_dict.pk
(bit-exact) and the MAP tracer obs of age_ens_runs_mcmc/map_dict.pk:

* c1  CE plumbing: PLM1, gases Ne/Ar/Kr/Xe, 100 walkers (sampler: 500 steps, seed 12345).
* c2  CE log-prob: 2048 walkers x 3 wells (PLM1, PLM6, PLM7) x 5 gases.
* c3  RTD log-prob: 2048 walkers x 1 well x 4 tracers (CFC12, SF6, H3, He4_ter), N=1200,
      exponential model, sampled log10 J (savenum-1 style), obs = MAP PLM1, sd = 0.10 obs.
* c4  joint CE + RTD: 2048 walkers x 64 wells x (5 gases + 5 tracers), N=1200, synthetic
      non-constant series, per-well obs perturbed lognormally.
* c5  c4 sharded as walker blocks over ranks.
"""
import json
import os

import numpy as np

from .spec import CEBlock, ModelSpec, RTDBlock, Series, Tracer, LOG10_J_HE4_DEFAULT

_DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data")


def field_data():
    with open(os.path.join(_DATA, "plm_field_data.json")) as f:
        return json.load(f)


def atmos_series(name, n=None):
    """The shipped input series C_in_dict[name] (prep.py:165-219), age-first
    (= np.flip(C_in_dict[name].values), convolution_integral_utils.py:336), its first n
    ages (= the last n rows of the DataFrame; default all 25256).  'He3' uses the H3
    history (run_age_mcmc.py:217-220)."""
    z = np.load(os.path.join(_DATA, "atmos_series.npz"), allow_pickle=False)
    key = "H3" if name == "He3" else name
    N = int(z["N_full"]) if n is None else int(n)
    fill = float(z[key + "_fill"])
    tail = np.asarray(z[key + "_tail"], dtype=np.float64)
    c = np.full(N, fill)
    m = min(N, len(tail))
    c[:m] = tail[:m]
    return Series(c, np.arange(N, dtype=np.float64), 0.0)


def tracer(name, n=None, series=None, log10_J=None):
    """Per-tracer convolution kwargs of run_age_mcmc.py:205-224."""
    s = series if series is not None else atmos_series(name, n)
    if name in ("CFC11", "CFC12", "CFC113", "SF6"):
        return Tracer(name, s)
    if name == "He4_ter":
        return Tracer(name, Series(s.c_by_age * 0.0, s.idx_by_age, s.dtp), rad_accum="4He",
                      log10_J=log10_J)
    if name == "He3":
        return Tracer(name, s, t_half=12.34, rad_accum="3He")
    if name == "H3":
        return Tracer(name, s, t_half=12.34)
    raise ValueError(name)


def map_obs(well):
    """MAP tracer observations map_dict[tracer].loc[well] (run_age_mcmc.py:44, prep.py:453-494)."""
    return {t: v[well] for t, v in field_data()["map_obs"].items() if well in v}


def ce_block(wells, gases, E_min=None, obs=None, sd=None):
    fd = field_data()
    if obs is None:
        obs = np.array([[fd["obs"][w][g] for g in gases] for w in wells])
    if sd is None:
        sd = obs * np.array([fd["err_percent"][g] / 100 for g in gases])
    if E_min is None:
        E_min = np.array([fd["well_elev"][w] - 10.0 for w in wells])
    return CEBlock(obs=obs, sd=sd, E_min=E_min, gases=tuple(gases))


def sample_prior(spec, W, rng):
    """Draw theta SoA [P][L][W] from the natural-space priors of ``spec``."""
    L = spec.n_wells
    th = np.zeros((spec.n_params, L, W))
    for i, role in enumerate(spec.roles):
        sh = (L, W)
        c, r = spec.ce, spec.rtd
        if role == "Ae_beta":
            v = rng.beta(*c.beta_Ae, size=sh)
        elif role == "F_beta":
            v = rng.beta(*c.beta_F, size=sh)
        elif role == "E_beta":
            v = rng.beta(*c.beta_E, size=sh)
        elif role == "m":
            v = rng.normal(c.m_mu, c.m_sd, size=sh)
        elif role == "b_beta":
            v = rng.beta(*c.beta_b, size=sh)
        elif role == "nu_ce_beta":
            v = rng.beta(*c.beta_nu, size=sh)
        elif role == "nu_rtd_beta":
            v = rng.beta(*r.beta_nu, size=sh)
        elif role in ("tau1", "tau2", "f1", "eta1", "eta2", "D1", "D2"):
            lo, hi = getattr(r, role)
            v = rng.uniform(lo, hi, size=sh)
        elif role == "J":
            v = rng.normal(r.J_mu, r.J_sd, size=sh)
        elif role == "thalf_cfc_beta":
            v = rng.beta(*r.beta_thalf, size=sh)
        elif role == "lamsf6":
            v = np.abs(rng.normal(0.0, r.lamsf6_sd, size=sh))
        else:
            raise ValueError(role)
        if role.endswith("_beta"):
            # rng.beta(2, 0.1) returns exactly 1.0 often; PyMC3 samples these in logodds
            # space and never sits on the boundary, so keep draws strictly inside (0, 1).
            v = np.clip(v, 1e-9, 1.0 - 1e-9)
        th[i] = v
    return th


def test_point(spec, W):
    """PyMC3 3.11's starting point of every chain when mc.sample gets no `start` and the step is
    not NUTS (run_age_mcmc_utils.py:412-417, noble_gas_mcmc.py:410-415): model.test_point, each
    free variable's default test value -- the median where the distribution defines one, else the
    mean (Distribution.get_test_val over defaults ("median", "mean", "mode")): Uniform (a + b)/2,
    Normal mu, Beta a/(a + b) (mean: no median), HalfNormal sigma sqrt(2/pi) (mean).  theta SoA
    [P][L][W], every chain at that point."""
    L = spec.n_wells
    th = np.zeros((spec.n_params, L, W))
    c, r = spec.ce, spec.rtd
    for i, role in enumerate(spec.roles):
        if role.endswith("_beta"):
            ab = {"Ae_beta": c.beta_Ae if c else None, "F_beta": c.beta_F if c else None, "E_beta": c.beta_E if c else None,
                  "b_beta": c.beta_b if c else None, "nu_ce_beta": c.beta_nu if c else None,
                  "nu_rtd_beta": r.beta_nu if r else None, "thalf_cfc_beta": r.beta_thalf if r else None}[role]
            v = ab[0] / (ab[0] + ab[1])
        elif role == "m":
            v = c.m_mu
        elif role in ("tau1", "tau2", "f1", "eta1", "eta2", "D1", "D2"):
            lo, hi = getattr(r, role)
            v = (lo + hi) / 2.0
        elif role == "J":
            v = r.J_mu
        elif role == "lamsf6":
            v = r.lamsf6_sd * np.sqrt(2.0 / np.pi)
        else:
            raise ValueError(role)
        th[i] = v
    return th


def prior_sd(spec):
    """Prior standard deviation of every theta row [P][L] -- a per-parameter proposal scale
    (PyMC3 DEMetropolisZ's S) that puts the U(-S, S) * scaling noise of every dimension on
    the same footing.  Uniform (b - a)/sqrt(12), Beta sqrt(ab/((a+b)^2 (a+b+1))), Normal sd,
    HalfNormal sd sqrt(1 - 2/pi)."""
    def beta_sd(ab):
        a, b = ab
        return np.sqrt(a * b / ((a + b) ** 2 * (a + b + 1)))
    c, r = spec.ce, spec.rtd
    sd = []
    for role in spec.roles:
        if role in ("Ae_beta", "F_beta", "E_beta", "b_beta", "nu_ce_beta"):
            v = beta_sd({"Ae_beta": c.beta_Ae, "F_beta": c.beta_F, "E_beta": c.beta_E, "b_beta": c.beta_b,
                         "nu_ce_beta": c.beta_nu}[role])
        elif role == "m":
            v = c.m_sd
        elif role == "nu_rtd_beta":
            v = beta_sd(r.beta_nu)
        elif role == "thalf_cfc_beta":
            v = beta_sd(r.beta_thalf)
        elif role in ("tau1", "tau2", "f1", "eta1", "eta2", "D1", "D2"):
            lo, hi = getattr(r, role)
            v = (hi - lo) / np.sqrt(12.0)
        elif role == "J":
            v = r.J_sd
        elif role == "lamsf6":
            v = r.lamsf6_sd * np.sqrt(1 - 2 / np.pi)
        else:
            raise ValueError(role)
        sd.append(v)
    return np.repeat(np.array(sd, dtype=np.float64)[:, None], spec.n_wells, axis=1)


def c1(W=100):
    spec = ModelSpec(n_wells=1, ce=ce_block(["PLM1"], ("Ne", "Ar", "Kr", "Xe")))
    return spec, sample_prior(spec, W, np.random.default_rng(12345))


def c2(W=2048):
    spec = ModelSpec(n_wells=3, ce=ce_block(["PLM1", "PLM6", "PLM7"], ("He", "Ne", "Ar", "Kr", "Xe")))
    return spec, sample_prior(spec, W, np.random.default_rng(12345))


def c3(W=2048, N=1200):
    fd = field_data()
    names = ("CFC12", "SF6", "H3", "He4_ter")
    mu = np.array([[map_obs("PLM1")[t] for t in names]])
    rtd = RTDBlock(tracers=[tracer(t, N) for t in names], obs=mu, sd=0.10 * mu,
                   mod_type1="exponential", par_names=("tau1", "J"))
    spec = ModelSpec(n_wells=1, rtd=rtd)
    return spec, sample_prior(spec, W, np.random.default_rng(23456))


def c4_spec(L=64, N=1200, seed=34567, mod_type1="exponential", mod_type2=None, par_names=("tau1",)):
    rng = np.random.default_rng(seed)
    fd = field_data()
    base_wells = ["PLM1", "PLM6", "PLM7"]
    wells = [base_wells[l % 3] for l in range(L)]
    gases = ("He", "Ne", "Ar", "Kr", "Xe")
    ce_obs = np.array([[fd["obs"][w][g] for g in gases] for w in wells]) * rng.lognormal(0, 0.1, (L, 5))
    ce = ce_block(wells, gases, obs=ce_obs)
    names = ("CFC12", "SF6", "H3", "He3", "He4_ter")
    trs = []
    for t in names:
        s = atmos_series(t, N)
        c = s.c_by_age * rng.lognormal(0.0, 0.05, N)   # non-constant everywhere
        trs.append(tracer(t, series=Series(c, s.idx_by_age, 0.0),
                          log10_J=LOG10_J_HE4_DEFAULT if t == "He4_ter" else None))
    base = map_obs("PLM1")
    rtd_obs = np.array([[base[t] for t in names]] * L) * rng.lognormal(0, 0.1, (L, len(names)))
    rtd = RTDBlock(tracers=trs, obs=rtd_obs, sd=0.10 * rtd_obs, mod_type1=mod_type1,
                   mod_type2=mod_type2, par_names=par_names)
    return ModelSpec(n_wells=L, ce=ce, rtd=rtd)


# the parameters each RTD model adds (run_age_mcmc.py:140-178: eta for exp_pist_flow, D for
# dispersion; tau2 and f1 for a BMM) and the savenum digits (1 J, 2 thalf_cfc, 3 lamsf6)
RTD_MODEL_PARS = {"exponential": (), "piston": (), "exp_pist_flow": ("eta",), "dispersion": ("D",)}


def model_par_names(mod_type1="exponential", mod_type2=None, savenum=""):
    """par_names of a model in the reference's order: tau1, [tau2, f1], the first component's
    eta1 / D1, the second's eta2 / D2, then the savenum parameters."""
    pn = ["tau1"] + (["tau2", "f1"] if mod_type2 else [])
    pn += [q + "1" for q in RTD_MODEL_PARS[mod_type1]]
    if mod_type2:
        pn += [q + "2" for q in RTD_MODEL_PARS[mod_type2]]
    pn += [{"1": "J", "2": "thalf_cfc", "3": "lamsf6"}[d] for d in str(savenum or "") if d in "123"]
    return tuple(pn)


def rtd_only_spec(L=64, N=1200, tracers=("CFC12", "SF6", "H3", "He4_ter"), mod_type1="exponential", mod_type2=None,
                  savenum="123", seed=34567):
    """The reference's own RTD model (run_age_mcmc.py:122-231: RTD-only, the 4-tracer set or
    one tracer; savenum digits 1 J, 2 thalf_cfc, 3 lamsf6 sampled) over L wells with c4's
    synthetic per-well obs and series (the same seeded draws, restricted to these tracers)."""
    import dataclasses
    names = ("CFC12", "SF6", "H3", "He3", "He4_ter")
    pn = model_par_names(mod_type1, mod_type2, savenum)
    base = c4_spec(L=L, N=N, seed=seed, mod_type1=mod_type1, mod_type2=mod_type2, par_names=pn)
    keep = [names.index(t) for t in tracers]
    r = base.rtd
    rtd = dataclasses.replace(r, tracers=[r.tracers[i] for i in keep], obs=r.obs[:, keep], sd=r.sd[:, keep])
    return ModelSpec(n_wells=L, rtd=rtd)


def ce_only_spec(L=64, gases=("Ne", "Ar", "Kr", "Xe"), seed=34567):
    """The reference's own CE model (noble_gas_mcmc.py:216-267: Ne, Ar, Kr, Xe) over L wells
    with c4's synthetic per-well obs."""
    import dataclasses
    base = c4_spec(L=L, N=60, seed=seed)
    keep = [base.ce.gases.index(g) for g in gases]
    c = base.ce
    return ModelSpec(n_wells=L, ce=dataclasses.replace(c, obs=c.obs[:, keep], sd=c.sd[:, keep], gases=tuple(gases)))


def c4(W=2048, L=64, N=1200):
    spec = c4_spec(L=L, N=N)
    return spec, sample_prior(spec, W, np.random.default_rng(34568))


def shard_walkers(W_total, rank, world):
    """Contiguous walker block of ``rank`` (c5: W/G walkers per GPU)."""
    per = (W_total + world - 1) // world
    lo = min(W_total, rank * per)
    return lo, min(W_total, lo + per)


def c_in_dict(names=("CFC11", "CFC12", "CFC113", "SF6", "He4_ter", "H3")):
    """The reference's input-series dict C_in_dict (age_ens_runs_mcmc/C_in_dict.pk, read at
    run_age_mcmc.py:46) rebuilt from the shipped data: per tracer a one-column DataFrame indexed
    by age tau = 25255 ... 0 (oldest first), column 'H3_tu' for H3 (prep.py:207-219)."""
    import pandas as pd
    out = {}
    for name in names:
        s = atmos_series(name)
        idx = np.flip(s.idx_by_age).astype(np.int64)
        out[name] = pd.DataFrame({("H3_tu" if name == "H3" else name): np.flip(s.c_by_age)},
                                 index=pd.Index(idx, name="tau"))
    return out


# run_age_mcmc.py:100-114: the analytical error added to every tracer (PLM6's contaminated SF6:
# 10.0); the commented dict of :104-108 is what the published exponential-piston run used (the
# sigma fits of tests/golden/make_pymc3_accept.py show it)
OBS_PERR = {"CFC12": 0.05, "SF6": 0.05, "H3": 0.05, "He3": 0.05, "He4_ter": 0.05}
OBS_PERR_ALT = {"CFC12": 0.15, "SF6": 0.15, "H3": 0.10, "He3": 0.15, "He4_ter": 0.10}


def reference_run_kwargs(well, tracers, mod_type1="exponential", mod_type2=False, savenum=(0,), mu=None, sd=None,
                         perr=None, tau1=(1.0, 1000.0), C_in=None):
    """The keyword dicts run_age_mcmc.py:122-224 hands to conv_mcmc for one well: okw (the
    observation ensemble and its percent error), pkw (priors and par_names, :143-198), ckw
    (convolution kwargs per tracer, :203-224).  ens_dict.pk is not shipped, so the ensemble is
    the two-point [mu - s, mu + s] with s = sd - mu perr: the same mean mu and
    std(ens) + mu perr = sd that conv_mcmc computes (run_age_mcmc_utils.py:353-356)."""
    import copy
    from .spec import LOG10_J_PRIOR_MU
    alt = perr is OBS_PERR_ALT
    perr = dict(perr or OBS_PERR)
    if well == "PLM6" and not alt and perr.get("SF6") == 0.05:
        perr["SF6"] = 10.0
    C_in = C_in if C_in is not None else c_in_dict()
    okw = {}
    for k, t in enumerate(tracers):
        s = float(sd[k]) - float(mu[k]) * perr[t]
        okw[t] = {"obs_df": np.array([float(mu[k]) - s, float(mu[k]) + s]), "obs_perr": perr[t]}
    pkw = {"tau1_low": float(tau1[0]), "tau1_high": float(tau1[1])}
    par_names = ["tau1"]
    if mod_type2:
        pkw.update(tau2_low=50.0, tau2_high=15000.0, f1_low=0.01, f1_high=0.99)
        par_names += ["tau2", "f1", "f2"]
    for c, m in ((1, mod_type1), (2, mod_type2)):
        if m == "exp_pist_flow":
            pkw["eta%d_low" % c], pkw["eta%d_high" % c] = 1.0, 5.0
            par_names += ["eta%d" % c]
        if m == "dispersion":
            pkw["D%d_low" % c], pkw["D%d_high" % c] = 0.01, 2.0
            par_names += ["D%d" % c]
    if "He4_ter" in tracers and 1 in savenum:
        pkw["J_mu"], pkw["J_sd"] = LOG10_J_PRIOR_MU, 0.33
        par_names += ["J"]
    if "CFC12" in tracers and 2 in savenum:
        pkw["cfc_thalf_lo"], pkw["cfc_thalf_hi"] = 5.0, 35.0
        par_names += ["thalf_cfc"]
    if "SF6" in tracers and 3 in savenum:
        par_names += ["lamsf6"]
    pkw["par_names"] = par_names
    ckw = {"mod_type1": mod_type1, "mod_type2": mod_type2}
    for t in tracers:
        ckw[t] = {}
        if t in ("CFC11", "CFC12", "CFC113", "SF6"):
            ckw[t]["C_t"] = copy.deepcopy(C_in[t])
        elif t == "He4_ter":
            ckw[t]["C_t"] = copy.deepcopy(C_in[t]) * 0.0
            ckw[t]["rad_accum"] = "4He"
        elif t == "He3":
            ckw[t]["C_t"] = copy.deepcopy(C_in["H3"])
            ckw[t]["t_half"] = 12.34
            ckw[t]["rad_accum"] = "3He"
        elif t == "H3":
            ckw[t]["C_t"] = copy.deepcopy(C_in["H3"])
            ckw[t]["t_half"] = 12.34
    return okw, ckw, pkw
