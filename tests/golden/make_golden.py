#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ from the REFERENCE's own code.

Run in the build container only (needs /root/reference):

    python tests/golden/make_golden.py

It imports the reference modules utils/noble_gas_utils.py and
utils/convolution_integral_utils.py unmodified.  The latter needs two in-process shims
that do not touch any hot-path arithmetic: ``scipy.integrate.trapz/cumtrapz`` (removed in
SciPy >= 1.14; used only by the 'frac_inf_diff*' models) and a stub ``numba`` whose ``jit``
is the identity (numba is not installed; it decorates only the 'frac_inf_diff' helpers).
The reference never travels to the GPU box: only the .npz outputs below are committed.

Fixtures (all float64):
  ce_golden.npz      noble_gas_fun(...) outputs for 4096+ seeded (E, T, Ae, F[, P, S]).
  conv_golden.npz    tracer_conv_integral(...).convolve() for 5 tracers x 4 RTD models x
                     N in {1200, 25256} x seeded params + edge cases; gen_g_tp() vectors.
  fwd_golden.npz     ForwardMod compositions (BMM, thalf_cfc, lamsf6, sampled J) built
                     from the reference class per run_age_mcmc_utils.py:81-163.
  prep_golden.npz    ng_parse.He_comps and cfc_ce_corr / sf6_ce_corr outputs (prep-stage
                     ensemble propagation) for 2048 seeded members + branch edges.
  logp_golden.npz    per-walker log-probs of small CE / RTD / joint workloads: reference
                     forward models + scipy.stats log-densities.
  sf6acc_golden.npz  rad_accum='SF6' (J_sf6) convolutions and the post-convolve g_tp.

Every RTD fixture runs on the shipped input series of age_ens_runs_mcmc/C_in_dict.pk: the
package's data/atmos_series.npz is checked bit for bit against that pickle (read without
unpickling, tools/pickle_extract.py) before anything is generated.
"""
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.abspath(os.path.join(HERE, "..", ".."))
REF = os.environ.get("NGRTD_REFERENCE", "/root/reference")


def import_reference():
    import scipy.integrate as si
    if not hasattr(si, "trapz"):
        si.trapz = np.trapezoid
    if not hasattr(si, "cumtrapz"):
        si.cumtrapz = si.cumulative_trapezoid
    if "numba" not in sys.modules:
        nb = types.ModuleType("numba")
        nb.jit = lambda *a, **k: (lambda f: f)
        sys.modules["numba"] = nb
    sys.path.insert(0, os.path.join(REF, "utils"))
    import noble_gas_utils as ng  # noqa: E402
    import convolution_integral_utils as conv  # noqa: E402
    return ng, conv


GASES = ["He", "Ne", "Ar", "Kr", "Xe"]


def make_ce(ng):
    rng = np.random.default_rng(1001)
    n = 4096
    E = rng.uniform(0.0, 4000.0, n)
    T = rng.uniform(-5.0, 110.0, n)          # covers T<0 (-9999), T>=65 (no Setchenow), T>99
    Ae = 10 ** rng.uniform(-4, -1, n)
    F = 10 ** rng.uniform(-1, 1, n)
    # exact branch boundaries
    T[:8] = [0.0, -0.0, 65.0, 99.0, 64.999999, 99.000001, -1e-9, 1e-9]
    pmode = np.zeros(n, dtype=np.int32)      # 0 lapse_rate, 1 '1atm', 2 float
    P = np.zeros(n)
    S = np.zeros(n)
    pmode[256:512] = 1
    pmode[512:768] = 2
    P[512:768] = rng.uniform(0.6e-4, 1.1e-4, 256)
    S[768:1024] = rng.uniform(0.0, 1.0, 256)
    keys = ["ce_total", "ce_excess", "equil_dry", "equil", "solubility"]
    out = {k: np.zeros((n, 5)) for k in keys}
    out["vapor"] = np.zeros(n)
    out["P"] = np.zeros(n)
    for i in range(n):
        Parg = "lapse_rate" if pmode[i] == 0 else ("1atm" if pmode[i] == 1 else float(P[i]))
        o = ng.noble_gas_fun(gases=list(GASES), E=float(E[i]), T=float(T[i]), Ae=float(Ae[i]),
                             F=float(F[i]), P=Parg, S=float(S[i]))
        a = o.ce_exc(True)
        b = o.ce_exc(False)
        c = o.equil_conc_dry()
        d = o.equil_conc()
        for j, g in enumerate(GASES):
            out["ce_total"][i, j] = a[g]
            out["ce_excess"][i, j] = b[g]
            out["equil_dry"][i, j] = c[g]
            out["equil"][i, j] = d[g]
            out["solubility"][i, j] = o.solubility(g)
        out["vapor"][i] = o.vapor_pressure()
        out["P"][i] = o.P
    # ce_exc_wrapper (noble_gas_mcmc.py:205-213): theta=[log10 Ae, log10 F, E, T]
    m = 512
    th = np.stack([rng.uniform(-4, -1, m), rng.uniform(-1, 1, m), rng.uniform(2700, 3300, m),
                   rng.uniform(-3, 8, m)])
    wrap = np.zeros((m, 4))
    for i in range(m):
        Ae_, F_ = 10 ** th[0, i], 10 ** th[1, i]
        r = ng.noble_gas_fun(gases=["Ne", "Ar", "Kr", "Xe"], E=th[2, i], T=th[3, i], Ae=Ae_, F=F_,
                             P="lapse_rate").ce_exc(add_eq_conc=True)
        wrap[i] = [r[g] for g in ["Ne", "Ar", "Kr", "Xe"]]
    J = ng.J_flux(Del=1., rho_r=2700, rho_w=1000, U=3.0, Th=10.0, phi=0.05)
    J2 = ng.J_flux(Del=1., rho_r=2700, rho_w=1000, U=3.7, Th=10.2, phi=0.05)
    np.savez_compressed(os.path.join(HERE, "ce_golden.npz"), E=E, T=T, Ae=Ae, F=F, P_in=P, S=S,
                        pmode=pmode, wrap_theta=th, wrap_out=wrap, J_U3Th10=J, J_U37Th102=J2,
                        **out)


def reference_frame(series, n, col="x"):
    """Reference DataFrame layout of the last n ages of an age-first Series (the column is
    named after the tracer, as in C_in_dict: the 4He branch indexes C_t['He4_ter'], :323)."""
    import pandas as pd
    c = series.c_by_age[:n]
    return pd.DataFrame({col: np.flip(c)}, index=np.arange(n - 1, -1, -1))


TRACERS = {
    # name: (series, t_half, rad_accum, J)
    "CFC12": ("CFC12", False, False, False),
    "SF6": ("SF6", False, False, False),
    "H3": ("H3", 12.34, False, False),
    "He3": ("H3", 12.34, "3He", False),
    "He4_ter": ("He4_ter", False, "4He", 3.30885e-11),
}
MODS = ["piston", "exponential", "exp_pist_flow", "dispersion"]


def conv_params(rng, mod, n, k):
    tau = rng.uniform(1.0, 1000.0, k)
    if n > 2000:
        tau[: k // 4] = rng.uniform(1000.0, 15000.0, k // 4)
    eta = rng.uniform(1.0, 5.0, k)
    D = rng.uniform(0.01, 2.0, k)
    extra_tau, extra_eta = [], []
    if mod == "piston":
        extra_tau = [0.5, 0.500005, 1.5, 2.5, 10.5, 37.5, 0.2, 1e-6, n - 1.0, n - 0.5, n + 10.0, 0.0]
        extra_eta = [2.0] * len(extra_tau)
    if mod == "exp_pist_flow":
        # mask boundary tp >= tau*(1-1/eta): exact integers, eta=1 (all), empty tail
        extra_tau = [2.0, 20.0, 200.0, 37.3, 5.0, 1.0, 4.0 * (n + 5)]
        extra_eta = [2.0, 2.0, 2.0, 1.0, 5.0, 1.25, 4.0 / 3.0]
    t = np.concatenate([tau, extra_tau]) if len(extra_tau) else tau
    e = np.concatenate([eta, extra_eta]) if len(extra_eta) else eta
    d = np.concatenate([D, np.full(len(extra_tau), 0.5)]) if len(extra_tau) else D
    return t, e, d


def make_conv(conv):
    sys.path.insert(0, REPO)
    from noblegas_rtd_mcmc_amd.workloads import atmos_series
    rng = np.random.default_rng(2002)
    out = {}
    for n in (1200, 25256):
        for tname, (sname, t_half, accum, J) in TRACERS.items():
            s = atmos_series(sname, n)
            if tname == "He4_ter":
                s.c_by_age = s.c_by_age * 0.0
            df = reference_frame(s, n, tname)
            for mod in MODS:
                k = 48 if n > 2000 else 64
                tau, eta, D = conv_params(rng, mod, n, k)
                res = np.zeros(len(tau))
                for i in range(len(tau)):
                    cm = conv.tracer_conv_integral(df.copy(), df.copy().index[-1])
                    cm.update_pars(tau=float(tau[i]), mod_type=mod, t_half=t_half, rad_accum=accum,
                                   J=J, eta=float(eta[i]), D=float(D[i]), bbar=False, Phi_im=False)
                    res[i] = cm.convolve()
                key = "%s_%s_%d" % (tname, mod, n)
                out[key + "_tau"] = tau
                out[key + "_eta"] = eta
                out[key + "_D"] = D
                out[key + "_out"] = res
    # t_samp shifted past the last index (dtp = floor(3.7) = 3)
    s = atmos_series("CFC12", 1200)
    df = reference_frame(s, 1200)
    for mod in MODS:
        tau, eta, D = conv_params(rng, mod, 1200, 16)
        res = np.zeros(len(tau))
        for i in range(len(tau)):
            cm = conv.tracer_conv_integral(df.copy(), df.index[-1] + 3.7)
            cm.update_pars(tau=float(tau[i]), mod_type=mod, eta=float(eta[i]), D=float(D[i]))
            res[i] = cm.convolve()
        key = "shift_%s" % mod
        out[key + "_tau"], out[key + "_eta"], out[key + "_D"], out[key + "_out"] = tau, eta, D, res
    # gen_g_tp vectors (N=1200, CFC12 series)
    gs = []
    gp = []
    for mod in MODS:
        for (tau, eta, D) in [(37.3, 2.0, 0.3), (500.0, 1.5, 1.2), (3.2, 4.0, 0.05)]:
            cm = conv.tracer_conv_integral(df.copy(), df.index[-1])
            cm.update_pars(tau=tau, mod_type=mod, eta=eta, D=D)
            gs.append(cm.gen_g_tp())
            gp.append([MODS.index(mod), tau, eta, D])
    out["gtp_params"] = np.array(gp)
    out["gtp"] = np.array(gs)
    # convolve(g_tau=...) with an externally supplied weight vector
    g_ext = rng.uniform(0.0, 1.0, 1200)
    g_ext /= g_ext.sum()
    cm = conv.tracer_conv_integral(df.copy(), df.index[-1])
    cm.update_pars(tau=10.0, mod_type="exponential", t_half=12.34)
    out["gext"] = g_ext
    out["gext_out"] = np.array(cm.convolve(g_tau=g_ext))
    np.savez_compressed(os.path.join(HERE, "conv_golden.npz"), **out)


def ref_forward_mod(conv, ng, tracer, C_t, mod_type1, mod_type2, t_half, rad_accum, par_names, theta):
    """ForwardMod.perform (run_age_mcmc_utils.py:81-163) composed from the reference class."""
    p = {"tau1": False, "tau2": 0.0, "f1": 1.0, "f2": 0.0, "eta1": False, "eta2": False,
         "D1": False, "D2": False, "J": False, "thalf_cfc": False, "lamsf6": False}
    for i in range(len(par_names)):
        p[par_names[i]] = theta[i]
    if tracer == "He4_ter" and p["J"] == False:  # noqa: E712
        p["J"] = np.log10(ng.J_flux(Del=1., rho_r=2700, rho_w=1000, U=3.0, Th=10.0, phi=0.05))
    cm = conv.tracer_conv_integral(C_t.copy(), C_t.copy().index[-1])
    cm.update_pars(tau=p["tau1"], mod_type=mod_type1, t_half=t_half, rad_accum=rad_accum,
                   J=10 ** p["J"], eta=p["eta1"], D=p["D1"], bbar=False, Phi_im=False)
    if "thalf_cfc" in par_names and tracer == "CFC12":
        cm.t_half = p["thalf_cfc"]
        cm.thalf_2_lambda(p["thalf_cfc"])
    cout1 = cm.convolve()
    cout2 = 0.0
    if mod_type2:
        cm2 = conv.tracer_conv_integral(C_t.copy(), C_t.copy().index[-1])
        cm2.update_pars(tau=p["tau2"], mod_type=mod_type2, t_half=t_half, rad_accum=rad_accum,
                        J=10 ** p["J"], eta=p["eta2"], D=p["D2"], bbar=False, Phi_im=False)
        if "thalf_cfc" in par_names and tracer == "CFC12":
            cm2.t_half = p["thalf_cfc"]
            cm2.thalf_2_lambda(p["thalf_cfc"])
        cout2 = cm2.convolve()
    cout = p["f1"] * cout1 + p["f2"] * cout2
    if tracer == "SF6" and "lamsf6" in p:
        cout *= (1 + p["lamsf6"])
    return float(cout)


FWD_CASES = [
    # (name, mod1, mod2, par_names)
    ("exp_J_thalf_lamsf6", "exponential", False, ["tau1", "J", "thalf_cfc", "lamsf6"]),
    ("epm", "exp_pist_flow", False, ["tau1", "eta1"]),
    ("disp", "dispersion", False, ["tau1", "D1"]),
    ("bmm_exp_piston", "exponential", "piston", ["tau1", "tau2", "f1", "f2"]),
    ("bmm_epm_piston", "exp_pist_flow", "piston", ["tau1", "tau2", "f1", "f2", "eta1"]),
    ("bmm_disp_exp", "dispersion", "exponential", ["tau1", "tau2", "f1", "f2", "D1"]),
    ("bmm_exp_epm", "exponential", "exp_pist_flow", ["tau1", "tau2", "f1", "f2", "eta2"]),
]


def fwd_theta(rng, par_names, k):
    cols = []
    f1 = rng.uniform(0.01, 0.99, k)
    for p in par_names:
        cols.append({"tau1": rng.uniform(1, 1000, k), "tau2": rng.uniform(50, 15000, k), "f1": f1,
                     "f2": 1 - f1, "eta1": rng.uniform(1, 5, k), "eta2": rng.uniform(1, 5, k),
                     "D1": rng.uniform(0.01, 2, k), "D2": rng.uniform(0.01, 2, k),
                     "J": rng.normal(-10.424, 0.33, k), "thalf_cfc": rng.uniform(5, 35, k),
                     "lamsf6": np.abs(rng.normal(0, 1 / 6, k))}[p])
    return np.stack(cols, axis=1)


def make_fwd(conv, ng):
    sys.path.insert(0, REPO)
    from noblegas_rtd_mcmc_amd.workloads import atmos_series
    rng = np.random.default_rng(3003)
    out = {}
    n = 1200
    for name, m1, m2, pn in FWD_CASES:
        th = fwd_theta(rng, pn, 24)
        out[name + "_theta"] = th
        for tname, (sname, t_half, accum, _) in TRACERS.items():
            s = atmos_series(sname, n)
            if tname == "He4_ter":
                s.c_by_age = s.c_by_age * 0.0
            df = reference_frame(s, n, tname)
            res = np.array([ref_forward_mod(conv, ng, tname, df, m1, m2, t_half, accum, pn, th[i])
                            for i in range(len(th))])
            out["%s_%s" % (name, tname)] = res
    np.savez_compressed(os.path.join(HERE, "fwd_golden.npz"), **out)


def ref_logp_units(conv, ng, spec, theta_soa):
    """Reference forward models + scipy.stats densities, per walker."""
    from scipy import stats
    L, W = spec.n_wells, theta_soa.shape[2]
    out = np.zeros(W)
    for w in range(W):
        tot = 0.0
        for l in range(L):
            p = {r: theta_soa[i, l, w] for i, r in enumerate(spec.roles)}
            if spec.ce is not None:
                c = spec.ce
                tot += (stats.beta.logpdf(p["Ae_beta"], *c.beta_Ae) + stats.beta.logpdf(p["F_beta"], *c.beta_F)
                        + stats.beta.logpdf(p["E_beta"], *c.beta_E) + stats.norm.logpdf(p["m"], c.m_mu, c.m_sd)
                        + stats.beta.logpdf(p["b_beta"], *c.beta_b) + stats.beta.logpdf(p["nu_ce_beta"], *c.beta_nu))
                Ae = p["Ae_beta"] * (c.logA_max - c.logA_min) + c.logA_min
                F = p["F_beta"] * (c.logF_max - c.logF_min) + c.logF_min
                E = p["E_beta"] * (c.E_max - c.E_min[l]) + c.E_min[l]
                b = p["b_beta"] * (c.b_max - c.b_min) + c.b_min
                T = (E - b) / p["m"]
                nu = p["nu_ce_beta"] * (c.nu_max - c.nu_min) + c.nu_min
                r = ng.noble_gas_fun(gases=list(c.gases), E=E, T=T, Ae=10 ** Ae, F=10 ** F,
                                     P="lapse_rate").ce_exc(add_eq_conc=True)
                mod = np.array([r[g] for g in c.gases])
                tot += np.sum(stats.t.logpdf(c.obs[l], nu, loc=mod, scale=c.sd[l]))
            if spec.rtd is not None:
                r_ = spec.rtd
                tot += stats.uniform.logpdf(p["tau1"], r_.tau1[0], r_.tau1[1] - r_.tau1[0])
                tot += stats.beta.logpdf(p["nu_rtd_beta"], *r_.beta_nu)
                pn, vals = [], []
                for name in r_.par_names:
                    if name == "J":
                        tot += stats.norm.logpdf(p["J"], r_.J_mu, r_.J_sd)
                        v = p["J"]
                    elif name == "thalf_cfc":
                        tot += stats.beta.logpdf(p["thalf_cfc_beta"], *r_.beta_thalf)
                        v = p["thalf_cfc_beta"] * (r_.thalf[1] - r_.thalf[0]) + r_.thalf[0]
                    elif name == "lamsf6":
                        tot += stats.halfnorm.logpdf(p["lamsf6"], scale=r_.lamsf6_sd)
                        v = p["lamsf6"]
                    elif name == "tau1":
                        v = p["tau1"]
                    else:
                        lo, hi = getattr(r_, name)
                        tot += stats.uniform.logpdf(p[name], lo, hi - lo)
                        v = p[name]
                    pn.append(name)
                    vals.append(v)
                    if name == "f1":
                        pn.append("f2")
                        vals.append(1 - v)
                nu = p["nu_rtd_beta"] * (r_.nu_max - r_.nu_min) + r_.nu_min
                mods = []
                for t in r_.tracers:
                    cv, ci, _ = t.series.reference_frame()
                    import pandas as pd
                    df = pd.DataFrame({t.name: cv}, index=ci.astype(np.int64))
                    pn_t, vals_t = list(pn), list(vals)
                    mods.append(ref_forward_mod(conv, ng, t.name, df, r_.mod_type1, r_.mod_type2 or False,
                                                t.t_half or False, t.rad_accum or False, pn_t, vals_t))
                tot += np.sum(stats.t.logpdf(r_.obs[l], nu, loc=np.array(mods), scale=r_.sd[l]))
        out[w] = tot
    return out


def spec_arrays(prefix, spec, theta):
    """Everything needed to rebuild the ModelSpec without the package's data files."""
    d = {prefix + "_theta": theta, prefix + "_L": np.array(spec.n_wells)}
    if spec.ce is not None:
        d[prefix + "_ce_obs"] = spec.ce.obs
        d[prefix + "_ce_sd"] = spec.ce.sd
        d[prefix + "_ce_Emin"] = spec.ce.E_min
        d[prefix + "_ce_gases"] = np.array(spec.ce.gases)
    if spec.rtd is not None:
        r = spec.rtd
        d[prefix + "_rtd_obs"] = r.obs
        d[prefix + "_rtd_sd"] = r.sd
        d[prefix + "_rtd_tracers"] = np.array([t.name for t in r.tracers])
        d[prefix + "_rtd_series"] = np.stack([t.series.c_by_age for t in r.tracers])
        d[prefix + "_rtd_mods"] = np.array([r.mod_type1, r.mod_type2 or ""])
        d[prefix + "_rtd_par_names"] = np.array(list(r.par_names))
    return d


def make_logp(conv, ng):
    sys.path.insert(0, REPO)
    from noblegas_rtd_mcmc_amd import workloads as wl
    out = {}
    spec, th = wl.c2(W=48)
    out.update(spec_arrays("c2", spec, th))
    out["c2_logp"] = ref_logp_units(conv, ng, spec, th)
    spec, th = wl.c3(W=48)
    out.update(spec_arrays("c3", spec, th))
    out["c3_logp"] = ref_logp_units(conv, ng, spec, th)
    spec = wl.c4_spec(L=4, N=1200)
    th = wl.sample_prior(spec, 12, np.random.default_rng(77))
    out.update(spec_arrays("c4", spec, th))
    out["c4_logp"] = ref_logp_units(conv, ng, spec, th)
    spec = wl.c4_spec(L=2, N=1200, mod_type1="exp_pist_flow", mod_type2="piston",
                      par_names=("tau1", "tau2", "f1", "eta1", "thalf_cfc", "lamsf6"))
    th = wl.sample_prior(spec, 8, np.random.default_rng(78))
    out.update(spec_arrays("bmm", spec, th))
    out["bmm_logp"] = ref_logp_units(conv, ng, spec, th)
    np.savez_compressed(os.path.join(HERE, "logp_golden.npz"), **out)


def make_prep(ng):
    """ng_parse.He_comps (noble_gas_utils.py:394-422) and cfc_utils.cfc_ce_corr /
    sf6_ce_corr (cfc_utils.py:25-306), one reference object per member as
    age_modeling_mcmc.prep.py:247-397 builds them."""
    sys.path.insert(0, os.path.join(REF, "utils"))
    import cfc_utils  # noqa: E402
    rng = np.random.default_rng(2002)
    n = 2048
    E = rng.uniform(2500.0, 3400.0, n)
    T = rng.uniform(-3.0, 20.0, n)
    Ae = 10 ** rng.uniform(-4, -1, n)
    F = rng.uniform(0.0, 1.0, n)
    T[:6] = [0.0, -0.5, 99.0, 99.5, 65.0, 120.0]     # T<0 sentinel, Antoine / Setchenow branches
    He4 = rng.normal(6.0e-8, 2.0e-8, n)
    He3 = rng.normal(1.0e-13, 3.0e-14, n)
    Rterr = 10 ** (rng.beta(2, 2, n) * 2.0 + np.log10(2.e-8) - 1.0)
    he = np.zeros((5, n))
    keys = ["He4_eq", "He4_atm", "He4_ter", "He4_del", "He3_tu"]
    for i in range(n):
        ngp = ng.ng_parse({"He4": float(He4[i]), "He3": float(He3[i])}, float(Ae[i]), float(F[i]),
                          float(E[i]), float(T[i]))
        ngp.He_comps(float(Rterr[i]))
        he[:, i] = [ngp.obs_dict_[k] for k in keys]
    S = np.zeros(n)
    S[1024:1280] = rng.uniform(0.0, 35.0, 256)
    cmeas = np.stack([rng.lognormal(np.log(2.5), 0.3, n), rng.lognormal(np.log(1.2), 0.3, n),
                      rng.lognormal(np.log(0.25), 0.3, n)])
    sf6_meas = rng.lognormal(np.log(1.5), 0.3, n)
    z_in = np.stack([rng.uniform(200, 300, n), rng.uniform(400, 550, n), rng.uniform(60, 90, n)])
    sf6_z = rng.uniform(2, 12, n)
    out = dict(E=E, T=T, Ae=Ae, F=F, He4=He4, He3=He3, Rterr=Rterr, he=he, S=S, cmeas=cmeas,
               sf6_meas=sf6_meas, z_in=z_in, sf6_z=sf6_z)
    res = {k: np.zeros((3, n)) for k in ("cfc_air", "cfc_aq", "cfc_exc", "cfc_sol")}
    res.update({k: np.zeros(n) for k in ("sf6_air", "sf6_aq", "sf6_exc", "sf6_sol", "pv_atm", "p_atm")})
    for i in range(n):
        c = cfc_utils.cfc_ce_corr(cfc_num=[11, 12, 113], E=float(E[i]), T=float(T[i]), Ae=float(Ae[i]),
                                  F=float(F[i]), S=float(S[i]))
        res["cfc_air"][:, i] = c.equil_air_conc_cfc(cmeas[:, i].copy())    # sets self.P
        res["cfc_aq"][:, i] = c.equil_aq_conc_cfc(z_in[:, i].copy())
        res["cfc_exc"][:, i] = c.ce_exc_conc_cfc(z_in[:, i].copy())
        res["cfc_sol"][:, i] = c.solubility_cfc()
        res["pv_atm"][i] = c.vapor_pressure_atm()
        res["p_atm"][i] = c.lapse_rate_atm()
        s6 = cfc_utils.sf6_ce_corr(E=float(E[i]), T=float(T[i]), Ae=float(Ae[i]), F=float(F[i]), S=float(S[i]))
        res["sf6_air"][i] = s6.equil_air_conc_sf6(float(sf6_meas[i]))
        res["sf6_aq"][i] = s6.equil_aq_conc_sf6(float(sf6_z[i]))
        res["sf6_exc"][i] = s6.ce_exc_conc_sf6(float(sf6_z[i]))
        res["sf6_sol"][i] = s6.solubility_sf6()
    out.update(res)
    np.savez_compressed(os.path.join(HERE, "prep_golden.npz"), **out)


def make_frac(conv):
    """'frac_inf_diff' (convolution_integral_utils.py:238-266): gen_g_tp() weights, FM_mu and
    convolve() of the reference class, with the dispersion advective RTD
    (frac_rtd_numba_disp) and with an external one (f_tadv_ext, frac_rtd_numba).
    Parameter ranges: aux_scripts/age_modeling_mcmc.rtd_explore.py:257-258 (bbar, Phi_im)."""
    sys.path.insert(0, REPO)
    from noblegas_rtd_mcmc_amd.workloads import atmos_series
    rng = np.random.default_rng(4004)
    out = {}
    k = 16
    tau = rng.uniform(2.0, 800.0, k)
    D = rng.uniform(0.01, 2.0, k)
    bbar = 10 ** rng.uniform(-5, -2, k)
    Phi = rng.uniform(0.005, 0.05, k)
    out.update(tau=tau, D=D, bbar=bbar, Phi=Phi)
    for n in (300, 1200):
        gs, fms = np.zeros((k, n)), np.zeros(k)
        for tname, (sname, t_half, accum, J) in TRACERS.items():
            s = atmos_series(sname, n)
            if tname == "He4_ter":
                s.c_by_age = s.c_by_age * 0.0
            df = reference_frame(s, n, tname)
            res = np.zeros(k)
            for i in range(k):
                cm = conv.tracer_conv_integral(df.copy(), df.copy().index[-1])
                cm.update_pars(tau=float(tau[i]), mod_type="frac_inf_diff", t_half=t_half, rad_accum=accum, J=J,
                               D=float(D[i]), bbar=float(bbar[i]), Phi_im=float(Phi[i]))
                res[i] = cm.convolve()
                if tname == "CFC12":
                    gs[i] = cm.g_tp
                    fms[i] = cm.FM_mu
            out["conc_%s_%d" % (tname, n)] = res
        out["g_%d" % n] = gs
        out["fm_%d" % n] = fms
    # external advective RTD (frac_rtd_numba): exponential / dispersion weights of the reference
    n = 600
    s = atmos_series("H3", n)
    df = reference_frame(s, n, "H3")
    ext, ke = [], 6
    for i in range(ke):
        cm = conv.tracer_conv_integral(df.copy(), df.index[-1])
        cm.update_pars(tau=float(tau[i]), mod_type="exponential" if i % 2 else "dispersion", D=float(D[i]))
        ext.append(cm.gen_g_tp())
    ext = np.array(ext)
    res, gs, fms = np.zeros(ke), np.zeros((ke, n)), np.zeros(ke)
    for i in range(ke):
        cm = conv.tracer_conv_integral(df.copy(), df.index[-1])
        cm.update_pars(tau=float(tau[i]), mod_type="frac_inf_diff", t_half=12.34, bbar=float(bbar[i]),
                       Phi_im=float(Phi[i]), f_tadv_ext=ext[i].copy())
        res[i] = cm.convolve()
        gs[i], fms[i] = cm.g_tp, cm.FM_mu
    out.update(ext=ext, ext_conc=res, ext_g=gs, ext_fm=fms)
    # sampling date past the last index (dtp = floor(3.7) = 3, :172-173) and the shortest
    # series the integral is defined on (N = 2)
    for key, n, tsh in (("shift", 300, 3.7), ("n2", 2, 0.0)):
        s = atmos_series("H3", n)
        df = reference_frame(s, n, "H3")
        res, fms = np.zeros(4), np.zeros(4)
        for i in range(4):
            cm = conv.tracer_conv_integral(df.copy(), df.index[-1] + tsh)
            cm.update_pars(tau=float(tau[i]), mod_type="frac_inf_diff", t_half=12.34, D=float(D[i]),
                           bbar=float(bbar[i]), Phi_im=float(Phi[i]))
            res[i] = cm.convolve()
            fms[i] = cm.FM_mu
        out[key + "_conc"], out[key + "_fm"] = res, fms
    # one long series (N = 25256, the shipped C_in_dict length)
    n = 25256
    s = atmos_series("CFC12", n)
    df = reference_frame(s, n, "CFC12")
    cm = conv.tracer_conv_integral(df.copy(), df.index[-1])
    cm.update_pars(tau=1500.0, mod_type="frac_inf_diff", D=0.5, bbar=3e-4, Phi_im=0.02)
    out["long_conc"] = np.array(cm.convolve())
    out["long_fm"] = np.array(cm.FM_mu)
    out["long_g_head"] = cm.g_tp[:2000].copy()
    np.savez_compressed(os.path.join(HERE, "frac_golden.npz"), **out)


def check_shipped_series():
    """The package's series ARE the shipped C_in_dict.pk series, bit for bit (read without
    unpickling by tools/pickle_extract.py), so every fixture below runs the reference's
    code on the reference's own inputs."""
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "tools"))
    from pickle_extract import read_frame_dict
    from noblegas_rtd_mcmc_amd.workloads import atmos_series
    frames = read_frame_dict(os.path.join(REF, "age_ens_runs_mcmc", "C_in_dict.pk"))
    for key, fr in frames.items():
        v = np.flip(fr["values"][0])
        got = atmos_series(key).c_by_age
        if not np.array_equal(got.view(np.int64), v.view(np.int64)):
            raise SystemExit("package series %s differs from C_in_dict.pk" % key)


def make_sf6_accum(conv):
    """rad_accum='SF6' (zero-order SF6 contamination, convolution_integral_utils.py:329-331):
    C_t['SF6'] + index * J_sf6, with J_sf6 a numpy float (the reference calls .copy())."""
    sys.path.insert(0, REPO)
    from noblegas_rtd_mcmc_amd.workloads import atmos_series
    rng = np.random.default_rng(2003)
    out = {}
    for n in (1200, 25256):
        s = atmos_series("SF6", n)
        df = reference_frame(s, n, "SF6")
        for mod in MODS:
            tau, eta, D = conv_params(rng, mod, n, 16)
            Js = rng.uniform(0.0, 0.05, len(tau))
            res = np.zeros(len(tau))
            for i in range(len(tau)):
                cm = conv.tracer_conv_integral(df.copy(), df.copy().index[-1])
                cm.update_pars(tau=float(tau[i]), mod_type=mod, rad_accum="SF6", J_sf6=np.float64(Js[i]),
                               eta=float(eta[i]), D=float(D[i]))
                res[i] = cm.convolve()
            key = "sf6acc_%s_%d" % (mod, n)
            out[key + "_tau"], out[key + "_eta"], out[key + "_D"] = tau, eta, D
            out[key + "_J"], out[key + "_out"] = Js, res
    # g_tp after convolve() is the DECAYED weight vector (:313-316): H3 exponential
    s = atmos_series("H3", 1200)
    df = reference_frame(s, 1200, "H3")
    gt = []
    for tau in (3.0, 37.3, 480.0):
        cm = conv.tracer_conv_integral(df.copy(), df.index[-1])
        cm.update_pars(tau=tau, mod_type="exponential", t_half=12.34)
        cm.convolve()
        gt.append(cm.g_tp.copy())
    out["gtp_after_conv_tau"] = np.array([3.0, 37.3, 480.0])
    out["gtp_after_conv"] = np.array(gt)
    np.savez_compressed(os.path.join(HERE, "sf6acc_golden.npz"), **out)


def main():
    ng, conv = import_reference()
    check_shipped_series()
    which = sys.argv[1:] or ["ce", "conv", "fwd", "logp", "prep", "frac", "sf6acc"]
    if "sf6acc" in which:
        make_sf6_accum(conv)
    if "frac" in which:
        make_frac(conv)
    if "prep" in which:
        make_prep(ng)
    if "ce" in which:
        make_ce(ng)
    if "conv" in which:
        make_conv(conv)
    if "fwd" in which:
        make_fwd(conv, ng)
    if "logp" in which:
        make_logp(conv, ng)


if __name__ == "__main__":
    main()
