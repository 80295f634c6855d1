"""Vectorised NumPy variant of the per-walker log-prob (oracle/models.py).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py): the second CPU baseline SURVEY.md §8d
asks for beside the reference-faithful per-walker loop -- the same arithmetic as the
reference, but every walker of a well at once: the CE model on [W] arrays
(utils/noble_gas_utils.py:103-253, oracle/ce.py), the RTD weights of
convolution_integral_utils.py:168-196 as a [W][N] matrix, the normalisation g / g.sum()
(:270) per row, the decay / accumulation of :305-333 and the dot with the flipped series
(:336-337) as one matrix-vector product per tracer, then the PyMC3 log densities
(oracle/stats.py).  Agrees with models.log_prob to ~1e-15 relative (different summation
order of the dot product); tests/test_oracle_golden.py checks it at rtol 1e-12.
"""
import numpy as np

from . import ce as _ce
from . import rtd as _rtd
from . import stats as _st


def gen_g_tp_batch(n, index_last, t_samp, tau, mod_type, eta=None, D=None):
    """gen_g_tp (:155-270) for parameter arrays tau/eta/D [W] -> normalised g [W][N]."""
    tp = _rtd.age_grid(n, index_last, t_samp)
    tau = np.asarray(tau, dtype=np.float64)[:, None]
    with np.errstate(all="ignore"):
        if mod_type == "piston":
            g = np.zeros((tau.shape[0], n))
            ix = np.abs(tp[None, :] - tau).argmin(axis=1)          # first minimum, :180
            g[np.arange(tau.shape[0]), ix] = 1.0
        elif mod_type == "exponential":
            g = (1. / tau) * np.exp(-tp[None, :] / tau)
        elif mod_type == "exp_pist_flow":
            eta = np.asarray(eta, dtype=np.float64)[:, None]
            mask = tp[None, :] >= tau * (1 - (1 / eta))
            val = (eta / tau) * np.exp(-(eta * tp[None, :] / tau) + eta - 1.)
            g = np.where(mask, val, 0.0)
        elif mod_type == "dispersion":
            D = np.asarray(D, dtype=np.float64)[:, None]
            f1 = (1. / tau) / (np.sqrt(4. * np.pi * D * (tp[None, :] / tau)))
            f2 = (1. / (tp[None, :] / tau)) * np.exp(-1. * (((1. - (tp[None, :] / tau)) ** 2)
                                                             / (4. * D * (tp[None, :] / tau))))
            g = f1 * f2
        else:
            raise ValueError(mod_type)
        return g / g.sum(axis=1, keepdims=True)


def convolve_batch(t, tau, mod_type, lamba, eta=None, D=None, J=None):
    """convolve (:284-340) of tracer ``t`` (spec.Tracer) for parameter arrays [W]."""
    cv, ci, t_samp = t.series.reference_frame()
    n = len(cv)
    g = gen_g_tp_batch(n, ci[-1], t_samp, tau, mod_type, eta, D)
    tp = _rtd.age_grid(n, ci[-1], t_samp)
    lam = np.asarray(lamba, dtype=np.float64)
    lam = lam[:, None] if lam.ndim else lam
    with np.errstate(all="ignore"):
        if t.rad_accum == "3He":
            g = g * (1 - np.exp(-lam * tp))
        else:
            g = g * np.exp(-lam * tp)
        if t.rad_accum == "4He":
            Jv = np.asarray(J, dtype=np.float64)
            C = cv[None, :] + ci[None, :] * (Jv[:, None] if Jv.ndim else Jv)
            return np.einsum("wn,wn->w", np.flip(C, axis=1), g)
        if t.rad_accum == "SF6":
            C = cv + ci * t.J_sf6
        else:
            C = cv
        return g @ np.flip(C)


def _beta(x, ab, jac):
    """Beta prior (+ the logodds transform's log|J| for the transformed-space log-prob, as
    models._beta_lp)."""
    return _st.beta_logp(x, ab[0], ab[1]) + (_st.jac_logodds(x) if jac else 0.0)


def _unif(x, lohi, jac):
    return _st.uniform_logp(x, lohi[0], lohi[1]) + (_st.jac_interval(x, lohi[0], lohi[1]) if jac else 0.0)


def log_prob_vec(spec, theta_soa):
    """Per-walker log-prob for theta SoA [P][L][W], vectorised over walkers (with the PyMC3
    transform Jacobians when spec.jacobian, as models.log_prob)."""
    theta_soa = np.asarray(theta_soa, dtype=np.float64)
    P, L, W = theta_soa.shape
    jac = spec.jacobian
    lp = np.zeros(W)
    for l in range(L):
        p = {role: theta_soa[i, l] for i, role in enumerate(spec.roles)}
        if spec.ce is not None:
            c = spec.ce
            if spec.include_prior:
                lp = lp + _beta(p["Ae_beta"], c.beta_Ae, jac)
                lp = lp + _beta(p["F_beta"], c.beta_F, jac)
                lp = lp + _beta(p["E_beta"], c.beta_E, jac)
                lp = lp + _st.normal_logp(p["m"], c.m_mu, c.m_sd)
                lp = lp + _beta(p["b_beta"], c.beta_b, jac)
                lp = lp + _beta(p["nu_ce_beta"], c.beta_nu, jac)
            if spec.include_like:
                Ae = p["Ae_beta"] * (c.logA_max - c.logA_min) + c.logA_min
                F = p["F_beta"] * (c.logF_max - c.logF_min) + c.logF_min
                E = p["E_beta"] * (c.E_max - c.E_min[l]) + c.E_min[l]
                b = p["b_beta"] * (c.b_max - c.b_min) + c.b_min
                with np.errstate(all="ignore"):
                    T = (E - b) / p["m"]
                nu = p["nu_ce_beta"] * (c.nu_max - c.nu_min) + c.nu_min
                mod = _ce.ce_exc_wrapper([Ae, F, E, T], gases=c.gases)          # [G][W]
                lp = lp + np.sum(_st.studentt_logp(c.obs[l][:, None], mod, c.sd[l][:, None], nu[None, :]), axis=0)
        if spec.rtd is not None:
            r = spec.rtd
            names = r.par_names
            if spec.include_prior:
                lp = lp + _unif(p["tau1"], r.tau1, jac)
                lp = lp + _beta(p["nu_rtd_beta"], r.beta_nu, jac)
                for nm in ("tau2", "f1", "eta1", "eta2", "D1", "D2"):
                    if nm in names:
                        lp = lp + _unif(p[nm], getattr(r, nm), jac)
                if "J" in names:
                    lp = lp + _st.normal_logp(p["J"], r.J_mu, r.J_sd)
                if "thalf_cfc" in names:
                    lp = lp + _beta(p["thalf_cfc_beta"], r.beta_thalf, jac)
                if "lamsf6" in names:
                    lp = lp + _st.halfnormal_logp(p["lamsf6"], r.lamsf6_sd) + (_st.jac_log(p["lamsf6"]) if jac else 0.0)
            if spec.include_like:
                nu = p["nu_rtd_beta"] * (r.nu_max - r.nu_min) + r.nu_min
                f1 = p["f1"] if "f1" in names else 1.0
                f2 = 1 - p["f1"] if "f1" in names else 0.0
                mods = []
                for t in r.tracers:
                    lam = _rtd.thalf_2_lambda(t.t_half) if t.t_half else 0.0
                    if "thalf_cfc" in names and t.name == "CFC12":
                        lam = _rtd.thalf_2_lambda(p["thalf_cfc_beta"] * (r.thalf[1] - r.thalf[0]) + r.thalf[0])
                    if "J" in names:
                        J = 10 ** p["J"]
                    elif t.name == "He4_ter":
                        J = 10 ** (t.log10_J if t.log10_J is not None else _rtd.J_he4_default())
                    else:
                        J = 10 ** 0.0 if t.log10_J is None else 10 ** t.log10_J
                    c1 = convolve_batch(t, p["tau1"], r.mod_type1, lam, p.get("eta1"), p.get("D1"), J)
                    c = f1 * c1
                    if r.mod_type2:
                        c = c + f2 * convolve_batch(t, p["tau2"], r.mod_type2, lam, p.get("eta2"), p.get("D2"), J)
                    else:
                        c = c + f2 * 0.0
                    if t.name == "SF6":
                        c = c * (1 + (p["lamsf6"] if "lamsf6" in names else False))
                    mods.append(c)
                mod = np.stack(mods)                                                # [K][W]
                lp = lp + np.sum(_st.studentt_logp(r.obs[l][:, None], mod, r.sd[l][:, None], nu[None, :]), axis=0)
    return lp
