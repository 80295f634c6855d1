"""NumPy restatement of the lumped-parameter RTD convolution integral.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  Follows
utils/convolution_integral_utils.py (class tracer_conv_integral, :105-340) and the
ForwardMod composition of age_ens_runs_mcmc/run_age_mcmc_utils.py:81-163 literally:
build the full weight vector g(tp), normalise by its sum, apply decay/accumulation,
flip the input series and take the dot product.  One call = one (walker, well, tracer).
"""
import numpy as np


def thalf_2_lambda(t_half):
    """convolution_integral_utils.py:146-152."""
    return -1 * np.log(0.5) / t_half


def age_grid(n, index_last, t_samp):
    """convolution_integral_utils.py:168-174 (and :307-311, identical)."""
    tp = np.arange(0, n).astype(float)
    tp[0] += 1e-5
    dtp = np.floor(t_samp - index_last)
    tp += dtp
    return tp


def gen_g_tp(n, index_last, t_samp, tau, mod_type, eta=None, D=None):
    """convolution_integral_utils.py:155-281 for piston / exponential / exp_pist_flow /
    dispersion, normalised by the discrete sum (:270)."""
    tp = age_grid(n, index_last, t_samp)
    # the reference receives its parameters as numpy float64 (theano dvector elements,
    # run_age_mcmc_utils.py:84-85): 1/0 is inf (with a warning), never ZeroDivisionError
    tau = np.float64(tau)
    with np.errstate(all="ignore"):
        if mod_type == "piston":
            g_tp = np.zeros(len(tp))
            ix = abs(tp - tau).argmin()
            g_tp[ix] = 1.
        elif mod_type == "exponential":
            g_tp = (1. / tau) * np.exp(-tp / tau)
        elif mod_type == "exp_pist_flow":
            g_tp = np.zeros(len(tp))
            exp_mask = tp >= tau * (1 - (1 / eta))
            g_tp[exp_mask] = (eta / tau) * np.exp(-(eta * tp[exp_mask] / tau) + eta - 1.)
        elif mod_type == "dispersion":
            f1 = (1. / tau) / (np.sqrt(4. * np.pi * D * (tp / tau)))
            f2 = (1. / (tp / tau)) * np.exp(-1. * (((1. - (tp / tau)) ** 2) / (4. * D * (tp / tau))))
            g_tp = f1 * f2
        else:
            raise ValueError("unsupported mod_type %r" % (mod_type,))
        g_tp = g_tp / g_tp.sum()
    return g_tp


def convolve(c_values, index_values, t_samp, tau, mod_type, lamba=0.0, rad_accum=False,
             J=False, eta=None, D=None, J_sf6=None, g_tau=None):
    """convolution_integral_utils.py:284-340.

    ``c_values``/``index_values`` are the C_t column and index in DataFrame order
    (oldest age first, index[-1] = most recent), exactly as the reference holds them.
    """
    c_values = np.asarray(c_values, dtype=np.float64)
    index_values = np.asarray(index_values)
    n = len(c_values)
    g = gen_g_tp(n, index_values[-1], t_samp, tau, mod_type, eta, D) if g_tau is None else np.asarray(g_tau)
    tp = age_grid(n, index_values[-1], t_samp)
    with np.errstate(all="ignore"):
        if rad_accum == "3He":
            g = g * (1 - np.exp(-lamba * tp))
        else:
            g = g * np.exp(-lamba * tp)
        if rad_accum == "4He":
            C = c_values + index_values * J
        elif rad_accum == "SF6":
            C = c_values + index_values * J_sf6
        else:
            C = c_values
        return float(np.dot(np.flip(C), g))


def J_he4_default():
    """run_age_mcmc_utils.py:90-91: log10 J_flux(U=3, Th=10)."""
    from .ce import J_flux
    return np.log10(J_flux(Del=1., rho_r=2700, rho_w=1000, U=3.0, Th=10.0, phi=0.05))


def forward_mod(tracer, conv_kwgs, par_names, theta):
    """ForwardMod.perform (run_age_mcmc_utils.py:81-163) for one tracer.

    conv_kwgs: dict with C_values, C_index, mod_type1, mod_type2, t_half, rad_accum
    (mirrors ForwardMod.__init__ :52-79).  Returns cout (float).
    """
    p = {"tau1": False, "tau2": 0.0, "f1": 1.0, "f2": 0.0, "eta1": False, "eta2": False,
         "D1": False, "D2": False, "J": False, "thalf_cfc": False, "lamsf6": False}
    for i, name in enumerate(par_names):
        p[name] = theta[i]
    if tracer == "He4_ter" and p["J"] == False:  # noqa: E712  (reference quirk :90)
        p["J"] = J_he4_default()
    cv, ci = conv_kwgs["C_values"], conv_kwgs["C_index"]
    t_samp = ci[-1]
    t_half = conv_kwgs.get("t_half", False)
    rad_accum = conv_kwgs.get("rad_accum", False)
    lam = thalf_2_lambda(t_half) if t_half else 0.0

    def one(tau, mod, eta, D):
        lam_ = lam
        if "thalf_cfc" in par_names and tracer == "CFC12":
            lam_ = thalf_2_lambda(p["thalf_cfc"])
        return convolve(cv, ci, t_samp, tau, mod, lamba=lam_, rad_accum=rad_accum,
                        J=10 ** p["J"], eta=eta, D=D)

    cout1 = one(p["tau1"], conv_kwgs["mod_type1"], p["eta1"], p["D1"])
    cout2 = 0.0
    if conv_kwgs.get("mod_type2", False):
        cout2 = one(p["tau2"], conv_kwgs["mod_type2"], p["eta2"], p["D2"])
    cout = p["f1"] * cout1 + p["f2"] * cout2
    if tracer == "SF6" and "lamsf6" in p:
        cout *= (1 + p["lamsf6"])
    return float(cout)


# ---------------------------------------------------------------- frac_inf_diff
def _trapz(y, x):
    """convolution_integral_utils.py:23-26."""
    return 0.5 * ((x[1:] - x[:-1]) * (y[1:] + y[:-1])).sum()


def frac_kappa(Phi_im):
    """convolution_integral_utils.py:245-248."""
    D_o = (2.3e-9) * 60 * 60 * 24 * 365
    R_im = 1
    return Phi_im * np.sqrt((D_o * Phi_im ** 2) * R_im)


def frac_inner(tp, tau, D, bbar, kappa, f_tadv_ext=None):
    """frac_rtd_numba_disp (:36-65) / frac_rtd_numba (:67-97): the inner integral per age."""
    f_t_tran = np.zeros_like(tp)
    with np.errstate(all="ignore"):
        for i in range(len(tp)):
            _tp = tp[i]
            tadv = np.logspace(-6, np.log10(_tp - 1.e-6), 1000)
            if f_tadv_ext is None:
                f_tadv = ((1. / tau) / (np.sqrt(4. * np.pi * D * (tadv / tau)))) * (1. / (tadv / tau)) \
                    * np.exp(-1. * (((1. - (tadv / tau)) ** 2) / (4. * D * (tadv / tau))))
            else:
                f_tadv = np.interp(tadv, tp[:i + 1], f_tadv_ext[:i + 1])
            t_ret = _tp - tadv
            Beta_tadv = tadv / bbar
            f_ret = (kappa * Beta_tadv) / (2 * np.sqrt(np.pi) * t_ret ** (3 / 2)) \
                * np.exp((-1 * kappa ** 2 * Beta_tadv ** 2) / (4 * t_ret))
            f_ret = f_ret / _trapz(f_ret[::-1], t_ret[::-1])
            f_t_tran[i] = _trapz(f_ret * f_tadv, tadv)
    return f_t_tran


def frac_g_tp(n, index_last, t_samp, tau, D, bbar, Phi_im, f_tadv_ext=None):
    """gen_g_tp() for 'frac_inf_diff' (:238-266, :270) -> (g, FM_mu)."""
    tp = age_grid(n, index_last, t_samp)
    f = frac_inner(tp, np.float64(tau), np.float64(D), np.float64(bbar), frac_kappa(np.float64(Phi_im)),
                   None if f_tadv_ext is None else np.asarray(f_tadv_ext, dtype=np.float64))
    with np.errstate(all="ignore"):
        f[0] = 0
        tp_ = tp.copy()
        tp_[0] = 0
        f = f / np.trapezoid(f, tp_)
        g = f
        fm = np.trapezoid(g * tp_, tp_) / np.trapezoid(g, tp_)
        g = g / g.sum()
    return g, fm
