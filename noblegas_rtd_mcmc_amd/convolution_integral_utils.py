"""Drop-in for the reference's ``utils/convolution_integral_utils.py`` on the GPU.

    conv = tracer_conv_integral(C_t, t_samp)
    conv.update_pars(tau=37.3, mod_type='exponential', t_half=12.34)
    conv.convolve()        # -> float, as convolution_integral_utils.py:284-340

``tau`` (and ``eta``/``D``/``t_half``/``J``) may also be numpy arrays: the convolutions of
all parameter sets then run in one launch and ``convolve`` returns an array -- the batched
form of the reference's posterior-predictive and sweep loops (run_age_mcmc.py:251-319,
age_modeling_mcmc.prep.py:739-778).

Supported models: piston, exponential, exp_pist_flow, dispersion (the hot-path models,
SURVEY.md §8a-a19) and the fracture / matrix-diffusion model 'frac_inf_diff' (:238-266,
SURVEY.md §8f rank 3; with the dispersion advective RTD of tau, D or an external one via
f_tadv_ext; 'frac_inf_diff.mint' (:199-236) is the same integral and prints its mean
travel time like the reference), which runs through ``ngrtd_frac_conv``.
"""
import ctypes as C
import hashlib

import numpy as np

from . import _lib
from .spec import ACCUM_IDS, MOD_IDS

_series_cache = {}
_FRAC = ("frac_inf_diff", "frac_inf_diff.mint")


def _series_arrays(C_t, rad_accum):
    """(values, index) of C_t in the reference's DataFrame order (oldest age first).

    The 4He branch reads the 'He4_ter' column when present (:322-327); otherwise the
    frame must hold a single column (convolve ravels it, :336).
    """
    try:
        import pandas as pd
    except ImportError:  # pragma: no cover
        pd = None
    if pd is not None and isinstance(C_t, pd.DataFrame):
        if rad_accum == "4He" and "He4_ter" in C_t.columns:
            s = C_t["He4_ter"]
            return s.to_numpy(dtype=np.float64), np.asarray(s.index)
        if rad_accum == "SF6" and "SF6" in C_t.columns:
            s = C_t["SF6"]
            return s.to_numpy(dtype=np.float64), np.asarray(s.index)
        if C_t.shape[1] != 1:
            raise ValueError("C_t must hold a single tracer column (convolution_integral_utils.py:336)")
        return C_t.to_numpy(dtype=np.float64).ravel(), np.asarray(C_t.index)
    if pd is not None and isinstance(C_t, pd.Series):
        return C_t.to_numpy(dtype=np.float64), np.asarray(C_t.index)
    v = np.asarray(C_t, dtype=np.float64).ravel()
    return v, np.arange(len(v) - 1, -1, -1)


def _series_id(ctx, values, index, t_samp):
    c_by_age = np.ascontiguousarray(np.flip(values))
    idx_by_age = np.ascontiguousarray(np.flip(index.astype(np.float64)))
    dtp = float(np.floor(t_samp - index[-1]))
    h = hashlib.blake2b(c_by_age.tobytes(), digest_size=16)
    h.update(idx_by_age.tobytes())
    key = (ctx.pid, ctx.device, h.hexdigest(), dtp)
    sid = _series_cache.get(key)
    if sid is None:
        sid = ctx.series_create(c_by_age, idx_by_age, dtp)
        _series_cache[key] = sid
    return sid, len(c_by_age)


def _arr(x, n):
    return None if x is None or x is False else np.ascontiguousarray(np.broadcast_to(np.asarray(x, dtype=np.float64), (n,)))


class tracer_conv_integral:
    """convolution_integral_utils.py:105-340 (same constructor, attributes and methods)."""

    _g_tp = None
    _g_lazy = None

    def __init__(self, C_t, t_samp, device=0):
        self.C_t = C_t
        self.t_samp = t_samp
        self._device = device

    @property
    def g_tp(self):
        """The weights convolve() used times its decay factor (3He: 1 - exp(-lamba tp)),
        as the reference leaves ``self.g_tp`` after convolve() (:300-316).  Nothing on the
        log-prob path reads it, so it is materialised on first access: the weights come
        from the device (ngrtd_rtd_weights / ngrtd_frac_conv), the decay factor is the
        reference's own NumPy expression."""
        if self._g_tp is None and self._g_lazy is not None:
            self._g_tp = self._g_lazy()
            self._g_lazy = None
        if self._g_tp is None:
            raise AttributeError("g_tp is set by convolve() (convolution_integral_utils.py:300)")
        return self._g_tp

    @g_tp.setter
    def g_tp(self, value):
        self._g_tp, self._g_lazy = value, None

    def _decayed(self, g, n, index_last, lamba, rad_accum, t_samp):
        """:305-316: g x exp(-lamba tp), or g x (1 - exp(-lamba tp)) for 3He."""
        tp = np.arange(0, n).astype(float)
        tp[0] += 1e-5
        tp += np.floor(t_samp - index_last)
        lam = np.asarray(lamba, dtype=np.float64)
        if lam.ndim:
            lam = lam.reshape(lam.shape + (1,))
        if rad_accum == '3He':
            return g * (1 - np.exp(-lam * tp))
        return g * np.exp(-lam * tp)

    def _defer_g_tp(self, n, index_last, g_tau=None):
        """Record what convolve() used so that g_tp can be built on access."""
        # everything gen_g_tp() and the decay read, as of this convolve() (t_samp / C_t too:
        # the reference applies the decay with convolve()'s t_samp, :307-316)
        snap = dict(tau=self.tau, mod_type=self.mod_type, eta=self.eta, D=self.D, lamba=self.lamba,
                    rad_accum=self.rad_accum, bbar=self.bbar, Phi_im=self.Phi_im, f_tadv_ext=self.f_tadv_ext,
                    t_samp=self.t_samp, C_t=self.C_t, t_half=getattr(self, "_thalf_src", None))

        def build():
            if g_tau is not None:
                g = np.asarray(g_tau, dtype=np.float64)
            else:
                saved = {k: getattr(self, k, None) for k in snap}
                saved_src = getattr(self, "_thalf_src", None)
                try:
                    for k, v in snap.items():
                        if k != "t_half":
                            setattr(self, k, v)
                    shape = np.broadcast_shapes(*[np.shape(snap[k]) for k in ("tau", "eta", "D")
                                                  if snap[k] is not None and snap[k] is not False])
                    if shape == () or self.mod_type in _FRAC:
                        g = self.gen_g_tp()
                    else:
                        taus = np.broadcast_to(np.asarray(snap["tau"], dtype=np.float64), shape)
                        etas = np.broadcast_to(np.asarray(snap["eta"] if snap["eta"] is not None else 0.0,
                                                          dtype=np.float64), shape)
                        Ds = np.broadcast_to(np.asarray(snap["D"] if snap["D"] is not None else 0.0,
                                                        dtype=np.float64), shape)
                        g = np.empty(shape + (n,))
                        for ix in np.ndindex(shape):
                            self.tau, self.eta, self.D = float(taus[ix]), float(etas[ix]), float(Ds[ix])
                            g[ix] = self.gen_g_tp()
                finally:
                    for k, v in saved.items():
                        setattr(self, k, v)
                    self._thalf_src = saved_src
            return self._decayed(g, n, index_last, snap["lamba"], snap["rad_accum"], snap["t_samp"])

        self._g_tp, self._g_lazy = None, build

    def update_pars(self, **kwargs):
        """:111-142 -- missing kwargs reset to None/False exactly like the reference."""
        self.tau = kwargs.get('tau', None)
        self.mod_type = kwargs.get('mod_type', None)
        self.t_half = kwargs.get('t_half', False)
        if np.any(np.asarray(self.t_half, dtype=object) != False):  # noqa: E712
            self.thalf_2_lambda(self.t_half)
        else:
            self.lamba = 0.0
        self.rad_accum = kwargs.get('rad_accum', False)
        self.J = kwargs.get('J', False)
        self.eta = kwargs.get('eta', None)
        self.D = kwargs.get('D', None)
        self.bbar = kwargs.get('bbar', None)
        self.Phi_im = kwargs.get('Phi_im', None)
        self.J_sf6 = kwargs.get('J_sf6', None)
        self.f_tadv_ext = kwargs.get('f_tadv_ext', None)

    def thalf_2_lambda(self, t_half):
        """:146-152."""
        lamba = -1 * np.log(0.5) / np.asarray(t_half, dtype=np.float64)
        self.lamba = float(lamba) if np.ndim(lamba) == 0 else lamba
        self._thalf_src = (t_half, self.lamba)
        return self.lamba

    def _check_model(self):
        if self.mod_type not in MOD_IDS and self.mod_type not in _FRAC:
            raise ValueError("unsupported mod_type %r" % (self.mod_type,))

    def _frac(self, sid, n, accum, Jv, want_conc, want_g):
        """One ngrtd_frac_conv call over the broadcast parameter sets -> (conc, g, FM_mu, shape)."""
        ctx = _lib.Context.get(self._device)
        if self.bbar is None or self.Phi_im is None:
            # the reference computes kappa = Phi_im*... and tadv / bbar with None: TypeError
            raise TypeError("frac_inf_diff needs bbar and Phi_im (convolution_integral_utils.py:246-251)")
        ext = self.f_tadv_ext
        try:
            len(ext)            # :249-253: an external advective RTD when f_tadv_ext has a length
            use_ext = True
        except TypeError:
            use_ext = False
        shapes = [np.shape(self.bbar), np.shape(self.Phi_im), np.shape(self.lamba), np.shape(Jv if Jv is not None else 0)]
        if use_ext:
            ext = np.asarray(ext, dtype=np.float64)
            if ext.shape[-1] != n:
                raise ValueError("External advective function does not match the length of the tracer input "
                                 "function (convolution_integral_utils.py:79-80)")
            shapes.append(ext.shape[:-1])
        else:
            shapes += [np.shape(self.tau), np.shape(self.D)]
        shape = np.broadcast_shapes(*shapes)
        m = int(np.prod(shape)) if shape else 1
        if use_ext:
            if ext.ndim == 1:
                exts, stride = np.ascontiguousarray(ext), 0
            else:
                exts, stride = np.ascontiguousarray(np.broadcast_to(ext, shape + (n,)).reshape(m, n)), n
        else:
            exts, stride = None, 0
        taus = None if use_ext else _arr(self.tau, m)
        Ds = None if use_ext else _arr(self.D, m)
        th = self._t_half_arg()
        per_th = np.ndim(th) > 0
        per_J = np.ndim(Jv) > 0 if Jv is not None else False
        conc = np.empty(m) if want_conc else None
        g = np.empty((m, n)) if want_g else None
        fm = np.empty(m)
        p = lambda a: a.ctypes.data_as(C.c_void_p) if a is not None else None  # noqa: E731
        bbars = np.ascontiguousarray(np.broadcast_to(np.asarray(self.bbar, dtype=np.float64), (m,)))
        phis = np.ascontiguousarray(np.broadcast_to(np.asarray(self.Phi_im, dtype=np.float64), (m,)))
        ctx.check(ctx.lib.ngrtd_frac_conv(ctx.h, sid, accum, p(taus), p(Ds), p(bbars), p(phis), p(exts), stride,
                                          p(_arr(th, m) if per_th else None), 0.0 if per_th else float(th),
                                          p(_arr(Jv, m) if per_J else None),
                                          0.0 if (per_J or Jv is None or Jv is False) else float(Jv),
                                          m, p(conc), p(g), p(fm), _lib.MEM_HOST), "ngrtd_frac_conv")
        self.FM_mu = float(fm[0]) if shape == () else fm.reshape(shape)
        if self.mod_type == "frac_inf_diff.mint":
            for v in np.ravel(self.FM_mu):
                print("mean travel time is " + '%3.2f' % v)
        return conc, g, shape

    def _t_half_arg(self):
        # the device recomputes lamba from the half-life exactly as thalf_2_lambda does; use
        # the half-life that produced self.lamba when it is still current
        src = getattr(self, "_thalf_src", None)
        if src is not None and src[1] is self.lamba:
            return np.asarray(src[0], dtype=np.float64)
        lam = np.asarray(self.lamba, dtype=np.float64)
        with np.errstate(divide="ignore"):
            th = np.where(lam != 0.0, -1 * np.log(0.5) / np.where(lam != 0.0, lam, 1.0), 0.0)
        return th

    def gen_g_tp(self):
        """:155-281 -- normalised weights g(tp) (N,) for scalar parameters."""
        self._check_model()
        ctx = _lib.Context.get(self._device)
        v, i = _series_arrays(self.C_t, self.rad_accum)
        sid, n = _series_id(ctx, v, i, self.t_samp)
        t = np.arange(0, n).astype(float)
        t[0] += 1e-5
        if self.mod_type in _FRAC:
            self.tau_list = t + np.floor(self.t_samp - i[-1])
            _, g, shape = self._frac(sid, n, 0, None, False, True)
            return g[0] if shape == () else g.reshape(shape + (n,))
        g = np.empty(n)
        eta = float(self.eta) if self.eta is not None and self.eta is not False else 0.0
        D = float(self.D) if self.D is not None and self.D is not False else 0.0
        ctx.check(ctx.lib.ngrtd_rtd_weights(ctx.h, sid, MOD_IDS[self.mod_type], float(self.tau), eta, D,
                                            g.ctypes.data_as(C.c_void_p), _lib.MEM_HOST), "ngrtd_rtd_weights")
        t = np.arange(0, n).astype(float)
        t[0] += 1e-5
        self.tau_list = t + np.floor(self.t_samp - i[-1])
        return g

    def convolve(self, **kwargs):
        """:284-340 -- concentration at the sampling time (float, or array for array params)."""
        g_tau = kwargs.get('g_tau', None)
        ctx = _lib.Context.get(self._device)
        v, i = _series_arrays(self.C_t, self.rad_accum)
        sid, n = _series_id(ctx, v, i, self.t_samp)
        accum = ACCUM_IDS.get(self.rad_accum if self.rad_accum in ("3He", "4He", "SF6") else None, 0)
        Jv = self.J_sf6 if self.rad_accum == "SF6" else self.J
        if g_tau is not None:
            g = np.ascontiguousarray(g_tau, dtype=np.float64)
            out = np.empty(1)
            th = float(self._t_half_arg())
            ctx.check(ctx.lib.ngrtd_conv_dot(ctx.h, sid, g.ctypes.data_as(C.c_void_p), th, accum,
                                             float(Jv or 0.0), out.ctypes.data_as(C.c_void_p), _lib.MEM_HOST),
                      "ngrtd_conv_dot")
            self._defer_g_tp(n, i[-1], g_tau=g)
            self.C_i = float(out[0])
            return self.C_i
        self._check_model()
        if self.mod_type in _FRAC:
            conc, _, shape = self._frac(sid, n, accum, Jv, True, False)
            self._defer_g_tp(n, i[-1])
            self.C_i = float(conc[0]) if shape == () else conc.reshape(shape)
            return self.C_i
        tau = np.asarray(self.tau, dtype=np.float64)
        shape = np.broadcast_shapes(tau.shape, np.shape(self.eta if self.eta is not None else 0),
                                    np.shape(self.D if self.D is not None else 0), np.shape(self.lamba),
                                    np.shape(Jv if Jv is not None else 0))
        m = int(np.prod(shape)) if shape else 1
        taus = _arr(tau, m)
        etas = _arr(self.eta, m) if self.mod_type == "exp_pist_flow" else None
        Ds = _arr(self.D, m) if self.mod_type == "dispersion" else None
        th = self._t_half_arg()
        per_th = np.ndim(th) > 0
        ths = _arr(th, m) if per_th else None
        per_J = np.ndim(Jv) > 0 if Jv is not None else False
        Js = _arr(Jv, m) if per_J else None
        out = np.empty(m)
        p = lambda a: a.ctypes.data_as(C.c_void_p) if a is not None else None  # noqa: E731
        ctx.check(ctx.lib.ngrtd_conv(ctx.h, sid, MOD_IDS[self.mod_type], accum, p(taus), p(etas), p(Ds), p(ths),
                                     0.0 if per_th else float(th), p(Js),
                                     0.0 if (per_J or Jv is None or Jv is False) else float(Jv),
                                     m, out.ctypes.data_as(C.c_void_p), _lib.MEM_HOST), "ngrtd_conv")
        self._defer_g_tp(n, i[-1])
        self.C_i = float(out[0]) if shape == () else out.reshape(shape)
        return self.C_i
