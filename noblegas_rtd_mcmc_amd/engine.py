"""Batched log-probability engine: ModelSpec -> ngrtd plan on the GPU.

``LogProb(spec)(theta)`` returns the per-walker log-probability of the reference models
(see spec.py) for a whole ensemble in one device pass -- the emcee ``vectorize=True``
shape.  theta may be

* a numpy float64 array [W][L][P] / [W][L*P] (natural-space parameters per walker), or
  already structure-of-arrays [P][L][W] with ``soa=True`` -- staged through host memory;
* a torch CUDA float64 tensor [P][L][W] -- used in place on the device (no copies), the
  kernels are enqueued on torch's current stream and a device tensor is returned.
"""
import ctypes as C

import numpy as np

from . import _lib
from .spec import ACCUM_IDS, GAS_IDS, MOD_IDS, ModelSpec

ROLE_ORDER = ("Ae_beta", "F_beta", "E_beta", "m", "b_beta", "nu_ce_beta", "tau1", "tau2", "f1", "eta1",
              "eta2", "D1", "D2", "J", "thalf_cfc_beta", "lamsf6", "nu_rtd_beta")


def torch_float64():
    import torch
    return torch.float64


def _is_torch(x):
    return type(x).__module__.startswith("torch")


class LogProb:
    """Compiled log-prob of a ModelSpec on one GPU (one plan, reusable for any W <= max_walkers)."""

    def __init__(self, spec: ModelSpec, max_walkers: int, device: int = 0):
        self.spec = spec
        self.max_walkers = int(max_walkers)
        self.ctx = _lib.Context.get(device)
        self.lib = self.ctx.lib
        self._series = []
        self._keep = []            # host arrays referenced by the descriptor during create
        d = _lib.ModelDesc()
        d.n_wells = spec.n_wells
        d.n_params = spec.n_params
        ri = spec.role_index()
        for i in range(_lib.ROLE_COUNT):
            d.role_index[i] = ri[i]
        d.flags = ((_lib.WANT_LIKE if spec.include_like else 0) | (_lib.WANT_PRIOR if spec.include_prior else 0)
                   | (_lib.WANT_JACOBIAN if spec.jacobian else 0) | (_lib.EXACT_RTD if spec.exact_rtd else 0)
                   | {"auto": 0, "wide": _lib.DISP_WIDE, "lane": _lib.DISP_LANE}[spec.disp_geometry])
        if spec.ce is not None:
            c = spec.ce
            d.ce_enabled = 1
            d.ce_n_gases = len(c.gases)
            for j, g in enumerate(c.gases):
                d.ce_gas_ids[j] = GAS_IDS[g]
            for name in ("obs", "sd", "E_min"):
                arr = np.ascontiguousarray(getattr(c, name), dtype=np.float64)
                self._keep.append(arr)
                setattr(d, {"obs": "ce_obs", "sd": "ce_sd", "E_min": "ce_E_min"}[name], _lib.dptr(arr))
            d.ce_E_max, d.ce_logA_min, d.ce_logA_max = c.E_max, c.logA_min, c.logA_max
            d.ce_logF_min, d.ce_logF_max, d.ce_b_min, d.ce_b_max = c.logF_min, c.logF_max, c.b_min, c.b_max
            d.ce_m_mu, d.ce_m_sd, d.ce_nu_min, d.ce_nu_max = c.m_mu, c.m_sd, c.nu_min, c.nu_max
            for i, ab in enumerate((c.beta_Ae, c.beta_F, c.beta_E, c.beta_b, c.beta_nu)):
                d.ce_beta_a[i], d.ce_beta_b[i] = ab
        if spec.rtd is not None:
            r = spec.rtd
            d.rtd_enabled = 1
            d.n_tracers = len(r.tracers)
            if d.n_tracers > _lib.MAX_TRACERS:
                raise ValueError("at most %d tracers" % _lib.MAX_TRACERS)
            d.mod_type1 = MOD_IDS[r.mod_type1]
            d.mod_type2 = MOD_IDS[r.mod_type2] if r.mod_type2 else _lib.MOD_NONE
            for k, t in enumerate(r.tracers):
                sid = self.ctx.series_create(t.series.c_by_age, t.series.idx_by_age, t.series.dtp)
                self._series.append(sid)
                td = d.tracers[k]
                td.series_id = sid
                td.accum = ACCUM_IDS[t.rad_accum]
                td.t_half = float(t.t_half) if t.t_half else 0.0
                if t.rad_accum == "SF6":
                    td.J = float(t.J_sf6)
                else:
                    # ForwardMod :90-91,101: J = 10**p_dict['J'] (He4_ter default log10 J_flux)
                    from .spec import LOG10_J_HE4_DEFAULT
                    lj = t.log10_J if t.log10_J is not None else (LOG10_J_HE4_DEFAULT if t.name == "He4_ter" else 0.0)
                    td.J = float(10 ** lj)
                td.is_cfc12 = int(t.name == "CFC12")
                td.is_sf6 = int(t.name == "SF6")
            for name, attr in (("obs", "rtd_obs"), ("sd", "rtd_sd")):
                arr = np.ascontiguousarray(getattr(r, name), dtype=np.float64)
                self._keep.append(arr)
                setattr(d, attr, _lib.dptr(arr))
            d.tau1_lo, d.tau1_hi = r.tau1
            d.tau2_lo, d.tau2_hi = r.tau2
            d.f1_lo, d.f1_hi = r.f1
            d.eta1_lo, d.eta1_hi = r.eta1
            d.eta2_lo, d.eta2_hi = r.eta2
            d.D1_lo, d.D1_hi = r.D1
            d.D2_lo, d.D2_hi = r.D2
            d.J_mu, d.J_sd = r.J_mu, r.J_sd
            d.thalf_lo, d.thalf_hi = r.thalf
            d.thalf_a, d.thalf_b = r.beta_thalf
            d.lamsf6_sd = r.lamsf6_sd
            d.rtd_nu_min, d.rtd_nu_max = r.nu_min, r.nu_max
            d.rtd_nu_a, d.rtd_nu_b = r.beta_nu
        self.desc = d
        h = C.c_void_p()
        self.ctx.check(self.lib.ngrtd_plan_create(self.ctx.h, C.byref(d), self.max_walkers, C.byref(h)),
                       "ngrtd_plan_create")
        self.plan = h
        self._keep = []

    # ------------------------------------------------------------------ calls
    def _host_soa(self, theta, soa):
        t = np.asarray(theta, dtype=np.float64)
        if not soa:
            t = self.spec.theta_soa(t)
        t = np.ascontiguousarray(t)
        P, L = self.spec.n_params, self.spec.n_wells
        if t.ndim != 3 or t.shape[0] != P or t.shape[1] != L:
            raise ValueError("theta must be [P=%d][L=%d][W] (got %s)" % (P, L, t.shape))
        if t.shape[2] > self.max_walkers:
            raise ValueError("W=%d exceeds max_walkers=%d" % (t.shape[2], self.max_walkers))
        return t

    def _check_dev(self, theta):
        import torch
        P, L = self.spec.n_params, self.spec.n_wells
        if theta.dtype != torch.float64 or not theta.is_cuda or not theta.is_contiguous():
            raise ValueError("device theta must be a contiguous CUDA float64 tensor")
        if theta.dim() != 3 or theta.shape[0] != P or theta.shape[1] != L or theta.shape[2] > self.max_walkers:
            raise ValueError("device theta must be [P=%d][L=%d][W<=%d]" % (P, L, self.max_walkers))
        self.ctx.set_stream(torch.cuda.current_stream(theta.device).cuda_stream)
        return theta.shape[2]

    def __call__(self, theta, soa=False, out=None):
        """Per-walker log-probability."""
        if _is_torch(theta):
            import torch
            W = self._check_dev(theta)
            if out is None:
                out = torch.empty(W, dtype=torch.float64, device=theta.device)
            self.ctx.check(self.lib.ngrtd_logp(self.plan, C.c_void_p(theta.data_ptr()), W,
                                               C.c_void_p(out.data_ptr()), _lib.MEM_DEVICE), "ngrtd_logp")
            return out
        t = self._host_soa(theta, soa)
        W = t.shape[2]
        res = np.empty(W, dtype=np.float64)
        self.ctx.check(self.lib.ngrtd_logp(self.plan, t.ctypes.data_as(C.c_void_p), W,
                                           res.ctypes.data_as(C.c_void_p), _lib.MEM_HOST), "ngrtd_logp")
        return res

    def units(self, theta, soa=False, out=None):
        """Per-(walker, well) log-probability [L][W] (ngrtd_logp_units): the log-prob of each
        well's own model -- what the per-well sampler's chains target; ``__call__`` is its sum
        over wells."""
        L = self.spec.n_wells
        if _is_torch(theta):
            import torch
            W = self._check_dev(theta)
            if out is None:
                out = torch.empty((L, W), dtype=torch.float64, device=theta.device)
            elif out.dtype != torch.float64 or not out.is_cuda or not out.is_contiguous() or out.numel() != L * W:
                raise ValueError("out must be a contiguous CUDA float64 tensor [L][W]")
            self.ctx.check(self.lib.ngrtd_logp_units(self.plan, C.c_void_p(theta.data_ptr()), W,
                                                     C.c_void_p(out.data_ptr()), _lib.MEM_DEVICE), "ngrtd_logp_units")
            return out
        t = self._host_soa(theta, soa)
        W = t.shape[2]
        res = np.empty((L, W), dtype=np.float64)
        self.ctx.check(self.lib.ngrtd_logp_units(self.plan, t.ctypes.data_as(C.c_void_p), W,
                                                 res.ctypes.data_as(C.c_void_p), _lib.MEM_HOST), "ngrtd_logp_units")
        return res

    def bind(self, theta, out):
        """Fast path for repeated log-probs of the same device buffers: returns a no-argument
        callable that enqueues ngrtd_logp(theta -> out) on torch's current stream of the
        moment of binding (checked once here, not per call)."""
        W = self._check_dev(theta)
        if out.dtype != theta.dtype or not out.is_cuda or not out.is_contiguous() or out.numel() != W:
            raise ValueError("out must be a contiguous CUDA float64 tensor [W]")
        f = self.lib.ngrtd_logp
        args = (self.plan, C.c_void_p(theta.data_ptr()), C.c_int64(W), C.c_void_p(out.data_ptr()),
                C.c_int32(_lib.MEM_DEVICE))
        keep = (theta, out)

        def run():
            st = f(*args)
            if st:
                self.ctx.check(st, "ngrtd_logp")
            return keep[1]
        return run

    def bind_n(self, theta, out):
        """As ``bind``, for k back-to-back log-probs per call: returns ``run(k)`` (one
        ngrtd_logp_n call enqueues k full launches; out holds the last)."""
        W = self._check_dev(theta)
        if out.dtype != theta.dtype or not out.is_cuda or not out.is_contiguous() or out.numel() != W:
            raise ValueError("out must be a contiguous CUDA float64 tensor [W]")
        f = self.lib.ngrtd_logp_n
        base = (self.plan, C.c_void_p(theta.data_ptr()), C.c_int64(W), C.c_void_p(out.data_ptr()))
        keep = (theta, out)

        def run(k):
            st = f(*base, C.c_int64(int(k)))
            if st:
                self.ctx.check(st, "ngrtd_logp_n")
            return keep[1]
        return run

    def region_ms(self):
        """Device time (ms) of the last ``bind_n`` call's launches, back to back: the event
        pair ngrtd_logp_n recorded around them on the plan's stream (waits for the end)."""
        ms = C.c_float()
        self.ctx.check(self.lib.ngrtd_plan_region_ms(self.plan, C.byref(ms)), "ngrtd_plan_region_ms")
        return float(ms.value)

    def forward(self, theta, soa=False):
        """Model outputs: (ce [G][L][W] or None, rtd [K][L][W] or None)."""
        spec = self.spec
        if _is_torch(theta):
            import torch
            W = self._check_dev(theta)
            ce = (torch.empty((len(spec.ce.gases), spec.n_wells, W), dtype=torch.float64, device=theta.device)
                  if spec.ce is not None else None)
            rt = (torch.empty((len(spec.rtd.tracers), spec.n_wells, W), dtype=torch.float64, device=theta.device)
                  if spec.rtd is not None else None)
            self.ctx.check(self.lib.ngrtd_forward(self.plan, C.c_void_p(theta.data_ptr()), W,
                                                  C.c_void_p(ce.data_ptr() if ce is not None else 0),
                                                  C.c_void_p(rt.data_ptr() if rt is not None else 0),
                                                  _lib.MEM_DEVICE), "ngrtd_forward")
            return ce, rt
        t = self._host_soa(theta, soa)
        W = t.shape[2]
        ce = np.empty((len(spec.ce.gases), spec.n_wells, W)) if spec.ce is not None else None
        rt = np.empty((len(spec.rtd.tracers), spec.n_wells, W)) if spec.rtd is not None else None
        self.ctx.check(self.lib.ngrtd_forward(self.plan, t.ctypes.data_as(C.c_void_p), W,
                                              ce.ctypes.data_as(C.c_void_p) if ce is not None else None,
                                              rt.ctypes.data_as(C.c_void_p) if rt is not None else None,
                                              _lib.MEM_HOST), "ngrtd_forward")
        return ce, rt

    def demcz(self, theta, logp, n_steps, state, accepted_log=None, logp_log=None, n_accepted=None,
              accept_log=None):
        """n_steps device-resident DEMetropolisZ steps (ngrtd_demcz_run) of the chains theta
        [P][L][W] (CUDA float64, logp = their log-prob: [W], or [L][W] for per-well chains),
        updated in place on torch's current stream.  state: sampler.ZState (its host counters
        advance).  accepted_log (uint8) / logp_log (float64): optional CUDA [n_steps][chains];
        n_accepted: optional CUDA int64 [1] counter; accept_log (float64, [n_steps][chains]):
        PyMC3's `accept` stat exp(logp(x*) - logp(x)) per step."""
        W = self._check_dev(theta)
        nc = W * (self.spec.n_wells if state.per_well else 1)
        if logp.dtype != torch_float64() or not logp.is_cuda or logp.numel() != nc or not logp.is_contiguous():
            raise ValueError("logp must be a contiguous CUDA float64 tensor of %d chains" % nc)
        R = self.spec.n_params * self.spec.n_wells
        if state.W != W or state.R != R:
            raise ValueError("state was built for R=%d, W=%d" % (state.R, state.W))
        import torch
        for name, t, dt in (("accepted_log", accepted_log, torch.uint8), ("logp_log", logp_log, torch.float64),
                            ("accept_log", accept_log, torch.float64)):
            if t is not None and (not t.is_cuda or t.dtype != dt or t.numel() < n_steps * nc or not t.is_contiguous()):
                raise ValueError("%s must be a contiguous CUDA %s tensor [n_steps][chains]" % (name, dt))
        if n_accepted is not None and (not n_accepted.is_cuda or n_accepted.dtype != torch.int64
                                       or n_accepted.numel() < 1):
            raise ValueError("n_accepted must be a CUDA int64 tensor [1]")
        state.c.accept_log = accept_log.data_ptr() if accept_log is not None else None
        self.ctx.check(self.lib.ngrtd_demcz_run(
            self.plan, C.c_void_p(theta.data_ptr()), C.c_void_p(logp.data_ptr()), W, int(n_steps),
            C.byref(state.c), C.c_void_p(accepted_log.data_ptr() if accepted_log is not None else 0),
            C.c_void_p(logp_log.data_ptr() if logp_log is not None else 0),
            C.c_void_p(n_accepted.data_ptr() if n_accepted is not None else 0)), "ngrtd_demcz_run")

    def kernel_stats(self, reset=False):
        ms = (C.c_double * 4)()
        n = (C.c_int64 * 4)()
        self.ctx.check(self.lib.ngrtd_plan_kernel_stats(self.plan, ms, n, 4, int(reset)), "kernel_stats")
        return {"rtd": (ms[0], n[0]), "unit": (ms[1], n[1]), "reduce": (ms[2], n[2]), "fused": (ms[3], n[3])}

    def info(self, W):
        v = (C.c_int64 * 16)()
        self.ctx.check(self.lib.ngrtd_plan_info(self.plan, int(W), v, 16), "plan_info")
        keys = ("R", "NW", "blocks", "slice_ages", "channels", "N", "lds_bytes", "units", "mfma_rows", "S_seg",
                "nsteps", "surrogate", "surrogate_err_e18", "c0_pieces", "disp_wide_g")
        d = dict(zip(keys, list(v)))
        d["surrogate_max_rel_err"] = d.pop("surrogate_err_e18") * 1e-18 if v[12] >= 0 else None
        return d

    def close(self):
        if getattr(self, "plan", None):
            self.lib.ngrtd_plan_destroy(self.plan)
            self.plan = None
            for sid in self._series:
                self.lib.ngrtd_series_destroy(self.ctx.h, sid)
            self._series = []

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
