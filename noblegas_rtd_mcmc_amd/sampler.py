"""DEMetropolisZ over the batched log-prob: the reference's sampler, one chain per walker.

The reference samples with PyMC3 3.11.2 ``DEMetropolisZ`` (run_age_mcmc_utils.py:412-417:
tune=10000, draws=10000, chains=3, tune_interval=1000; ng_interp/noble_gas_mcmc.py:410-415:
tune=10000, draws=50000, chains=4, tune_interval=5000), one log-prob per proposal per
chain, chains in separate processes.  Here W chains run at once and every step evaluates
ONE batched log-prob.  Each chain is exactly a PyMC3 DEMetropolisZ chain
(pymc3/step_methods/metropolis.py ``DEMetropolisZ.astep``/``stop_tuning``):

* proposal  x* = x + lamb_w (z1 - z2) + eps,  eps ~ U(-1, 1) * S * scaling_w per parameter
  (S: PyMC3's proposal scale vector, default ones), with
  z1 != z2 drawn uniformly from the chain's OWN history of past states (noise only while
  the history holds fewer than 2 entries).  Chains never read each other's states, so they
  stay independent (no population move, nothing to shard but the log-prob);
* accept iff mr = logp(x*) - logp(x) is finite and log(u) < mr (``metrop_select``);
* tuning (tune='lambda' by default, or 'scaling', or None): every ``tune_interval`` steps
  of the tuning phase the chain's lamb (or scaling) is multiplied by ``pymc3_tune`` of its
  acceptance rate over the interval;
* ``stop_tuning`` before the first draw drops the oldest ``tune_drop_fraction`` of the
  history, so draws are not proposed from unconverged tuning states.

The chains sample the PyMC3 models' free variables in their natural (untransformed)
space; PyMC3 proposes in its transformed space (logodds / interval / log).  Both target
the same posterior; the proposal geometry differs (parity of the chains themselves is
unpinned -- PyMC3 is not installed anywhere here; tests check the stationary
distribution: analytic prior moments, and the reference's posterior summaries).

Random numbers are counter-based (splitmix64 of (seed, step, chain[, element])), the same
stream in ``DEMetropolisZ`` (torch ops, any device, any batched log_prob) and
``DeviceDEMetropolisZ`` (libngrtd ``ngrtd_demcz_run``: joint plans run up to 256 whole
steps per launch, each block stepping its own chains; other plans a proposal + history
append kernel and a log-prob + decision + tuning kernel per step; no host round trip),
so on the same log-prob the two produce bitwise the same chains.
"""
import math

import torch

from . import _lib

_M64 = (1 << 64) - 1


def _s64(v):
    """Python uint64 -> the int64 with the same bits."""
    v &= _M64
    return v - (1 << 64) if v >> 63 else v


def _lsr(z, k):
    """Logical right shift of int64 tensors (torch's >> is arithmetic)."""
    return (z >> k) & ((1 << (64 - k)) - 1)


_C1, _C2, _C3 = _s64(0x9E3779B97F4A7C15), _s64(0xBF58476D1CE4E5B9), _s64(0x94D049BB133111EB)


def mix_t(z):
    """splitmix64 finaliser on int64 tensors (wrapping arithmetic), = ngrtd_kernels.hpp rng_mix."""
    z = z + _C1
    z = (z ^ _lsr(z, 30)) * _C2
    z = (z ^ _lsr(z, 27)) * _C3
    return z ^ _lsr(z, 31)


def mix_int(z):
    z = (z + 0x9E3779B97F4A7C15) & _M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _M64
    return z ^ (z >> 31)


def step_key(seed, step):
    """demc_key: the random key of step `step` of a run seeded `seed`."""
    return mix_int((mix_int(seed & _M64) + step) & _M64)


def unit_t(h):
    """(0, 1) uniform of a hash (rng_unit): ((h >> 11) + 0.5) 2^-53."""
    return (_lsr(h, 11).to(torch.float64) + 0.5) * (1.0 / 9007199254740992.0)


def _dev_ctx(t):
    """The libngrtd context of a CUDA tensor's device, enqueueing on torch's current stream;
    None for a CPU tensor (CPU runs of this restatement use torch's own exp / log)."""
    if not t.is_cuda:
        return None
    ctx = _lib.Context.get(t.device.index or 0)
    ctx.set_stream(torch.cuda.current_stream(t.device).cuda_stream)
    return ctx


def fm_log(x):
    """log(x) as the device DEMetropolisZ kernels take it for the accept draw (the table-driven
    flog, <= 1 ulp: ngrtd_fm_log) on CUDA tensors, so that both samplers make the same
    decisions bit for bit; torch.log on the CPU."""
    ctx = _dev_ctx(x)
    if ctx is None:
        return torch.log(x)
    if x.dtype != torch.float64:
        raise TypeError("fm_log: the device log takes float64 tensors, got %s" % (x.dtype,))
    x = x.contiguous()
    out = torch.empty_like(x)
    ctx.check(ctx.lib.ngrtd_fm_log(ctx.h, x.data_ptr(), out.data_ptr(), x.numel()), "ngrtd_fm_log")
    return out


def pymc3_tune(scale, acc_rate):
    """pymc3.step_methods.metropolis.tune (3.11): multiplicative update from the
    acceptance rate of the last tune interval (elementwise on tensors)."""
    c = lambda v: torch.full_like(scale, v)   # noqa: E731  (float64 factors, as numpy's)
    f = torch.where(acc_rate < 0.001, c(0.1), torch.where(acc_rate < 0.05, c(0.5), torch.where(
        acc_rate < 0.2, c(0.9), torch.where(acc_rate > 0.95, c(10.0), torch.where(
            acc_rate > 0.75, c(2.0), torch.where(acc_rate > 0.5, c(1.1), c(1.0)))))))
    return scale * f


def default_lamb(ndim):
    """PyMC3: 2.38 / sqrt(2 ndim), optimal for normal targets."""
    return 2.38 / math.sqrt(2 * ndim)


class Transform:
    """PyMC3 3.11 default transforms of the free variables, per theta row
    (pymc3/distributions/transforms.py): Beta -> LogOdds, Uniform -> Interval(a, b),
    HalfNormal -> Log, Normal -> none.  ``backward`` is the same arithmetic as the
    device's pymc3_backward (ngrtd_kernels.hpp), so both give the same bits."""

    NONE, LOGODDS, INTERVAL, LOG = 0, 1, 2, 3

    def __init__(self, kind, a, b, L=1):
        self.kind = [int(k) for k in kind]        # per parameter p
        self.a = [float(v) for v in a]
        self.b = [float(v) for v in b]
        self.L = int(L)

    @classmethod
    def from_spec(cls, spec):
        kind, a, b = [], [], []
        for role in spec.roles:
            lo = hi = 0.0
            if role.endswith("_beta"):
                k = cls.LOGODDS
            elif role in ("tau1", "tau2", "f1", "eta1", "eta2", "D1", "D2"):
                k = cls.INTERVAL
                lo, hi = getattr(spec.rtd, role)
            elif role == "lamsf6":
                k = cls.LOG
            else:                                   # m, J: Normal priors, untransformed
                k = cls.NONE
            kind.append(k)
            a.append(lo)
            b.append(hi)
        return cls(kind, a, b, spec.n_wells)

    def _rows(self, t):
        return t.reshape(-1, len(self.kind), self.L, t.shape[-1])

    def backward(self, u):
        """u [..., P, L, W] (any leading dims) -> natural x.  On CUDA tensors through
        ngrtd_pymc3_backward -- the device DEMetropolisZ kernels' own function (its exp is the
        table-driven fexp, <= 1 ulp), so that the two samplers' chains agree bit for bit;
        torch's exp on the CPU."""
        ctx = _dev_ctx(u)
        if ctx is not None:
            import ctypes as C
            if u.dtype != torch.float64:
                raise TypeError("Transform.backward: the device transform takes float64 tensors, got %s" % (u.dtype,))
            uc = u.contiguous()
            out = torch.empty_like(uc)
            P = len(self.kind)
            inner = self.L * int(uc.shape[-1])
            lead = uc.numel() // (P * inner) if inner else 0
            kind = (C.c_int32 * P)(*self.kind)
            a = (C.c_double * P)(*self.a)
            b = (C.c_double * P)(*self.b)
            ctx.check(ctx.lib.ngrtd_pymc3_backward(ctx.h, uc.data_ptr(), out.data_ptr(), lead, P, inner, kind, a, b),
                      "ngrtd_pymc3_backward")
            return out.reshape(u.shape)
        ur = self._rows(u)
        out = torch.empty_like(ur)
        for p, k in enumerate(self.kind):
            v = ur[:, p]
            if k == self.LOGODDS:
                out[:, p] = 1.0 / (1.0 + torch.exp(-v))
            elif k == self.INTERVAL:
                sg = 1.0 / (1.0 + torch.exp(-v))
                out[:, p] = sg * self.b[p] + (1.0 - sg) * self.a[p]
            elif k == self.LOG:
                out[:, p] = torch.exp(v)
            else:
                out[:, p] = v
        return out.reshape(u.shape)

    def forward(self, x):
        """natural x -> u (logit, log((x - a) / (b - x)), log)."""
        xr = self._rows(x)
        out = torch.empty_like(xr)
        for p, k in enumerate(self.kind):
            v = xr[:, p]
            if k == self.LOGODDS:
                out[:, p] = torch.log(v) - torch.log1p(-v)
            elif k == self.INTERVAL:
                out[:, p] = torch.log(v - self.a[p]) - torch.log(self.b[p] - v)
            elif k == self.LOG:
                out[:, p] = torch.log(v)
            else:
                out[:, p] = v
        return out.reshape(x.shape)

    def fill(self, c):
        """Copy into an ngrtd_demcz_state (tr_kind / tr_a / tr_b per parameter row)."""
        for p, k in enumerate(self.kind):
            c.tr_kind[p], c.tr_a[p], c.tr_b[p] = k, self.a[p], self.b[p]


def _result(hist, lp_log, acc_log, tune, draws, lamb, scaling, x, lp, ar_log=None):
    acc = acc_log[tune:].to(torch.float64)
    return {"samples": hist[tune:tune + draws], "logp": lp_log[tune:tune + draws],
            "accepted": acc_log[tune:tune + draws], "accept_rate": float(acc.mean()) if draws else 0.0,
            "accept": ar_log[tune:tune + draws] if ar_log is not None else None,   # PyMC3's exp(mr) stat
            "tune_accept_rate": float(acc_log[:tune].to(torch.float64).mean()) if tune else 0.0,
            "lamb": lamb, "scaling": scaling, "x": x, "lp": lp, "tuning_steps": tune}


def pw_cid(well0, L, Wg, chain0, W, device):
    """Per-well chains: the random-stream id of every unit [L][W] (= ngrtd_kernels.hpp dz_cid),
    (well0 + l) Wg + chain0 + w -- the same in a run of all L wells and in a run of well l
    alone (well0 = l), and in every walker-block shard (chain0)."""
    l = torch.arange(L, device=device, dtype=torch.int64)[:, None] + int(well0)
    w = torch.arange(W, device=device, dtype=torch.int64)[None, :] + int(chain0)
    return l * int(Wg) + w


PW_ROW_STRIDE = 32      # = ngrtd_kernels.hpp kPwRowStride: noise element cid * 32 + p



class DEMetropolisZ:
    """PyMC3 DEMetropolisZ for the W chains of x0 [..., W] on torch ops (any device).

    log_prob: callable theta [..., W] -> logp [W] (e.g. engine.LogProb, or a CPU oracle).

    per_well=True: x0 is [P][L][W] and every (walker w, well l) is its own P-dimensional
    chain -- the reference's structure, one PyMC3 model per well (run_age_mcmc.py:122-231,
    noble_gas_mcmc.py:95-104).  log_prob must then return the per-unit log-prob [L][W]
    (engine.LogProb.units); lamb (default 2.38 / sqrt(2 P)), scaling, the tuning counters,
    the decisions and the logs are per unit ([L][W]); the proposal noise and the accept
    draws are keyed by the unit's pw_cid (well0: global index of well 0), the history
    partner indices by the walker (each well reading its own history), the device sampler's
    streams bit for bit."""

    def __init__(self, log_prob, lamb=None, scaling=0.001, tune="lambda", tune_interval=100,
                 tune_drop_fraction=0.9, seed=123423, chain0=0, n_chains_total=None, S=None, transform=None,
                 per_well=False, well0=0):
        if tune not in (None, "none", "scaling", "lambda"):
            raise ValueError('tune must be None, "scaling" or "lambda" (pymc3 DEMetropolisZ)')
        self.per_well = bool(per_well)
        self.well0 = int(well0)
        self.transform = transform               # Transform: chains in PyMC3's transformed space
        self.S = S                               # proposal scale per parameter (x[..., 0] shape), None = ones
        self.chain0 = int(chain0)                # global index of chain 0 (walker-block shards)
        self.n_chains_total = n_chains_total
        self.log_prob = log_prob
        self.lamb = lamb
        self.scaling = scaling
        self.tune = tune
        self.tune_interval = int(tune_interval)
        self.tune_drop_fraction = float(tune_drop_fraction)
        self.seed = int(seed)

    def run(self, x0, tune, draws):
        """Returns dict(samples [draws, ..., W] (natural space), logp [draws, W], accepted
        [draws, W] (uint8), accept_rate, lamb [W], scaling [W], x, lp).  With a transform the
        chains move in u = transform.forward(x0), log_prob must return the log-density of u
        (natural log-prob + log|Jacobian|, e.g. a LogProb of a spec with jacobian=True), and
        it is called on the natural values backward(u)."""
        if self.per_well:
            return self._run_per_well(x0, tune, draws)
        tf = self.transform
        u = tf.forward(x0) if tf is not None else x0.clone()
        x = u
        lead, W = x.shape[:-1], x.shape[-1]
        R = int(x[..., 0].numel())
        dev = x.device
        lamb = torch.full((W,), self.lamb if self.lamb is not None else default_lamb(R), dtype=torch.float64,
                          device=dev)
        scaling = torch.full((W,), float(self.scaling), dtype=torch.float64, device=dev)
        lp = self.log_prob(tf.backward(x) if tf is not None else x).clone()
        if not bool(torch.isfinite(lp).all()):
            raise ValueError("initial log-prob is not finite for every chain (pymc3: 'Initial evaluation of model "
                             "at starting point failed')")
        n = tune + draws
        hist = torch.empty((n,) + tuple(x.shape), dtype=x.dtype, device=dev)
        lp_log = torch.empty((n, W), dtype=torch.float64, device=dev)
        acc_log = torch.empty((n, W), dtype=torch.uint8, device=dev)
        ar_log = torch.empty((n, W), dtype=torch.float64, device=dev)
        n_acc_tune = torch.zeros(W, dtype=torch.int32, device=dev)
        hist_lo = 0
        w_loc = torch.arange(W, device=dev, dtype=torch.int64)
        w_idx = w_loc + self.chain0                                      # global chain index
        Wg = int(self.n_chains_total or W)
        e_idx = (torch.arange(R, device=dev, dtype=torch.int64)[:, None] * Wg + w_idx[None, :])  # r Wg + chain
        target = {"scaling": 1, "lambda": 2}.get(self.tune, 0)
        S = None if self.S is None else torch.as_tensor(self.S, dtype=torch.float64, device=dev).reshape(R, 1)
        for s in range(n):
            if s == tune and tune > 0:                       # stop_tuning: drop the oldest entries
                hist_lo += int(self.tune_drop_fraction * (s - hist_lo))
            key = step_key(self.seed, s)
            it = s - hist_lo
            xr = x.reshape(R, W)
            if it > 1:
                hp = mix_t(w_idx + _s64(mix_int((key + 1) & _M64)))
                iz1 = (_lsr(hp, 32) * it) >> 32
                iz2 = ((hp & 0xFFFFFFFF) * (it - 1)) >> 32
                iz2 = iz2 + (iz2 >= iz1).to(torch.int64)
                hr = hist.reshape(n, R, W)
                z1 = hr[hist_lo + iz1, :, w_loc].T            # [R][W]
                z2 = hr[hist_lo + iz2, :, w_loc].T
                y = xr + lamb * (z1 - z2)
            else:
                y = xr
            ke = _s64(mix_int((key + 2) & _M64))
            u2 = 2.0 * unit_t(mix_t(e_idx + ke)) - 1.0
            eps = (u2 if S is None else u2 * S) * scaling
            prop = (y + eps).reshape(x.shape)
            lp_prop = self.log_prob(tf.backward(prop) if tf is not None else prop)
            logu = fm_log(unit_t(mix_t(w_idx + _s64(mix_int((key + 3) & _M64)))))
            mr = lp_prop - lp
            acc = torch.isfinite(mr) & (logu < mr)
            x = torch.where(acc, prop, x)
            lp = torch.where(acc, lp_prop, lp)
            n_acc_tune += acc.to(torch.int32)
            if target and s + 1 < tune and (s + 1) % self.tune_interval == 0:
                rate = n_acc_tune.to(torch.float64) / self.tune_interval
                if target == 2:
                    lamb = pymc3_tune(lamb, rate)
                else:
                    scaling = pymc3_tune(scaling, rate)
                n_acc_tune.zero_()
            hist[s] = x
            lp_log[s] = lp
            acc_log[s] = acc.to(torch.uint8)
            ar_log[s] = torch.exp(mr)
        if tf is not None:
            hist = tf.backward(hist)
            x = tf.backward(x)
        return _result(hist, lp_log, acc_log, tune, draws, lamb, scaling, x, lp, ar_log)


    def _run_per_well(self, x0, tune, draws):
        """per_well=True: the chains are the units of x0 [P][L][W] (see the class doc)."""
        tf = self.transform
        x = tf.forward(x0) if tf is not None else x0.clone()
        if x.dim() != 3:
            raise ValueError("per-well chains need theta [P][L][W]")
        P, L, W = x.shape
        dev = x.device
        lamb = torch.full((L, W), self.lamb if self.lamb is not None else default_lamb(P), dtype=torch.float64,
                          device=dev)
        scaling = torch.full((L, W), float(self.scaling), dtype=torch.float64, device=dev)
        lp = self.log_prob(tf.backward(x) if tf is not None else x).clone()
        if tuple(lp.shape) != (L, W):
            raise ValueError("per-well chains need a per-unit log_prob [L][W] (engine.LogProb.units)")
        if not bool(torch.isfinite(lp).all()):
            raise ValueError("initial log-prob is not finite for every chain (pymc3: 'Initial evaluation of model "
                             "at starting point failed')")
        n = tune + draws
        hist = torch.empty((n, P, L, W), dtype=x.dtype, device=dev)
        lp_log = torch.empty((n, L, W), dtype=torch.float64, device=dev)
        acc_log = torch.empty((n, L, W), dtype=torch.uint8, device=dev)
        ar_log = torch.empty((n, L, W), dtype=torch.float64, device=dev)
        n_acc_tune = torch.zeros((L, W), dtype=torch.int32, device=dev)
        hist_lo = 0
        Wg = int(self.n_chains_total or W)
        cid = pw_cid(self.well0, L, Wg, self.chain0, W, dev)                     # [L][W]
        wkey = (torch.arange(W, device=dev, dtype=torch.int64) + self.chain0)[None, :].expand(L, W)
        e_idx = cid[None] * PW_ROW_STRIDE + torch.arange(P, device=dev, dtype=torch.int64)[:, None, None]
        li = torch.arange(L, device=dev)[:, None].expand(L, W)
        wi = torch.arange(W, device=dev)[None, :].expand(L, W)
        target = {"scaling": 1, "lambda": 2}.get(self.tune, 0)
        S = None if self.S is None else torch.as_tensor(self.S, dtype=torch.float64, device=dev).reshape(P, L, 1)
        for s in range(n):
            if s == tune and tune > 0:                       # stop_tuning: drop the oldest entries
                hist_lo += int(self.tune_drop_fraction * (s - hist_lo))
            key = step_key(self.seed, s)
            it = s - hist_lo
            if it > 1:              # partner indices keyed by the walker (every well alike)
                hp = mix_t(wkey + _s64(mix_int((key + 1) & _M64)))
                iz1 = (_lsr(hp, 32) * it) >> 32
                iz2 = ((hp & 0xFFFFFFFF) * (it - 1)) >> 32
                iz2 = iz2 + (iz2 >= iz1).to(torch.int64)
                z1 = hist[hist_lo + iz1, :, li, wi].permute(2, 0, 1)      # [P][L][W]
                z2 = hist[hist_lo + iz2, :, li, wi].permute(2, 0, 1)
                y = x + lamb * (z1 - z2)
            else:
                y = x
            ke = _s64(mix_int((key + 2) & _M64))
            u2 = 2.0 * unit_t(mix_t(e_idx + ke)) - 1.0
            eps = (u2 if S is None else u2 * S) * scaling
            prop = y + eps
            lp_prop = self.log_prob(tf.backward(prop) if tf is not None else prop)
            logu = fm_log(unit_t(mix_t(cid + _s64(mix_int((key + 3) & _M64)))))
            mr = lp_prop - lp
            acc = torch.isfinite(mr) & (logu < mr)
            x = torch.where(acc, prop, x)
            lp = torch.where(acc, lp_prop, lp)
            n_acc_tune += acc.to(torch.int32)
            if target and s + 1 < tune and (s + 1) % self.tune_interval == 0:
                rate = n_acc_tune.to(torch.float64) / self.tune_interval
                if target == 2:
                    lamb = pymc3_tune(lamb, rate)
                else:
                    scaling = pymc3_tune(scaling, rate)
                n_acc_tune.zero_()
            hist[s] = x
            lp_log[s] = lp
            acc_log[s] = acc.to(torch.uint8)
            ar_log[s] = torch.exp(mr)
        if tf is not None:
            hist = tf.backward(hist)
            x = tf.backward(x)
        return _result(hist, lp_log, acc_log, tune, draws, lamb, scaling, x, lp, ar_log)


class ZState:
    """Device state of a DEMetropolisZ run (ngrtd_demcz_state): per-chain lamb / scaling /
    tuning counters and the chain histories [cap][W][R] (chain-major: a chain's state is one
    contiguous run), which also hold the draws."""

    def __init__(self, R, W, hist_cap, device, lamb, scaling, n_tune, tune_interval, tune_target,
                 drop_fraction, seed, chain0=0, n_chains_total=0, S=None, per_well=False, L=1, well0=0,
                 n_wells_total=0):
        self.R, self.W = int(R), int(W)
        self.per_well, self.L = bool(per_well), int(L)
        shp = (self.L, W) if self.per_well else (W,)      # per-well chains: [L][W]
        self.lamb = torch.full(shp, float(lamb), dtype=torch.float64, device=device)
        self.scaling = torch.full(shp, float(scaling), dtype=torch.float64, device=device)
        self.n_acc_tune = torch.zeros(shp, dtype=torch.int32, device=device)
        self.P = self.R // self.L
        self.hist = torch.empty((int(hist_cap), W, self.R), dtype=torch.float64, device=device)
        self.u = None                     # transformed-space chains (set by DeviceDEMetropolisZ.start)
        self.S = (None if S is None else
                  torch.as_tensor(S, dtype=torch.float64).reshape(self.R).contiguous().to(device))
        self.c = _lib.DemczState(lamb=self.lamb.data_ptr(), scaling=self.scaling.data_ptr(),
                                 n_acc_tune=self.n_acc_tune.data_ptr(), hist=self.hist.data_ptr(),
                                 hist_cap=int(hist_cap), hist_len=0, hist_lo=0, steps_done=0, n_tune=int(n_tune),
                                 tune_interval=int(tune_interval), tune_target=int(tune_target),
                                 drop_fraction=float(drop_fraction), seed=int(seed) & _M64,
                                 chain0=int(chain0), n_chains_total=int(n_chains_total or 0),
                                 S=self.S.data_ptr() if self.S is not None else None,
                                 per_well=int(self.per_well), well0=int(well0),
                                 n_wells_total=int(n_wells_total or 0))

    def entries(self, lo, hi):
        """History entries [lo, hi) as [hi - lo][R][W] (per-well chains: [hi - lo][P][L][W])."""
        if self.per_well:
            return self.hist[lo:hi].reshape(hi - lo, self.W, self.P, self.L).permute(0, 2, 3, 1)
        return self.hist[lo:hi].permute(0, 2, 1)


class DeviceDEMetropolisZ:
    """The same DEMetropolisZ run device-resident by libngrtd (ngrtd_demcz_run): one C call
    for the whole run (up to 256 steps per launch for the joint plans, else two launches per
    step), no host synchronisation until the end.
    Same random stream as DEMetropolisZ, so on the same log-prob the chains agree bitwise.

    transformed: chains in PyMC3's transformed space (Transform.from_spec) -- the default
    when the plan's spec has jacobian=True (the log-prob is then the density of u); else
    the natural space.

    per_well (default True): every (walker, well) unit is its own chain, as the reference
    runs one PyMC3 model per well (the wells of every reference model share no parameter);
    logp / lamb / scaling / the logs are then [L][W].  False: one chain per walker over all
    its wells (one decision on the sum of the wells' log-probs)."""

    def __init__(self, logprob, lamb=None, scaling=0.001, tune="lambda", tune_interval=100,
                 tune_drop_fraction=0.9, seed=123423, chain0=0, n_chains_total=None, S=None, transformed=None,
                 per_well=True, well0=0, n_wells_total=None):
        if tune not in (None, "none", "scaling", "lambda"):
            raise ValueError('tune must be None, "scaling" or "lambda" (pymc3 DEMetropolisZ)')
        self.per_well = bool(per_well)
        self.well0 = int(well0)
        # the run's total wells: the device rejects a well range [well0, well0 + L) beyond it
        # (streams keyed by the global well index must not collide between calls); None = unchecked
        self.n_wells_total = n_wells_total
        if transformed is None:
            transformed = bool(logprob.spec.jacobian)
        if transformed and not logprob.spec.jacobian:
            raise ValueError("transformed-space chains need a LogProb of a spec with jacobian=True")
        self.transform = Transform.from_spec(logprob.spec) if transformed else None
        self.S = S
        self.chain0 = int(chain0)
        self.n_chains_total = n_chains_total
        self.lp = logprob               # engine.LogProb
        self.lamb = lamb
        self.scaling = scaling
        self.tune = tune
        self.tune_interval = int(tune_interval)
        self.tune_drop_fraction = float(tune_drop_fraction)
        self.seed = int(seed)

    def start(self, x0, n_tune, hist_cap):
        """Device state for chains x0 [P][L][W] (natural space, CUDA float64): (x, lp, ZState);
        x = backward(forward(x0)) for transformed chains (ZState.u holds the chains)."""
        tf = self.transform
        u = tf.forward(x0).contiguous() if tf is not None else None
        x = tf.backward(u).contiguous() if tf is not None else x0.clone().contiguous()
        W = x.shape[-1]
        R = int(x[..., 0].numel())
        P, L = self.lp.spec.n_params, self.lp.spec.n_wells
        lp = (self.lp.units(x) if self.per_well else self.lp(x)).clone()
        if not bool(torch.isfinite(lp).all()):
            raise ValueError("initial log-prob is not finite for every chain (pymc3: 'Initial evaluation of model "
                             "at starting point failed')")
        lamb = self.lamb if self.lamb is not None else default_lamb(P if self.per_well else R)
        z = ZState(R, W, hist_cap, x.device, lamb, self.scaling,
                   n_tune, self.tune_interval, _lib.TUNE_TARGET[self.tune], self.tune_drop_fraction, self.seed,
                   self.chain0, self.n_chains_total, self.S, per_well=self.per_well, L=L, well0=self.well0,
                   n_wells_total=self.n_wells_total)
        if tf is not None:
            z.u = u
            z.c.theta_u = u.data_ptr()
            tf.fill(z.c)
        return x, lp, z

    def run(self, x0, tune, draws):
        n = tune + draws
        x, lp, z = self.start(x0, tune, n)
        shp = tuple(lp.shape)                   # [W], or [L][W] for per-well chains
        acc_log = torch.empty((n,) + shp, dtype=torch.uint8, device=x.device)
        lp_log = torch.empty((n,) + shp, dtype=torch.float64, device=x.device)
        ar_log = torch.empty((n,) + shp, dtype=torch.float64, device=x.device)
        self.lp.demcz(x, lp, n, z, accepted_log=acc_log, logp_log=lp_log, accept_log=ar_log)
        hist = z.entries(0, n).reshape((n,) + tuple(x.shape))
        if self.transform is not None:              # the histories hold u: report natural draws
            hist = self.transform.backward(hist)
        return _result(hist, lp_log, acc_log, tune, draws, z.lamb, z.scaling, x, lp, ar_log)


def sample_model(spec, max_walkers, device, x0, tune, draws, seed, tune_interval, sampler="device",
                 space="transformed", cache=None, per_well=True):
    """DEMetropolisZ on the log-prob of ``spec`` (the drivers' mc.sample replacement):
    space "transformed" samples PyMC3's free variables (a plan with the Jacobian),
    "natural" theta itself.  per_well: one chain per (walker, well), as the reference's one
    model per well (logp / accepted [draws][L][W]); False: one chain per walker.
    ``cache``: a dict that keeps the sampling plan between calls."""
    import dataclasses
    from .engine import LogProb
    if space not in ("transformed", "natural"):
        raise ValueError('space must be "transformed" or "natural"')
    jac = space == "transformed"
    cache = {} if cache is None else cache
    key = "_sampling_lp_%s" % space
    lp = cache.get(key)
    if lp is None:
        lp = LogProb(dataclasses.replace(spec, jacobian=jac), max_walkers, device)
        cache[key] = lp
    import time
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if sampler == "device":
        res = DeviceDEMetropolisZ(lp, tune_interval=tune_interval, seed=seed, transformed=jac,
                                  per_well=per_well).run(x0, tune, draws)
    else:
        tf = Transform.from_spec(spec) if jac else None
        f = (lambda th: lp.units(th)) if per_well else (lambda th: lp(th))
        res = DEMetropolisZ(f, tune_interval=tune_interval, seed=seed, transform=tf,
                            per_well=per_well).run(x0, tune, draws)
    torch.cuda.synchronize()
    res["sampling_time"] = time.perf_counter() - t0          # PyMC3's trace attribute, seconds
    return res
