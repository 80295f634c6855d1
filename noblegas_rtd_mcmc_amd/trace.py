"""Posterior traces in ArviZ's InferenceData layout, in the reference's container.

The reference saves every run with ``az.to_netcdf(az.from_pymc3(trace), trace_name)``
(age_ens_runs_mcmc/run_age_mcmc_utils.py:420-425, ng_interp/noble_gas_mcmc.py:422-447;
ArviZ 0.11.4, PyMC3 3.11.2, netCDF 4.8.1): ONE netCDF-4 (HDF5) file with the groups

* ``posterior``: one variable per PyMC3 random variable and deterministic, dims (chain, draw);
* ``sample_stats``: DEMetropolisZ's stats accept (exp(logp(x*) - logp(x))), accepted
  (int8, ``dtype = "bool"``), lambda, scaling;
* ``observed_data``: the likelihood's observations ``like`` (dim like_dim_0);

each with the attributes created_at, arviz_version, inference_library,
inference_library_version (+ sampling_time [s], tuning_steps on posterior / sample_stats).
The reference reads it back with ``az.from_netcdf`` (run_age_mcmc_utils.py:434,
run_age_mcmc.post_plots.comp.py:171, age_modeling_mcmc.post_plots.py:128).  ``to_netcdf``
writes that file with h5lite (HDF5 written from the format specification; h5py / netCDF4 are
not in this image): same groups, variable names, dims, dtypes, attributes, dimension scales
and storage (one shuffle + deflate chunk per variable) as the shipped
``conv_traces/*.netcdf``, which ``tests/test_trace_cpu.py`` reads and diffs against.

Variable names follow the reference models: CE (noble_gas_mcmc.py:216-267) Ae_beta, F_beta,
E_beta, m, b_beta, nu_ and the deterministics Ae, F (log10 values, as the model defines them:
:229-230), E, b, T, nu; RTD (run_age_mcmc_utils.py:286-344) tau1, nu_, nu, J, tau2, f1, f2,
tau, eta1, eta2, D1, D2, thalf_cfc_, thalf_cfc, lamsf6.  A model with both blocks prefixes the
CE nu variables with ``ce_``.  Walkers are chains; a model of several wells (the reference
writes one file per well) gets a trailing ``well`` dim.
"""
import datetime
import os

import numpy as np

CE_NAMES = {"Ae_beta": "Ae_beta", "F_beta": "F_beta", "E_beta": "E_beta", "m": "m", "b_beta": "b_beta",
            "nu_ce_beta": "nu_"}
RTD_NAMES = {"tau1": "tau1", "tau2": "tau2", "f1": "f1", "eta1": "eta1", "eta2": "eta2", "D1": "D1", "D2": "D2",
             "J": "J", "thalf_cfc_beta": "thalf_cfc_", "lamsf6": "lamsf6", "nu_rtd_beta": "nu_"}


def _np(x):
    return x.detach().cpu().numpy() if hasattr(x, "detach") else np.asarray(x)


LIBRARY_VERSION = "0.3"


def inference_data(res, spec, sampling_time=None, wells=None, library="noblegas_rtd_mcmc_amd", observed=None):
    """Result of sampler.*DEMetropolisZ.run (samples [draw][P][L][chain]) -> dict with
    'posterior' and 'sample_stats' ({name: (dims, array)}), 'observed' (the likelihood's
    observations, az.from_pymc3's observed_data 'like'), 'attrs' and 'coords'."""
    s = _np(res["samples"])                                  # [draw, P, L, chain]
    D, P, L, W = s.shape
    by_role = {r: np.moveaxis(s[:, i], -1, 0) for i, r in enumerate(spec.roles)}   # [chain, draw, L]
    post = {}

    def put(name, arr):
        arr = np.asarray(arr, dtype=np.float64)
        if L == 1:
            post[name] = (("chain", "draw"), arr[..., 0])
        else:
            post[name] = (("chain", "draw", "well"), arr)

    both = spec.ce is not None and spec.rtd is not None
    if spec.ce is not None:
        c = spec.ce
        for role, name in CE_NAMES.items():
            put(("ce_" + name) if (both and role == "nu_ce_beta") else name, by_role[role])
        Emin = np.asarray(c.E_min)[None, None, :]
        # the reference's Deterministics 'Ae' / 'F' live in log10 space (par_bnd holds
        # log10 bounds, noble_gas_mcmc.py:183-185, 229-230); ce_exc_wrapper takes 10** (:207)
        put("Ae", by_role["Ae_beta"] * (c.logA_max - c.logA_min) + c.logA_min)
        put("F", by_role["F_beta"] * (c.logF_max - c.logF_min) + c.logF_min)
        E = by_role["E_beta"] * (c.E_max - Emin) + Emin
        b = by_role["b_beta"] * (c.b_max - c.b_min) + c.b_min
        put("E", E)
        put("b", b)
        with np.errstate(all="ignore"):
            put("T", (E - b) / by_role["m"])
        put("ce_nu" if both else "nu", by_role["nu_ce_beta"] * (c.nu_max - c.nu_min) + c.nu_min)
    if spec.rtd is not None:
        r = spec.rtd
        for role, name in RTD_NAMES.items():
            if role in by_role:
                put(name, by_role[role])
        put("nu", by_role["nu_rtd_beta"] * (r.nu_max - r.nu_min) + r.nu_min)
        if "f1" in by_role:
            f2 = 1 - by_role["f1"]
            put("f2", f2)
            put("tau", by_role["f1"] * by_role["tau1"] + f2 * by_role["tau2"])
        if "thalf_cfc_beta" in by_role:
            put("thalf_cfc", by_role["thalf_cfc_beta"] * (r.thalf[1] - r.thalf[0]) + r.thalf[0])
    # per-chain stats: [draw, chain] (one chain per walker) or [draw, L, chain] (per-well
    # chains) -> [chain, draw(, well)]
    def per_chain(a):
        a = _np(a)
        return a.T if a.ndim == 2 else np.moveaxis(a, (2, 0, 1), (0, 1, 2))
    # DEMetropolisZ's sample stats as az.from_pymc3 keeps them (the shipped traces'
    # sample_stats: accept = exp(logp(x*) - logp(x)), accepted, lambda, scaling; 'tune' is
    # dropped and DEMetropolisZ records no lp)
    acc = per_chain(res["accepted"]).astype(np.int8)
    ar = res.get("accept")
    ar = per_chain(ar).astype(np.float64) if ar is not None else np.full(acc.shape, np.nan)

    def tuned(v):        # final lamb / scaling per chain, [W] or [L][W]
        v = _np(v)
        v = v[:, None] if v.ndim == 1 else v.T[:, None, :]
        return np.broadcast_to(v, acc.shape).astype(np.float64)
    sd = ("chain", "draw") if acc.ndim == 2 else ("chain", "draw", "well")
    stats = {"lambda": (sd, tuned(res["lamb"])), "accepted": (sd, acc), "accept": (sd, ar),
             "scaling": (sd, tuned(res["scaling"]))}
    if acc.ndim == 3 and L == 1:
        stats = {k: (("chain", "draw"), v[..., 0]) for k, (dims, v) in stats.items()}
    attrs = {"created_at": datetime.datetime.now(datetime.timezone.utc).isoformat(),
             "arviz_version": "none (ArviZ 0.11.4 InferenceData layout, written by h5lite)",
             "inference_library": library,
             "inference_library_version": LIBRARY_VERSION,
             "sampler": "DEMetropolisZ (pymc3 3.11.2 algorithm, device-resident)",
             "tuning_steps": int(res.get("tuning_steps", 0)),
             "sampling_time": float(sampling_time if sampling_time is not None else res.get("sampling_time", np.nan))}
    if wells is not None and L > 1:
        attrs["wells"] = ",".join(wells)
    obs = None if observed is None else np.asarray(observed, dtype=np.float64)
    if obs is not None and obs.ndim == 2 and obs.shape[0] == 1:
        obs = obs[0]
    return {"posterior": post, "sample_stats": stats, "attrs": attrs, "observed": obs,
            "coords": {"chain": np.arange(W, dtype=np.int64), "draw": np.arange(D, dtype=np.int64),
                       "well": np.arange(L, dtype=np.int64)}}


def prior_group(spec, theta_soa):
    """The ``prior`` group az.from_pymc3(trace, prior=prior_checks) adds
    (ng_interp/noble_gas_mcmc.py:402-419: mc.sample_prior_predictive draws; the plotting at
    :544 reads idata.prior[v]): the same variable names and deterministics as the posterior
    (inference_data), dims (chain = 1, draw), from prior draws theta SoA [P][L][draws]."""
    th = np.asarray(theta_soa, dtype=np.float64)
    res = {"samples": np.moveaxis(th, -1, 0)[:, :, :, None],           # [draw, P, L, chain = 1]
           "accepted": np.zeros((th.shape[-1], 1), dtype=np.uint8), "lamb": np.zeros(1), "scaling": np.zeros(1)}
    return inference_data(res, spec)["posterior"]


class Dataset(dict):
    """One InferenceData group, the access patterns the reference's scripts use on an
    xarray Dataset: ``ds[name]`` and ``ds.name`` give the variable as a numpy array
    (``np.asarray(ds[name])`` is [chain, draw(, well)], as run_age_mcmc.py:251-276 indexes
    it), ``ds.var_dims[name]`` its dimension names, ``ds.dims`` the group's {dimension: size}
    (xarray's ``Dataset.dims``), ``ds.attrs`` the group attributes."""

    def __init__(self, variables=None, attrs=None):
        super().__init__()
        self.var_dims = {}
        self.attrs = dict(attrs or {})
        for name, (dims, arr) in (variables or {}).items():
            self[name] = np.asarray(arr)
            self.var_dims[name] = tuple(dims)

    @property
    def data_vars(self):
        return list(self.keys())

    @property
    def dims(self):
        """{dimension name: size} over the group's variables, as xarray's Dataset.dims."""
        out = {}
        for name, dims in self.var_dims.items():
            for d, n in zip(dims, np.shape(self[name])):
                out.setdefault(d, int(n))
        return out

    def __getattr__(self, name):
        try:
            return self[name]
        except KeyError:
            raise AttributeError(name) from None

    def copy(self):
        d = Dataset(attrs=self.attrs)
        for k, v in self.items():
            d[k] = v.copy()
            d.var_dims[k] = self.var_dims[k]
        return d


class InferenceData(dict):
    """What the reference's ``conv_mcmc.sample_mcmc`` returns (``az.from_pymc3(trace)``,
    run_age_mcmc_utils.py:407-429) in the form its caller consumes: groups ``posterior``,
    ``sample_stats``, ``observed_data`` (and ``prior`` when given) as :class:`Dataset`, read
    as ``mc_out['posterior'][v]`` / ``mc_out.posterior[v]`` (run_age_mcmc.py:231-276) and
    ``mc_out.copy()``.  ``raw`` extra keys (the sampler's own result: samples, logp,
    accepted, lamb, scaling, ...) sit beside the groups under their own names."""

    GROUPS = ("posterior", "sample_stats", "observed_data", "prior")

    @classmethod
    def from_dict(cls, idata, raw=None, prior=None):
        """``inference_data()``'s dict (+ the sampler result ``raw``, + a prior group dict
        {name: (dims, array)}) -> InferenceData."""
        out = cls()
        attrs = dict(idata.get("attrs", {}))
        out["posterior"] = Dataset(idata["posterior"], attrs)
        out["sample_stats"] = Dataset(idata["sample_stats"], attrs)
        if idata.get("observed") is not None:
            obs = np.asarray(idata["observed"])
            out["observed_data"] = Dataset({"like": (tuple("like_dim_%d" % i for i in range(obs.ndim)), obs)})
        if prior is not None:
            out["prior"] = Dataset(prior, attrs)
        out.attrs = attrs
        out.coords = dict(idata.get("coords", {}))
        for k, v in (raw or {}).items():
            if k not in cls.GROUPS:
                out[k] = v
        return out

    def __getattr__(self, name):
        try:
            return self[name]
        except KeyError:
            raise AttributeError(name) from None

    def groups(self):
        return [g for g in self.GROUPS if g in self]

    def copy(self):
        out = InferenceData()
        for k, v in self.items():
            out[k] = v.copy() if hasattr(v, "copy") else v
        out.attrs = dict(getattr(self, "attrs", {}))
        out.coords = dict(getattr(self, "coords", {}))
        return out

    def to_dict(self):
        """Back to ``inference_data()``'s dict layout (what ``to_netcdf`` writes)."""
        d = {g: {n: (self[g].var_dims[n], a) for n, a in self[g].items()} for g in ("posterior", "sample_stats")}
        d["attrs"] = dict(self.attrs)
        d["coords"] = dict(self.coords)
        d["observed"] = self["observed_data"]["like"] if "observed_data" in self else None
        if "prior" in self:
            d["prior"] = {n: (self["prior"].var_dims[n], a) for n, a in self["prior"].items()}
        return d


def hdi(a, hdi_prob=0.94):
    """The highest-density interval ArviZ 0.11's ``az.hdi`` returns for one unimodal sample:
    sort the values, take every window of floor(hdi_prob * n) + 1 consecutive order
    statistics and keep the narrowest (the first one on ties)."""
    a = np.sort(np.asarray(a, dtype=np.float64).ravel())
    n = a.size
    inc = int(np.floor(hdi_prob * n))
    n_int = n - inc
    if n_int <= 0:
        raise ValueError("too few draws for an HDI of %g" % hdi_prob)
    width = a[inc:] - a[:n_int]
    i = int(np.argmin(width))
    return a[i], a[i + inc]


def summary(idata, round_to=None, hdi_prob=0.94):
    """The columns of ``az.summary`` the reference's scripts read (run_age_mcmc.py:232 prints
    it and takes ``list(trace_summary.index)`` as the variable list of the posterior
    predictive loop): one row per posterior variable, mean, sd (ddof = 1) and the
    highest-density interval of ``hdi_prob`` over all chains and draws (``hdi``: the
    narrowest window, as ArviZ computes it; columns hdi_3% / hdi_97% at the default 0.94)."""
    import pandas as pd
    post = idata["posterior"]
    rows = {}
    lo_q, hi_q = (1 - hdi_prob) / 2, 1 - (1 - hdi_prob) / 2
    for name in post:
        a = np.asarray(post[name], dtype=np.float64).ravel()
        lo, hi = hdi(a, hdi_prob)
        rows[name] = {"mean": a.mean(), "sd": a.std(ddof=1) if a.size > 1 else 0.0,
                      "hdi_%g%%" % (100 * lo_q): lo, "hdi_%g%%" % (100 * hi_q): hi}
    df = pd.DataFrame.from_dict(rows, orient="index")
    return df.round(round_to) if round_to is not None else df


def to_netcdf(idata, path):
    """Write ``idata`` as ONE netCDF-4 file at ``path`` (az.to_netcdf's layout)."""
    from . import h5lite
    if isinstance(idata, InferenceData):
        idata = idata.to_dict()
    attrs = idata["attrs"]
    base = {k: attrs[k] for k in ("created_at", "arviz_version", "inference_library", "inference_library_version")}
    run = dict(base, sampling_time=np.array([float(attrs["sampling_time"])]),
               tuning_steps=np.array([int(attrs["tuning_steps"])], dtype=np.int64))
    if "wells" in attrs:                  # several wells in one file (the reference: one file per well)
        run["wells"] = attrs["wells"]
    groups = {}
    if idata.get("prior") is not None:    # az.from_pymc3(trace, prior=...) (noble_gas_mcmc.py:419)
        g = idata["prior"]
        used = []
        for dims, _ in g.values():
            used += [d for d in dims if d not in used]
        n = {d: next(a.shape[i] for dims, a in g.values() for i, dd in enumerate(dims) if dd == d) for d in used}
        groups["prior"] = {"attrs": base, "dims": {d: np.arange(n[d], dtype=np.int64) for d in used},
                           "vars": {name: (dims, np.asarray(arr), {}) for name, (dims, arr) in g.items()}}
    for gname in ("posterior", "sample_stats"):
        g = idata[gname]
        used = []
        for dims, _ in g.values():
            used += [d for d in dims if d not in used]
        gv = {}
        for name, (dims, arr) in g.items():
            a = np.asarray(arr)
            gv[name] = (dims, a, {"dtype": "bool"} if name == "accepted" else {})
        groups[gname] = {"attrs": run, "dims": {d: idata["coords"][d].astype(np.int64) for d in used}, "vars": gv}
    if idata.get("observed") is not None:
        obs = np.asarray(idata["observed"], dtype=np.float64)
        dims = tuple("like_dim_%d" % i for i in range(obs.ndim))
        groups["observed_data"] = {"attrs": base, "dims": {d: np.arange(n, dtype=np.int64) for d, n in zip(dims, obs.shape)},
                                   "vars": {"like": (dims, obs, {})}}
    h5lite.write_netcdf4(path, groups)
    return path


def from_netcdf(path):
    """Read a trace file (ours, or the reference's conv_traces/*.netcdf) into the dict layout
    of ``inference_data``."""
    from . import h5lite
    f = h5lite.read_netcdf4(path)
    out = {"attrs": {}, "coords": {}}
    for gname in ("posterior", "sample_stats", "observed_data", "prior"):
        if gname not in f:
            continue
        g = f[gname]
        if gname != "prior":              # the prior's own (chain, draw) sizes stay in its group
            for k, v in g["attrs"].items():
                v = v[0] if isinstance(v, np.ndarray) and v.shape == (1,) else v
                out["attrs"][k] = v.item() if isinstance(v, np.generic) else v
            for d, c in g["dims"].items():
                out["coords"][d] = c
        out[gname] = {name: (dims, arr) for name, (dims, arr, _) in g["vars"].items()}
    return out
