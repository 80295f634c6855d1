"""Posterior traces in ArviZ's InferenceData layout (the reference's az.to_netcdf).

The reference saves every run with ``az.to_netcdf(az.from_pymc3(trace), trace_name)``
(age_ens_runs_mcmc/run_age_mcmc_utils.py:420-425; ArviZ 0.11.4, PyMC3 3.11.2): a netCDF4
file with a ``posterior`` group -- one variable per PyMC3 random variable AND
deterministic, dims (chain, draw[, ...]) -- a ``sample_stats`` group (the step method's
stats: lp, accepted, tune, scaling, lambda) and attributes (created_at,
inference_library, sampling_time [s], tuning_steps).

netCDF4/HDF5 writers (h5py, netCDF4, xarray) are not available in this image, so
``to_netcdf`` writes the SAME groups as one netCDF-3 file per group into a directory
(``<trace>/posterior.nc``, ``<trace>/sample_stats.nc``, classic format through
scipy.io.netcdf_file -- readable by xarray's scipy engine, hence by
``az.InferenceData(posterior=xr.open_dataset(".../posterior.nc"), sample_stats=...)``),
with the global attributes on every group file.  Variable names follow the reference
models: CE (ng_interp/noble_gas_mcmc.py:216-267) Ae_beta, F_beta, E_beta, m, b_beta, nu_
and the deterministics Ae, F, E, b, T, nu; RTD (run_age_mcmc_utils.py:286-344) tau1,
nu_, nu, J, tau2, f1, f2, tau, eta1, eta2, D1, D2, thalf_cfc_, thalf_cfc, lamsf6.  A
model with both blocks prefixes the CE nu variables with ``ce_``.  Walkers are chains;
a model of several wells gets a trailing ``well`` dim.
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


def inference_data(res, spec, sampling_time=None, wells=None, library="noblegas_rtd_mcmc_amd"):
    """Result of sampler.*DEMetropolisZ.run (samples [draw][P][L][chain]) -> dict with
    'posterior' and 'sample_stats' ({name: (dims, array)}) and 'attrs'."""
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
    lp = per_chain(res["logp"]).astype(np.float64)
    acc = per_chain(res["accepted"]).astype(np.int8)

    def tuned(v):        # final lamb / scaling per chain, [W] or [L][W]
        v = _np(v)
        v = v[:, None] if v.ndim == 1 else v.T[:, None, :]
        return np.broadcast_to(v, lp.shape).astype(np.float64)
    sd = ("chain", "draw") if lp.ndim == 2 else ("chain", "draw", "well")
    stats = {"lp": (sd, lp), "accepted": (sd, acc), "tune": (sd, np.zeros_like(acc)),
             "lambda": (sd, tuned(res["lamb"])), "scaling": (sd, tuned(res["scaling"]))}
    if lp.ndim == 3 and L == 1:
        stats = {k: (("chain", "draw"), v[..., 0]) for k, (dims, v) in stats.items()}
    attrs = {"created_at": datetime.datetime.now(datetime.timezone.utc).isoformat(),
             "inference_library": library,
             "sampler": "DEMetropolisZ (pymc3 3.11.2 algorithm, device-resident)",
             "tuning_steps": int(res.get("tuning_steps", 0)),
             "sampling_time": float(sampling_time if sampling_time is not None else res.get("sampling_time", np.nan))}
    if wells is not None and L > 1:
        attrs["wells"] = ",".join(wells)
    return {"posterior": post, "sample_stats": stats, "attrs": attrs,
            "coords": {"chain": np.arange(W, dtype=np.int64), "draw": np.arange(D, dtype=np.int64),
                       "well": np.arange(L, dtype=np.int64)}}


def to_netcdf(idata, path):
    """Write the groups as <path>/<group>.nc (netCDF-3 classic, one file per group)."""
    from scipy.io import netcdf_file
    os.makedirs(path, exist_ok=True)
    for group in ("posterior", "sample_stats"):
        fn = os.path.join(path, group + ".nc")
        with netcdf_file(fn, "w", version=2) as f:
            for k, v in idata["attrs"].items():
                setattr(f, k, v)
            dims_used = set()
            for dims, _ in idata[group].values():
                dims_used.update(dims)
            for d in ("chain", "draw", "well"):
                if d in dims_used:
                    f.createDimension(d, len(idata["coords"][d]))
                    cv = f.createVariable(d, "i", (d,))
                    cv[:] = idata["coords"][d].astype(np.int32)
            for name, (dims, arr) in idata[group].items():
                v = f.createVariable(name, "d" if arr.dtype.kind == "f" else "b", dims)
                v[:] = arr
    return path


def from_netcdf(path):
    """Read a trace written by to_netcdf back into the same dict layout."""
    from scipy.io import netcdf_file
    out = {"attrs": {}, "coords": {}}
    for group in ("posterior", "sample_stats"):
        with netcdf_file(os.path.join(path, group + ".nc"), "r", mmap=False) as f:
            grp = {}
            for name, v in f.variables.items():
                if name in ("chain", "draw", "well"):
                    out["coords"][name] = np.array(v[:])
                    continue
                grp[name] = (tuple(v.dimensions), np.array(v[:]))
            out[group] = grp
            for k, v in f._attributes.items():
                out["attrs"][k] = v.decode() if isinstance(v, bytes) else v
    return out
