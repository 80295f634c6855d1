"""Rebuild the ModelSpecs stored in tests/golden/logp_golden.npz (self-contained: the
series and obs are in the fixture, so the spec does not depend on package data)."""
import numpy as np

from noblegas_rtd_mcmc_amd.spec import CEBlock, ModelSpec, RTDBlock, Series
from noblegas_rtd_mcmc_amd import workloads as wl


def spec_from_golden(z, prefix):
    L = int(z[prefix + "_L"])
    ce = rtd = None
    if prefix + "_ce_obs" in z:
        ce = CEBlock(obs=z[prefix + "_ce_obs"], sd=z[prefix + "_ce_sd"], E_min=z[prefix + "_ce_Emin"],
                     gases=tuple(str(g) for g in z[prefix + "_ce_gases"]))
    if prefix + "_rtd_obs" in z:
        names = [str(t) for t in z[prefix + "_rtd_tracers"]]
        series = z[prefix + "_rtd_series"]
        trs = []
        for name, c in zip(names, series):
            t = wl.tracer(name, series=Series(c, np.arange(len(c), dtype=np.float64), 0.0),
                          log10_J=wl.LOG10_J_HE4_DEFAULT if name == "He4_ter" else None)
            if name == "He4_ter":
                t.series = Series(c, np.arange(len(c), dtype=np.float64), 0.0)
            trs.append(t)
        m1, m2 = [str(m) for m in z[prefix + "_rtd_mods"]]
        rtd = RTDBlock(tracers=trs, obs=z[prefix + "_rtd_obs"], sd=z[prefix + "_rtd_sd"], mod_type1=m1,
                       mod_type2=m2 or None, par_names=tuple(str(p) for p in z[prefix + "_rtd_par_names"]))
    return ModelSpec(n_wells=L, ce=ce, rtd=rtd), z[prefix + "_theta"]


def pymc3_runs():
    """The reference runs frozen by tests/golden/make_pymc3_accept.py: [(key, entry, arrays)]
    with entry the fit report (trace name, well, tracers, models, savenum, tau1 bounds, mu, the
    fitted sigma, role order) and arrays the fixture's x0 / x1 [n][P] natural-space states and
    dlogp [n] = log(accept) of each kept accepted transition."""
    import json
    import os
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    rep = json.load(open(os.path.join(here, "pymc3_accept_fit.json")))
    z = np.load(os.path.join(here, "pymc3_accept.npz"), allow_pickle=False)
    out = []
    for key in sorted(rep):
        out.append((key, rep[key], {k: z[key + "_" + k] for k in ("x0", "x1", "dlogp", "mu", "sd", "tau1")}))
    return out


def pymc3_run_spec(entry, jacobian=True):
    """The reference run's RTD model (run_age_mcmc.py:140-224: one well, its tracers on the full
    shipped series N = 25 256, its models, savenum, tau1 bounds) with the trace's mu and the
    fitted sigma; PyMC3's transformed-space log-prob (jacobian=True) unless asked otherwise."""
    sv = "" if entry["savenum"] == "0" else entry["savenum"]
    pn = wl.model_par_names(entry["mod1"], entry["mod2"], sv)
    rtd = RTDBlock(tracers=[wl.tracer(t, None) for t in entry["tracers"]], obs=np.array([entry["mu"]]),
                   sd=np.array([entry["sd"]]), mod_type1=entry["mod1"], mod_type2=entry["mod2"], par_names=pn,
                   tau1=tuple(entry["tau1"]))
    spec = ModelSpec(n_wells=1, rtd=rtd, jacobian=jacobian)
    assert list(spec.roles) == list(entry["roles"])
    return spec
