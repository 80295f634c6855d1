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
