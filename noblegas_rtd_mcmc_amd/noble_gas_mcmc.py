"""The CE noble-gas inference model of ``ng_interp/noble_gas_mcmc.py`` on the GPU engine.

* ``ce_exc_wrapper(theta)``  -- :205-213, theta = [log10 Ae, log10 F, E, T] -> conc[G]
  (the Theano ``as_op`` boundary of the reference, here a plain function; W=1 of the
  batched kernel).
* ``CEModel``                -- ``mcmc_model()`` (:216-267): priors, the T = (E-b)/m
  lapse-rate mapping and the StudentT likelihood, compiled to one batched log-prob over an
  ensemble of walkers; ``sample()`` replaces ``mc.sample(step=DEMetropolisZ)`` (:408-415).
* ``frombeta`` / ``find_T_lapse`` -- :189-199, :50-63.
"""
import numpy as np

from . import noble_gas_utils as ng
from .engine import LogProb
from .spec import CEBlock, ModelSpec

GASES_DEFAULT = ('Ne', 'Ar', 'Kr', 'Xe')                                      # :109
ERR_DEFAULT = {'He': 1.5, 'Ne': 1.5, 'Ar': 2.5, 'Kr': 3.1, 'Xe': 15.1}        # :107
WELL_ELEV = {'PLM1': 2786.889893, 'PLM6': 2759.569824, 'PLM7': 2782.550049}   # :80-82
PAR_ORDER = ('Ae_beta', 'F_beta', 'E_beta', 'm', 'b_beta', 'nu_')


def find_T_lapse(E_lapse, E_lapse_int, lapse_slope):
    """:50-63."""
    return (E_lapse - E_lapse_int) / lapse_slope


def ce_exc_wrapper(theta, gases=GASES_DEFAULT):
    """:205-213 -- [log10 Ae, log10 F, E, T] -> CE concentrations (add_eq_conc=True)."""
    Ae_log, F_log, E, T = theta
    Ae, F = 10 ** Ae_log, 10 ** F_log
    ce_mod = ng.noble_gas_fun(gases=list(gases), E=E, T=T, Ae=Ae, F=F, P='lapse_rate').ce_exc(add_eq_conc=True)
    return np.array([ce_mod[i] for i in gases])


def frombeta(plist, blist, par_bnd_):
    """:189-199 -- map Beta [0, 1] values onto [min, max] parameter bounds."""
    vals = list(blist)
    for i, p in enumerate(plist):
        vals[i] = blist[i] * (par_bnd_[p]['max'] - par_bnd_[p]['min']) + par_bnd_[p]['min']
    return vals


class CEModel:
    """mcmc_model() of noble_gas_mcmc.py:216-267 for one or several wells.

    obs: {well: {gas: value}} (the xlsx rows, :72-78); err_dict: percent errors (:107).
    Walkers carry, per well, (Ae_beta, F_beta, E_beta, m, b_beta, nu_) in natural space.
    """

    def __init__(self, obs, wells, gases=GASES_DEFAULT, err_dict=None, well_elev=None, lapse_slope=-146.0,
                 err_lapse_slope=17.0, lapse_b=3354.0, Amin=1.0e-4, Amax=1.0e-1, Fmin=1.0e-1, Fmax=1.0e+1,
                 Emax=3300.0, max_walkers=4096, device=0):
        err_dict = err_dict or ERR_DEFAULT
        well_elev = well_elev or WELL_ELEV
        self.wells = list(wells)
        self.gases = tuple(gases)
        obs_mu = np.array([[obs[w][g] for g in self.gases] for w in self.wells])
        obs_sd = obs_mu * np.array([err_dict[g] / 100 for g in self.gases])          # :256
        err_b = abs(lapse_slope) * 2.5                                                # :129
        block = CEBlock(obs=obs_mu, sd=obs_sd, E_min=np.array([well_elev[w] - 10.0 for w in self.wells]),
                        gases=self.gases, E_max=Emax, logA_min=float(np.log10(Amin)), logA_max=float(np.log10(Amax)),
                        logF_min=float(np.log10(Fmin)), logF_max=float(np.log10(Fmax)),
                        b_min=lapse_b - err_b, b_max=lapse_b + err_b, m_mu=lapse_slope, m_sd=err_lapse_slope)
        self.spec = ModelSpec(n_wells=len(self.wells), ce=block)
        self.max_walkers = max_walkers
        self.device = device
        self._lp = None

    @property
    def logp(self):
        if self._lp is None:
            self._lp = LogProb(self.spec, self.max_walkers, self.device)
        return self._lp

    def log_prob(self, theta):
        """theta [W][L*6] (or torch [6][L][W] on the device) -> [W]."""
        return self.logp(theta)

    def deterministics(self, theta_soa):
        """E, b, T, nu of theta SoA [6][L][W] (the mc.Deterministic nodes, :229-250) and Ae, F
        as LINEAR values -- 10 ** the reference's log10 Deterministics 'Ae' / 'F' (:229-230), i.e.
        what ce_exc_wrapper feeds the model (:207) and what the reference's plots convert
        them to (:281-283, :438-440).  The trace keeps the log10 values (trace.py)."""
        c = self.spec.ce
        t = np.asarray(theta_soa)
        Ae = 10 ** (t[0] * (c.logA_max - c.logA_min) + c.logA_min)
        F = 10 ** (t[1] * (c.logF_max - c.logF_min) + c.logF_min)
        E = t[2] * (c.E_max - c.E_min[:, None]) + c.E_min[:, None]
        b = t[4] * (c.b_max - c.b_min) + c.b_min
        T = (E - b) / t[3]
        nu = t[5] * (c.nu_max - c.nu_min) + c.nu_min
        return {"Ae": Ae, "F": F, "E": E, "b": b, "m": t[3], "T": T, "nu": nu}

    def sample(self, nwalkers=100, tune=500, draws=500, seed=12345, tune_interval=100, sampler="device",
               space="transformed", prior_samples=10000, start="test_point"):
        """DEMetropolisZ on the GPU log-prob (replaces mc.sample, :408-415): one chain per
        (walker, well), each well its own model as the reference runs them (logp / accepted
        [draws][L][W]).  sampler: "device" (ngrtd_demcz_run, device-resident) or "torch"
        (sampler.DEMetropolisZ on torch ops; same random stream).  space: "transformed"
        (PyMC3's: logodds for the Beta variables; the log-prob adds the Jacobian) or
        "natural".  start: "test_point" (PyMC3's default start for a non-NUTS step: every chain
        at model.test_point) or "prior" (independent prior draws, seeded)."""
        import torch
        from .sampler import sample_model
        from .workloads import sample_prior, test_point
        if start not in ("test_point", "prior"):
            raise ValueError('start must be "test_point" or "prior"')
        x0 = (test_point(self.spec, nwalkers) if start == "test_point"
              else sample_prior(self.spec, nwalkers, np.random.default_rng(seed)))
        x = torch.from_numpy(x0).to("cuda:%d" % self.device)
        res = sample_model(self.spec, self.max_walkers, self.device, x, tune, draws, seed, tune_interval, sampler,
                           space, cache=self.__dict__)
        from . import trace
        idd = trace.inference_data(res, self.spec, wells=self.wells, observed=self.spec.ce.obs)
        res["samples"] = res["samples"].cpu().numpy()
        res["logp"] = res["logp"].cpu().numpy()
        res["idata"] = trace.InferenceData.from_dict(idd, prior=self.prior_checks(prior_samples))
        return res

    def prior_checks(self, samples=10000, seed=10):
        """The prior group az.from_pymc3(trace, prior=prior_checks) stores (:276-283, :419):
        ``samples`` prior draws of every variable and deterministic (one chain), with Ae / F
        converted to linear values as the reference does before storing them (:281-283).
        Draws from NumPy's generator (seed 10), not PyMC3's stream (not installed here); the
        likelihood's prior-predictive 'like' draws are not included."""
        from . import trace
        from .workloads import sample_prior
        th = sample_prior(self.spec, int(samples), np.random.default_rng(seed))
        g = trace.prior_group(self.spec, th)
        for p in ("Ae", "F"):
            dims, a = g[p]
            g[p] = (dims, 10 ** a)
        return g
