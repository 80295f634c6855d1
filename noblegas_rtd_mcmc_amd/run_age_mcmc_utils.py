"""Drop-in for ``age_ens_runs_mcmc/run_age_mcmc_utils.py`` on the GPU engine.

* ``ForwardMod(conv_kwgs, par_names, tracer)`` -- :47-163.  ``perform(node, inputs,
  outputs)`` has the Theano Op signature the reference's PyMC3 graph calls and writes
  ``outputs[0][0] = np.array(cout)``; ``batch(theta[W, P])`` evaluates W parameter vectors
  in one launch.
* ``conv_mcmc(well, tracer, obs_kwgs, conv_kwgs, prior_kwgs, savedir, savenum)`` --
  :189-462.  ``build_mcmc_model_joint_sT()`` returns the batched log-prob (ModelSpec
  compiled on the GPU) of the same priors / obs statistics / StudentT likelihood;
  ``sample_mcmc()`` runs DEMetropolisZ (one chain per walker) on the GPU instead of PyMC3,
  saves the trace in ArviZ's group layout (trace.py) and returns it as the InferenceData
  the reference's caller indexes (trace.InferenceData).
"""
import copy
import os

import numpy as np

from . import convolution_integral_utils as conv
from .engine import LogProb
from .spec import LOG10_J_HE4_DEFAULT, ModelSpec, RTDBlock, Series, Tracer


class ForwardMod:
    """Wrapper of the convolution forward model for one tracer (reference :47-163)."""
    itypes = ["dvector"]
    otypes = ["dscalar"]

    def __init__(self, conv_kwgs, par_names, tracer):
        kwargs = conv_kwgs.copy()
        self.C_t = kwargs.get('C_t', False)
        self.mod_type1 = kwargs.get('mod_type1', False)
        self.mod_type2 = kwargs.get('mod_type2', False)
        self.t_half = kwargs.get('t_half', False)
        self.rad_accum = kwargs.get('rad_accum', False)
        self.J = kwargs.get('J', False)
        self.eta = kwargs.get('eta', False)
        self.D = kwargs.get('D', False)
        self.bbar = kwargs.get('bbar', False)
        self.Phi_im = kwargs.get('Phi_im', False)
        self.t = tracer
        self.p_names = par_names
        self.p_dict = {'tau1': False, 'tau2': 0.0, 'f1': 1.0, 'f2': 0.0, 'eta1': False, 'eta2': False,
                       'D1': False, 'D2': False, 'J': False, 'thalf_cfc': False, 'lamsf6': False}

    def _conv(self, tau, mod_type, eta, D, J, thalf_cfc):
        c = conv.tracer_conv_integral(self.C_t, self.C_t.index[-1])
        c.update_pars(tau=tau, mod_type=mod_type, t_half=self.t_half, rad_accum=self.rad_accum, J=J,
                      eta=eta, D=D, bbar=self.bbar, Phi_im=self.Phi_im)
        if thalf_cfc is not None:
            c.t_half = thalf_cfc
            c.thalf_2_lambda(thalf_cfc)
        return c.convolve()

    def _evaluate(self, p):
        thalf = p['thalf_cfc'] if ('thalf_cfc' in self.p_names and self.t == 'CFC12') else None
        J = 10 ** np.asarray(p['J'], dtype=np.float64)
        cout1 = self._conv(p['tau1'], self.mod_type1, p['eta1'], p['D1'], J, thalf)
        cout2 = 0.0
        if self.mod_type2:
            cout2 = self._conv(p['tau2'], self.mod_type2, p['eta2'], p['D2'], J, thalf)
        cout = p['f1'] * cout1 + p['f2'] * cout2
        if self.t == 'SF6' and 'lamsf6' in p:
            cout = cout * (1 + np.asarray(p['lamsf6'], dtype=np.float64))
        return cout

    def perform(self, node, inputs, outputs):
        """Forward model of one parameter vector (reference :81-163)."""
        for i in range(len(self.p_names)):
            self.p_dict[self.p_names[i]] = inputs[0][i]
        if self.t == 'He4_ter' and self.p_dict['J'] == False:  # noqa: E712  (quirk :90)
            self.p_dict['J'] = LOG10_J_HE4_DEFAULT
        outputs[0][0] = np.array(float(self._evaluate(self.p_dict)))

    def __call__(self, theta):
        out = [[None]]
        self.perform(None, [np.asarray(theta, dtype=np.float64)], out)
        return out[0][0]

    def batch(self, theta):
        """theta [W, len(par_names)] -> cout [W] in one device launch per RTD component."""
        theta = np.asarray(theta, dtype=np.float64)
        p = dict(self.p_dict)
        for i, name in enumerate(self.p_names):
            p[name] = theta[:, i]
        if self.t == 'He4_ter' and 'J' not in self.p_names and p['J'] == False:  # noqa: E712
            p['J'] = LOG10_J_HE4_DEFAULT
        return np.broadcast_to(self._evaluate(p), (theta.shape[0],)).astype(np.float64)


def _series_from_frame(C_t, tracer, rad_accum):
    vals, idx = conv._series_arrays(C_t, rad_accum)
    return Series.from_reference_frame(vals, idx, idx[-1])


class conv_mcmc:
    """conv_mcmc of the reference (:189-462) on the batched GPU log-prob."""

    def __init__(self, well, tracer, obs_kwgs, conv_kwgs, prior_kwgs, savedir, savenum, max_walkers=4096,
                 device=0):
        self.well = well
        self.tracer = list(tracer)
        pk = prior_kwgs
        self.tau1_low, self.tau1_high = pk.get('tau1_low', False), pk.get('tau1_high', False)
        self.f1_low, self.f1_high = pk.get('f1_low', False), pk.get('f1_high', False)
        self.tau2_low, self.tau2_high = pk.get('tau2_low', False), pk.get('tau2_high', False)
        self.eta1_low, self.eta1_high = pk.get('eta1_low', False), pk.get('eta1_high', False)
        self.eta2_low, self.eta2_high = pk.get('eta2_low', False), pk.get('eta2_high', False)
        self.D1_low, self.D1_high = pk.get('D1_low', False), pk.get('D1_high', False)
        self.D2_low, self.D2_high = pk.get('D2_low', False), pk.get('D2_high', False)
        self.J_mu, self.J_sd = pk.get('J_mu', False), pk.get('J_sd', False)
        self.cfc_thalf_lo, self.cfc_thalf_hi = pk.get('cfc_thalf_lo', False), pk.get('cfc_thalf_hi', False)
        self.par_names = pk.get('par_names', False)
        self.obs = obs_kwgs.copy()
        self.conv_kwgs = conv_kwgs.copy()
        self.mod_type1 = conv_kwgs.get('mod_type1', False)
        self.mod_type2 = conv_kwgs.get('mod_type2', False)
        self.savedir, self.savenum = savedir, savenum
        self.max_walkers = max_walkers
        self.device = device
        self.idata = None
        self._lp = None
        tl = '.'.join(self.tracer)
        mt = '{}-{}'.format(self.mod_type1, self.mod_type2) if self.mod_type2 else self.mod_type1
        # :255 -- ONE netCDF-4 (HDF5) file, az.to_netcdf's container (trace.to_netcdf)
        self.trace_name = os.path.join(savedir, '{}.{}.{}.{}.netcdf'.format(well, tl, mt, savenum))

    def frombeta(self, betaval, low, high):
        return betaval * (high - low) + low

    def fromlog(self, logval):
        return 10 ** logval

    def obs_stats(self):
        """:353-356 -- mu = mean(ens), sd = std(ens) + mu * perr."""
        mu = np.array([np.asarray(self.obs[w]['obs_df'], dtype=np.float64).mean() for w in self.tracer])
        nerr = np.array([np.asarray(self.obs[w]['obs_df'], dtype=np.float64).std() for w in self.tracer])
        perr = mu * np.array([self.obs[w]['obs_perr'] for w in self.tracer])
        return mu, nerr + perr

    def spec(self):
        mu, sd = self.obs_stats()
        trs = []
        for w in self.tracer:
            kw = self.conv_kwgs[w]
            accum = kw.get('rad_accum', False) or None
            trs.append(Tracer(w, _series_from_frame(kw['C_t'], w, accum), t_half=kw.get('t_half', False) or None,
                              rad_accum=accum, log10_J=LOG10_J_HE4_DEFAULT if w == 'He4_ter' else None))
        names = [p for p in self.par_names if p != 'f2']
        blk = RTDBlock(tracers=trs, obs=mu[None, :], sd=sd[None, :], mod_type1=self.mod_type1,
                       mod_type2=self.mod_type2 or None, par_names=names,
                       tau1=(self.tau1_low, self.tau1_high),
                       tau2=(self.tau2_low, self.tau2_high) if 'tau2' in names else (50.0, 15000.0),
                       f1=(self.f1_low, self.f1_high) if 'f1' in names else (0.01, 0.99),
                       eta1=(self.eta1_low, self.eta1_high) if 'eta1' in names else (1.0, 5.0),
                       eta2=(self.eta2_low, self.eta2_high) if 'eta2' in names else (1.0, 5.0),
                       D1=(self.D1_low, self.D1_high) if 'D1' in names else (0.01, 2.0),
                       D2=(self.D2_low, self.D2_high) if 'D2' in names else (0.01, 2.0),
                       J_mu=self.J_mu if 'J' in names else LOG10_J_HE4_DEFAULT,
                       J_sd=self.J_sd if 'J' in names else 0.33,
                       thalf=(self.cfc_thalf_lo, self.cfc_thalf_hi) if 'thalf_cfc' in names else (5.0, 35.0))
        return ModelSpec(n_wells=1, rtd=blk)

    def build_mcmc_model_joint_sT(self):
        """The batched log-prob of the reference model (priors + StudentT, :275-397)."""
        if self._lp is None:
            self._lp = LogProb(self.spec(), self.max_walkers, self.device)
        return self._lp

    def sample_mcmc(self, chains=3, tune=10000, draws=10000, seed=123423, tune_interval=1000, sampler="device",
                    space="transformed", nwalkers=None, start="test_point"):
        """DEMetropolisZ on the GPU log-prob (replaces mc.sample, :407-429, with its
        arguments as defaults: 3 chains, tune 10 000, draws 10 000, seed 123423,
        tune_interval 1000), one chain per walker of this one well.  sampler: "device"
        (ngrtd_demcz_run, device-resident) or "torch" (sampler.DEMetropolisZ on torch ops;
        same random stream).  space: "transformed" (PyMC3's: logodds / interval / log; the
        log-prob adds the Jacobian) or "natural".  ``nwalkers``: alias of ``chains``.
        ``start``: "test_point" (PyMC3's default for a non-NUTS step: every chain starts at
        model.test_point, workloads.test_point) or "prior" (independent prior draws, seeded).

        Returns what the reference returns, the InferenceData of the run
        (trace.InferenceData: ``out['posterior'][v]`` is [chain, draw], the indexing of
        run_age_mcmc.py:251-276), with the sampler's own result fields (samples, logp,
        accepted, lamb, scaling, roles, ...) beside the groups."""
        import torch
        from .sampler import sample_model
        from .workloads import sample_prior, test_point
        if nwalkers is not None:
            chains = nwalkers
        if start not in ("test_point", "prior"):
            raise ValueError('start must be "test_point" or "prior"')
        lp = self.build_mcmc_model_joint_sT()
        x0 = test_point(lp.spec, chains) if start == "test_point" else sample_prior(lp.spec, chains,
                                                                                     np.random.default_rng(seed))
        x = torch.from_numpy(x0).to("cuda:%d" % self.device)
        res = sample_model(lp.spec, self.max_walkers, self.device, x, tune, draws, seed, tune_interval, sampler,
                           space, cache=self.__dict__)
        from . import trace
        idd = trace.inference_data(res, lp.spec, wells=[self.well], observed=lp.spec.rtd.obs)
        raw = {k: (v.cpu().numpy() if hasattr(v, "cpu") else v) for k, v in res.items()}
        raw["roles"] = list(lp.spec.roles)
        out = trace.InferenceData.from_dict(idd, raw=raw)
        if self.savedir:
            # az.to_netcdf(idata, self.trace_name) (:425): same groups / names / attrs
            trace.to_netcdf(out, self.trace_name)
        self.idata = out
        return out


def deepcopy_kwargs(kw):
    return copy.deepcopy(kw)
