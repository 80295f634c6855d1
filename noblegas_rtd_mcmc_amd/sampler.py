"""Ensemble Differential-Evolution Metropolis sampler over the batched log-prob.

The reference samples with PyMC3 3.11.2 ``DEMetropolisZ`` (run_age_mcmc_utils.py:412-417,
ng_interp/noble_gas_mcmc.py:410-415): one log-prob per proposal per chain, chains in
separate processes.  Here the whole ensemble of W walkers moves at once (population
DE-MC, ter Braak 2006 -- PyMC3's ``DEMetropolis`` flavour): every step proposes

    x*_i = x_i + lamb * (x_r1 - x_r2) + eps_i,   r1 != r2 != i,  eps ~ U(-scaling, scaling)

for all walkers, evaluates ONE batched log-prob on the GPU and accepts per walker with the
Metropolis rule.  ``scaling`` is tuned every ``tune_interval`` steps with PyMC3's
acceptance-rate schedule (pymc3/step_methods/metropolis.py ``tune``); ``lamb`` defaults to
2.38 / sqrt(2 d) as in PyMC3.  Walkers are the LAST axis of every array ([..., W]), which
is the structure-of-arrays layout the engine consumes with no transposes.

Runs on torch tensors (CUDA for the GPU engine, CPU for tests with a CPU log-prob).
"""
import math

import torch


def pymc3_tune(scale, acc_rate):
    """pymc3.step_methods.metropolis.tune (3.11): multiplicative scaling update."""
    if acc_rate < 0.001:
        return scale * 0.1
    if acc_rate < 0.05:
        return scale * 0.5
    if acc_rate < 0.2:
        return scale * 0.9
    if acc_rate > 0.95:
        return scale * 10.0
    if acc_rate > 0.75:
        return scale * 2.0
    if acc_rate > 0.5:
        return scale * 1.1
    return scale


class DEMetropolis:
    """Vectorised population DE-MC over walkers (last axis)."""

    def __init__(self, log_prob, lamb=None, scaling=1e-3, tune_interval=100, seed=123423):
        self.log_prob = log_prob
        self.lamb = lamb
        self.scaling = scaling
        self.tune_interval = tune_interval
        self.seed = seed

    def run(self, x0, tune, draws, thin=1, callback=None):
        """x0: [..., W] tensor.  Returns dict(samples [n_kept, ..., W], logp [n_kept, W],
        accept_rate, scaling)."""
        x = x0.clone()
        W = x.shape[-1]
        d = int(x[..., 0].numel())
        if W < 3:
            raise ValueError("population DE needs at least 3 walkers")
        lamb = self.lamb if self.lamb is not None else 2.38 / math.sqrt(2 * d)
        g = torch.Generator(device=x.device)
        g.manual_seed(self.seed)
        lp = self.log_prob(x)
        scaling = self.scaling
        samples, logps = [], []
        n_acc_window = torch.zeros((), dtype=torch.float64, device=x.device)
        n_acc_total = torch.zeros((), dtype=torch.float64, device=x.device)
        idx = torch.arange(W, device=x.device)
        for it in range(tune + draws):
            # two distinct partners r1 != r2, both != i
            r1 = (idx + torch.randint(1, W, (W,), generator=g, device=x.device)) % W
            off = torch.randint(1, W - 1, (W,), generator=g, device=x.device)
            r2 = (r1 + off) % W
            r2 = torch.where(r2 == idx, (r2 + 1) % W, r2)
            r2 = torch.where(r2 == r1, (r2 + 1) % W, r2)
            eps = (torch.rand(x.shape, generator=g, device=x.device, dtype=x.dtype) * 2 - 1) * scaling
            prop = x + lamb * (x[..., r1] - x[..., r2]) + eps
            lp_prop = self.log_prob(prop)
            logu = torch.log(torch.rand((W,), generator=g, device=x.device, dtype=lp.dtype))
            acc = (lp_prop - lp) > logu
            acc = acc & ~torch.isnan(lp_prop)
            x = torch.where(acc, prop, x)
            lp = torch.where(acc, lp_prop, lp)
            na = acc.sum().to(torch.float64)
            n_acc_window += na
            if it >= tune:
                n_acc_total += na
                if (it - tune) % thin == 0:
                    samples.append(x.clone())
                    logps.append(lp.clone())
            elif (it + 1) % self.tune_interval == 0:
                rate = float(n_acc_window) / (self.tune_interval * W)
                scaling = pymc3_tune(scaling, rate)
                n_acc_window.zero_()
            if callback is not None:
                callback(it, x, lp)
        return {"samples": torch.stack(samples) if samples else x[None][:0],
                "logp": torch.stack(logps) if logps else lp[None][:0],
                "accept_rate": float(n_acc_total) / max(1, draws * W),
                "scaling": scaling, "lamb": lamb}


class DeviceDEMetropolis:
    """The same population DE-MC as DEMetropolis, run device-resident by libngrtd
    (ngrtd_demc_run: a proposal kernel + the log-prob kernel with the Metropolis accept in
    its per-walker reduction, 2 launches per step, counter-based random numbers).  The host
    only intervenes every ``tune_interval`` steps (PyMC3 scaling schedule) and every
    ``thin`` draws (sample snapshot).  Same result dict as DEMetropolis.run; the random
    stream differs, so chains match DEMetropolis in distribution, not bit for bit."""

    def __init__(self, logprob, lamb=None, scaling=1e-3, tune_interval=100, seed=123423):
        self.lp = logprob               # engine.LogProb
        self.lamb = lamb
        self.scaling = scaling
        self.tune_interval = tune_interval
        self.seed = seed

    def run(self, x0, tune, draws, thin=1, callback=None):
        x = x0.clone().contiguous()
        W = x.shape[-1]
        d = int(x[..., 0].numel())
        if W < 3:
            raise ValueError("population DE needs at least 3 walkers")
        lamb = self.lamb if self.lamb is not None else 2.38 / math.sqrt(2 * d)
        lp = self.lp(x).clone()
        cnt = torch.zeros(1, dtype=torch.int64, device=x.device)
        scaling = self.scaling
        step = 0
        # tuning: chunks of tune_interval steps, PyMC3 schedule on the chunk's rate
        while step < tune:
            n = min(self.tune_interval, tune - step)
            cnt.zero_()
            self.lp.demc(x, lp, n, lamb, scaling, self.seed, step, n_accepted=cnt)
            step += n
            if n == self.tune_interval:
                scaling = pymc3_tune(scaling, float(cnt.item()) / (n * W))
            if callback is not None:
                callback(step - 1, x, lp)
        samples, logps = [], []
        cnt.zero_()
        kept = 0
        while kept * thin < draws:
            n = min(thin, draws - kept * thin)
            self.lp.demc(x, lp, n, lamb, scaling, self.seed, step, n_accepted=cnt)
            step += n
            samples.append(x.clone())
            logps.append(lp.clone())
            kept += 1
            if callback is not None:
                callback(step - 1, x, lp)
        return {"samples": torch.stack(samples) if samples else x[None][:0],
                "logp": torch.stack(logps) if logps else lp[None][:0],
                "accept_rate": float(cnt.item()) / max(1, draws * W),
                "scaling": scaling, "lamb": lamb}
