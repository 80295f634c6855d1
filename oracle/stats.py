"""Restatement of the PyMC3 3.11.2 log-densities used by the reference models.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  PyMC3 is a third-party dependency
of the reference (pymc3==3.11.2, read from the inference_library_version attribute of
age_ens_runs_mcmc/conv_traces/*.netcdf) and is not installed here; these are its
published formulas (pymc3/distributions/continuous.py, StudentT/Beta/Normal/Uniform/
HalfNormal .logp, each wrapped in ``bound`` -> -inf outside the support).  Pinned in
tests against scipy.stats (t, beta, norm, uniform, halfnorm).
"""
import math

import numpy as np
from scipy.special import gammaln

NEG_INF = -np.inf


def studentt_logp(value, mu, sigma, nu):
    lam = sigma ** -2.0
    with np.errstate(all="ignore"):
        lp = (gammaln((nu + 1.0) / 2.0) + 0.5 * np.log(lam / (nu * np.pi)) - gammaln(nu / 2.0)
              - (nu + 1.0) / 2.0 * np.log1p(lam * (value - mu) ** 2 / nu))
    ok = (lam > 0) & (nu > 0) & (sigma > 0)
    return np.where(ok, lp, NEG_INF)


def betaln(a, b):
    return gammaln(a) + gammaln(b) - gammaln(a + b)


def beta_logp(x, alpha, beta):
    with np.errstate(all="ignore"):
        lp = ((0.0 if alpha == 1 else (alpha - 1) * np.log(x))
              + (0.0 if beta == 1 else (beta - 1) * np.log1p(-x)) - betaln(alpha, beta))
    return np.where((x >= 0) & (x <= 1), lp, NEG_INF)


def normal_logp(x, mu, sigma):
    tau = sigma ** -2.0
    return (-tau * (x - mu) ** 2 + np.log(tau / np.pi / 2.0)) / 2.0


def uniform_logp(x, lower, upper):
    return np.where((x >= lower) & (x <= upper), -np.log(upper - lower), NEG_INF)


def halfnormal_logp(x, sigma):
    tau = sigma ** -2.0
    return np.where(x >= 0, -0.5 * tau * x ** 2 + 0.5 * np.log(tau * 2.0 / np.pi), NEG_INF)


# PyMC3 default transforms' log|Jacobian| (pymc3/distributions/transforms.py):
# logodds for Beta, interval for Uniform, log for HalfNormal.  "Parity unpinned".
def jac_logodds(x):
    with np.errstate(all="ignore"):
        return np.log(x) + np.log1p(-x)


def jac_interval(x, a, b):
    with np.errstate(all="ignore"):
        return np.log(x - a) + np.log(b - x) - np.log(b - a)


def jac_log(x):
    with np.errstate(all="ignore"):
        return np.log(x)


LOG_PI = math.log(math.pi)
