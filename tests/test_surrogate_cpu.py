"""The piecewise-Chebyshev surrogate of the exponential RTD channel sums (host-only part of
libngrtd: ngrtd_surrogate_check, no GPU needed).

The log-prob kernel replaces Y_c(tau) = sum_{j>=0} A_c[1+j] exp(-j/tau) -- the exponential
weights of convolution_integral_utils.py:184 against the decay-folded input series
(:305-340) -- by a Chebyshev expansion in log(tau).  A plan uses it only when the library's
own validation bound (5e-14 relative) holds; these tests check that the bound holds for
the shipped series at both input lengths and for the c4 workload, and evaluate the
returned coefficients independently in NumPy against a direct float64 sum.
"""
import ctypes as C

import numpy as np
import pytest

from noblegas_rtd_mcmc_amd import workloads

N_COEF, PIECES = 12, 77
SUB, OCT0, OCTS, S_HI = 4, -1, 19, 2.0 ** -18


@pytest.fixture(scope="module")
def lib():
    import __graft_entry__ as g
    g.build()
    from noblegas_rtd_mcmc_amd import _lib
    return _lib.load()


def channels(tracers):
    """Channel columns as the plan builds them (ngrtd.hip build_table)."""
    cols = []
    for t in tracers:
        s = t.series
        tp = np.arange(s.n, dtype=np.float64) + s.dtp
        tp[0] = 1e-5 + s.dtp
        lam = -np.log(0.5) / t.t_half if t.t_half else 0.0
        e = np.exp(-lam * tp)
        d = (1 - e) if t.rad_accum == "3He" else e
        hasB = t.rad_accum in ("4He", "SF6")
        if np.any(s.c_by_age != 0) or not hasB:
            cols.append(s.c_by_age * d)
        if hasB:
            cols.append(s.idx_by_age * d)
    return np.ascontiguousarray(cols, dtype=np.float64)


def check(lib, cols, dtp=0.0):
    Cn, N = cols.shape
    CP = (Cn + 2) & ~1
    coef = np.zeros(PIECES * N_COEF * CP)
    err = C.c_double()
    dp = C.POINTER(C.c_double)
    assert lib.ngrtd_surrogate_check(cols.ctypes.data_as(dp), Cn, N, dtp, coef.ctypes.data_as(dp),
                                     C.byref(err)) == 0
    return err.value, coef.reshape(PIECES, N_COEF, CP)


def numpy_surrogate(coef, tau, c):
    """The kernel's piece lookup (ngrtd_kernels.hpp cheb_piece) and Horner sum, in NumPy."""
    if tau >= 2.0 ** (OCT0 + OCTS):
        p, x = PIECES - 1, (1.0 / tau) * (2.0 / S_HI) - 1.0
    else:
        m, e = np.frexp(tau)                   # tau = m 2^e, m in [1/2, 1)
        m, e = 2.0 * m, e - 1
        j = int((m - 1.0) * 4.0)
        p = (e - OCT0) * SUB + j
        x = (m - (1.125 + 0.25 * j)) * 8.0
    return np.polynomial.polynomial.polyval(x, coef[p, :, c])   # monomial form of the Chebyshev fit


@pytest.mark.parametrize("n", [1200, 25256])
def test_shipped_series_within_bound(lib, n):
    trs = [workloads.tracer(name, n) for name in ("CFC11", "CFC12", "CFC113", "SF6", "H3", "He4_ter")]
    err, coef = check(lib, channels(trs))
    assert err <= 5e-14, err
    cols = channels(trs)
    j = np.arange(n - 1, dtype=np.float64)
    d01 = 1.0 - (0.0 + 1e-5)                 # tp_1 - tp_0 (dtp = 0)
    for tau in (0.5, 0.731, 1.0, 7.3, 37.3, 333.3, 1000.0, 2.2e5, 3e6, np.inf):
        q = np.exp(-j / tau)
        s01 = np.exp(-d01 / tau)
        for c in range(cols.shape[0] + 1):      # channels, then the normaliser
            col = cols[c, 1:] if c < cols.shape[0] else np.ones(n - 1)
            ref = s01 * np.dot(col, q)
            assert abs(numpy_surrogate(coef, tau, c) - ref) <= 1e-13 * ref, (tau, c)


def test_reconstructs_reference_convolution(lib):
    """(A_0 + Z_c) / (1 + Z_G) from the surrogate equals the reference convolve() of the
    exponential model (conv_golden.npz fixtures, N = 1200) for the fixture's taus >= 1/2."""
    import os
    here = os.path.dirname(os.path.abspath(__file__))
    z = np.load(os.path.join(here, "golden", "conv_golden.npz"))
    keys = [k for k in z.files if k.endswith("_exponential_1200_out")]
    assert keys
    checked = 0
    for k in keys:
        name = k.split("_exponential_")[0]
        t = workloads.tracer(name, 1200)
        if t.rad_accum in ("4He", "SF6") or name == "He3":
            continue                  # J-weighted / 3He channels: covered by the GPU tests
        cols = channels([t])
        err, coef = check(lib, cols)
        assert err <= 5e-14
        taus = z[k.replace("_out", "_tau")]
        ref = z[k]
        for tau, r in zip(taus, ref):
            if not tau >= 0.5:
                continue
            val = (cols[0, 0] + numpy_surrogate(coef, tau, 0)) / (1 + numpy_surrogate(coef, tau, 1))
            assert abs(val - r) <= 1e-12 * abs(r), (name, tau, val, r)
            checked += 1
    assert checked >= 50, checked


def test_c4_workload_series_within_bound(lib):
    spec = workloads.c4_spec(L=4)
    err, _ = check(lib, channels(spec.rtd.tracers))
    assert err <= 5e-14, err


def test_positive_rough_series_within_bound(lib):
    """Non-negative columns of any roughness stay within the bound: each term exp(-j/tau)
    is analytic in log(tau) with |.| <= 1 in the strip |Im log tau| < pi/2, whatever A is."""
    rng = np.random.default_rng(5)
    col = 10.0 ** rng.uniform(-8, 8, 1200)
    err, _ = check(lib, np.ascontiguousarray(col[None, :]))
    assert err <= 5e-14, err


def test_signed_or_nonfinite_series_is_rejected(lib):
    """Mixed signs (no relative bound) or NaN/inf entries: the plan keeps the exact path."""
    rng = np.random.default_rng(6)
    col = rng.standard_normal(1200)
    err, _ = check(lib, np.ascontiguousarray(col[None, :]))
    assert not err <= 5e-14
    col = np.abs(col)
    col[7] = np.nan
    err, _ = check(lib, np.ascontiguousarray(col[None, :]))
    assert not err <= 5e-14
