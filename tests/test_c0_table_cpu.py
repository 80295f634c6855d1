"""The Student-t normaliser table (host-only part of libngrtd: ngrtd_c0_check, no GPU).

Every Student-t block of the log-prob (StudentT.logp behind run_age_mcmc_utils.py:390/396
and noble_gas_mcmc.py:266) needs c0(nu) = lgamma((nu+1)/2) - lgamma(nu/2) - log(pi nu)/2.
Plans replace it with a piecewise polynomial over the octaves of the nu priors' supports
(ngrtd_math.hpp c0_piece / c0_poly).  These tests evaluate the returned coefficients
independently (NumPy Horner, scipy gammaln) over the shipped prior ranges and wider ones,
and check that degenerate ranges get no table (the plan then keeps the exact form).
"""
import ctypes as C

import numpy as np
import pytest
from scipy.special import gammaln

N, SUB, MAXP = 12, 4, 64


@pytest.fixture(scope="module")
def lib():
    import __graft_entry__ as g
    g.build()
    from noblegas_rtd_mcmc_amd import _lib
    return _lib.load()


def build(lib, lo, hi):
    coef = np.zeros(MAXP * N)
    e0, npc, err = C.c_int32(), C.c_int32(), C.c_double()
    assert lib.ngrtd_c0_check(lo, hi, coef.ctypes.data_as(C.POINTER(C.c_double)), C.byref(e0), C.byref(npc),
                              C.byref(err)) == 0
    return e0.value, npc.value, err.value, coef[: npc.value * N].reshape(-1, N)


def table_c0(e0, coef, nu):
    m, e = np.frexp(nu)                        # nu = m 2^e, m in [1/2, 1)
    m, e = 2 * m, e - 1
    j = np.floor((m - 1) * 4).astype(int)
    p = (e - e0) * SUB + j
    x = (m - (1.125 + 0.25 * j)) * 8.0
    return np.array([np.polynomial.polynomial.polyval(xi, coef[pi]) for xi, pi in zip(x, p)])


def exact_c0(nu):
    return gammaln((nu + 1) / 2) - gammaln(nu / 2) - 0.5 * np.log(np.pi * nu)


@pytest.mark.parametrize("lo,hi", [(1.0, 30.0), (1.0, 50.0), (0.1, 100.0), (2.0, 2.0), (3.7, 1.0e4)])
def test_table_matches_lgamma(lib, lo, hi):
    e0, npc, err, coef = build(lib, lo, hi)
    assert err <= 2e-14, err
    assert npc % SUB == 0 and npc <= MAXP
    assert 2.0 ** e0 <= lo < 2.0 ** (e0 + 1)
    assert hi < 2.0 ** (e0 + npc // SUB)
    rng = np.random.default_rng(11)
    nu = np.concatenate([np.geomspace(lo, hi, 200), rng.uniform(lo, hi, 200), [lo, hi]])
    got = table_c0(e0, coef, nu)
    ref = exact_c0(nu)
    # scipy's float64 gammaln difference carries a few ulp of each |lgamma| itself
    tol = 4e-15 + 1e-15 * (np.abs(gammaln((nu + 1) / 2)) + np.abs(gammaln(nu / 2)))
    assert np.all(np.abs(got - ref) <= tol), np.max(np.abs(got - ref) - tol)


def test_nu_one_is_minus_log_pi(lib):
    e0, npc, err, coef = build(lib, 1.0, 30.0)
    assert e0 == 0 and npc == 5 * SUB
    assert abs(table_c0(e0, coef, np.array([1.0]))[0] + np.log(np.pi)) <= 1e-15


@pytest.mark.parametrize("lo,hi", [(0.0, 30.0), (-1.0, 5.0), (np.nan, 5.0), (1.0, np.inf), (5.0, 1.0),
                                   (1e-3, 1e20)])
def test_degenerate_ranges_get_no_table(lib, lo, hi):
    _, npc, err, _ = build(lib, lo, hi)
    assert npc == 0 or not err <= 2e-14
    assert not err <= 2e-14
