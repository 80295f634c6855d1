"""The exp_pist_flow channel-table window (host-only part of libngrtd: ngrtd_epm_window_check,
no GPU).  A plan with tau1 ~ U(., tau_hi), eta1 ~ U(., eta_hi) stages only the table rows its
in-support units read (ngrtd.hip epm_window): a unit's head block [B - 16, B), B =
(m // 16 + 1) 16 past its first unmasked age m, plus 64 rows of the exact short tail.  The
bound must hold for the reference's mask itself, tp >= tau*(1-(1/eta)) in float64
(convolution_integral_utils.py:189), evaluated here with NumPy at the support's worst corner
and on a dense grid near it, for the published priors and random ones."""
import ctypes as C

import numpy as np
import pytest


@pytest.fixture(scope="module")
def lib():
    import __graft_entry__ as g
    g.build()
    from noblegas_rtd_mcmc_amd import _lib
    return _lib.load()


def rows_of(lib, tau_hi, eta_hi, dtp, N):
    r = C.c_int32()
    assert lib.ngrtd_epm_window_check(tau_hi, eta_hi, dtp, N, C.byref(r)) == 0
    return r.value


def first_unmasked(tau, eta, dtp, N):
    """The reference's mask (:169-174 grid, :189 mask) -> first unmasked index (N if none)."""
    tp = np.arange(0, N).astype(float)
    tp[0] += 1e-5
    tp += dtp
    with np.errstate(all="ignore"):
        mask = tp >= np.float64(tau) * (1 - (1 / np.float64(eta)))
    idx = np.nonzero(mask)[0]
    return int(idx[0]) if idx.size else N


def needed_rows(m):
    m = max(m, 1)
    B = (m // 16 + 1) * 16
    return B + 64                       # the head block's end + the exact short tail


@pytest.mark.parametrize("tau_hi,eta_hi,dtp,N", [(1000.0, 5.0, 0.0, 25256), (500.0, 5.0, 0.0, 25256),
                                                 (1000.0, 5.0, 0.0, 1200), (15000.0, 5.0, 0.0, 25256),
                                                 (1000.0, 1.0, 0.0, 25256), (1000.0, 5.0, 3.0, 25256),
                                                 (999.9, 4.9, 0.0, 25256)])
def test_window_covers_every_in_support_unit(lib, tau_hi, eta_hi, dtp, N):
    rows = rows_of(lib, tau_hi, eta_hi, dtp, N)
    assert rows % 16 == 0 and rows > 0
    worst = first_unmasked(tau_hi, eta_hi, dtp, N)
    assert needed_rows(worst) <= rows, (worst, rows)
    # the threshold tau (1 - 1/eta) grows with both: the corner is the worst unit; a dense grid
    # near it (and a random sample of the box) never needs more
    rng = np.random.default_rng(5)
    taus = np.concatenate([tau_hi - np.linspace(0, 1e-6 * tau_hi, 7), rng.uniform(1.0, tau_hi, 200)])
    etas = np.concatenate([eta_hi - np.linspace(0, 1e-9, 5), rng.uniform(1.0, eta_hi, 40)])
    for t in taus[::3]:
        for e in etas[::2]:
            assert needed_rows(first_unmasked(t, e, dtp, N)) <= rows
    # a window is not larger than needed by more than a block and the tail margin
    assert rows <= needed_rows(worst) + 32


def test_no_window_when_the_priors_do_not_bound_the_mask(lib):
    """No window: the threshold past the series (every age of a far unit masked), a
    non-finite or degenerate bound -> -1 (the plan keeps the whole table)."""
    assert rows_of(lib, 40000.0, 5.0, 0.0, 25256) == -1
    assert rows_of(lib, np.inf, 5.0, 0.0, 25256) == -1
    assert rows_of(lib, np.nan, 5.0, 0.0, 25256) == -1
    assert rows_of(lib, 1000.0, 0.5, 0.0, 25256) == -1
    assert rows_of(lib, 1000.0, np.nan, 0.0, 25256) == -1
