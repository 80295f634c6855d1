"""GPU tests of the fracture / matrix-diffusion RTD 'frac_inf_diff' 
through the drop-in tracer_conv_integral (ngrtd_frac_conv) against the golden vectors of
the reference's own class (tests/golden/make_golden.py make_frac).

Tolerance (written here): rtol 1e-12 on concentrations and FM_mu (the
SURVEY.md §8d bar), and on the weights g rtol 1e-11 + atol 1e-13 * max(g).  The reference's
own inner grid is libm-defined (tadv = 10**linspace(...) and t_ret**1.5 go through pow(),
whose last-ulp rounding differs between glibc, SVML and numba), so the bar leaves room for
that; measured on MI355X: <= 7e-16 on concentrations, 6e-15 of max(g) on weights."""
import ctypes as C

import numpy as np
import pandas as pd
import pytest

pytestmark = pytest.mark.gpu

TRACERS = {"CFC12": ("CFC12", False, False, False), "SF6": ("SF6", False, False, False),
           "H3": ("H3", 12.34, False, False), "He3": ("H3", 12.34, "3He", False),
           "He4_ter": ("He4_ter", False, "4He", 3.30885e-11)}
RT_C, RT_G, AT_G = 1e-12, 1e-11, 1e-13


def frame(sname, n, col):
    from noblegas_rtd_mcmc_amd.workloads import atmos_series
    s = atmos_series(sname, n)
    c = s.c_by_age[:n] * (0.0 if col == "He4_ter" else 1.0)
    return pd.DataFrame({col: np.flip(c)}, index=np.arange(n - 1, -1, -1))


def rel(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return np.max(np.abs(a - b) / np.maximum(np.abs(b), 1e-300))


def g_ok(g, ref):
    return np.all(np.abs(g - ref) <= RT_G * np.abs(ref) + AT_G * np.abs(ref).max(axis=-1, keepdims=True))


@pytest.mark.parametrize("n", [300, 1200])
def test_frac_batched_all_tracers(golden, n):
    from noblegas_rtd_mcmc_amd.convolution_integral_utils import tracer_conv_integral
    z = golden("frac_golden.npz")
    for tname, (sname, t_half, accum, J) in TRACERS.items():
        df = frame(sname, n, tname)
        cm = tracer_conv_integral(df, df.index[-1])
        cm.update_pars(tau=z["tau"], mod_type="frac_inf_diff", t_half=t_half, rad_accum=accum, J=J, D=z["D"],
                       bbar=z["bbar"], Phi_im=z["Phi"])
        got = cm.convolve()
        print(tname, n, "conc max rel err %.2e" % rel(got, z["conc_%s_%d" % (tname, n)]))
        assert got.shape == z["tau"].shape
        assert rel(got, z["conc_%s_%d" % (tname, n)]) <= RT_C, tname
        assert rel(cm.FM_mu, z["fm_%d" % n]) <= RT_C
    df = frame("CFC12", n, "CFC12")
    cm = tracer_conv_integral(df, df.index[-1])
    cm.update_pars(tau=z["tau"], mod_type="frac_inf_diff", D=z["D"], bbar=z["bbar"], Phi_im=z["Phi"])
    g = cm.gen_g_tp()
    assert g.shape == (z["tau"].size, n)
    print("g max abs err / max g %.2e" % np.max(np.abs(g - z["g_%d" % n]) / z["g_%d" % n].max(axis=1, keepdims=True)))
    assert g_ok(g, z["g_%d" % n])
    assert np.allclose(g.sum(axis=1), 1.0, rtol=1e-13)


def test_frac_scalar_call_and_mint(golden, capsys):
    from noblegas_rtd_mcmc_amd.convolution_integral_utils import tracer_conv_integral
    z = golden("frac_golden.npz")
    df = frame("H3", 300, "H3")
    cm = tracer_conv_integral(df, df.index[-1])
    cm.update_pars(tau=float(z["tau"][3]), mod_type="frac_inf_diff", t_half=12.34, D=float(z["D"][3]),
                   bbar=float(z["bbar"][3]), Phi_im=float(z["Phi"][3]))
    v = cm.convolve()
    assert isinstance(v, float) and isinstance(cm.FM_mu, float)
    assert rel(v, z["conc_H3_300"][3]) <= RT_C
    g = cm.gen_g_tp()
    assert g.shape == (300,) and len(cm.tau_list) == 300
    cm.update_pars(tau=float(z["tau"][3]), mod_type="frac_inf_diff.mint", D=float(z["D"][3]),
                   bbar=float(z["bbar"][3]), Phi_im=float(z["Phi"][3]))
    cm.gen_g_tp()
    assert "mean travel time is %3.2f" % z["fm_300"][3] in capsys.readouterr().out


def test_frac_external_advective_rtd(golden):
    """frac_rtd_numba (:67-97): np.interp of f_tadv_ext on the age grid, per-set rows and one
    shared row."""
    from noblegas_rtd_mcmc_amd.convolution_integral_utils import tracer_conv_integral
    z = golden("frac_golden.npz")
    ke = z["ext"].shape[0]
    df = frame("H3", 600, "H3")
    cm = tracer_conv_integral(df, df.index[-1])
    cm.update_pars(tau=z["tau"][:ke], mod_type="frac_inf_diff", t_half=12.34, bbar=z["bbar"][:ke],
                   Phi_im=z["Phi"][:ke], f_tadv_ext=z["ext"])
    got = cm.convolve()
    print("ext conc max rel err %.2e" % rel(got, z["ext_conc"]))
    assert rel(got, z["ext_conc"]) <= RT_C and rel(cm.FM_mu, z["ext_fm"]) <= RT_C
    # one shared row (stride 0) broadcast against per-set bbar / Phi_im
    cm.update_pars(mod_type="frac_inf_diff", t_half=12.34, bbar=z["bbar"][:ke], Phi_im=z["Phi"][:ke],
                   f_tadv_ext=z["ext"][2])
    got = cm.convolve()
    assert rel(got[2], z["ext_conc"][2]) <= RT_C
    with pytest.raises(ValueError):
        cm.update_pars(mod_type="frac_inf_diff", bbar=1e-3, Phi_im=0.01, f_tadv_ext=np.ones(10))
        cm.convolve()


def test_frac_long_series(golden):
    """N = 25256 (the shipped C_in_dict length): 25.3 M inner grid points in one call."""
    from noblegas_rtd_mcmc_amd.convolution_integral_utils import tracer_conv_integral
    z = golden("frac_golden.npz")
    df = frame("CFC12", 25256, "CFC12")
    cm = tracer_conv_integral(df, df.index[-1])
    cm.update_pars(tau=1500.0, mod_type="frac_inf_diff", D=0.5, bbar=3e-4, Phi_im=0.02)
    v = cm.convolve()
    print("long conc rel err %.2e fm %.2e" % (rel(v, z["long_conc"]), rel(cm.FM_mu, z["long_fm"])))
    assert rel(v, z["long_conc"]) <= RT_C and rel(cm.FM_mu, z["long_fm"]) <= RT_C
    g = cm.gen_g_tp()
    assert g_ok(g[:2000], z["long_g_head"])


def test_frac_device_pointers(golden):
    """ngrtd_frac_conv on device memory: conc, g and FM_mu straight into torch tensors;
    results identical to the host-staged call; argument errors."""
    import torch
    from noblegas_rtd_mcmc_amd import _lib
    from noblegas_rtd_mcmc_amd.convolution_integral_utils import _series_arrays, _series_id
    z = golden("frac_golden.npz")
    ctx = _lib.Context.get(0)
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    df = frame("CFC12", 300, "CFC12")
    v, i = _series_arrays(df, False)
    sid, n = _series_id(ctx, v, i, df.index[-1])
    k = z["tau"].size
    d = {key: torch.from_numpy(np.ascontiguousarray(z[key])).cuda() for key in ("tau", "D", "bbar", "Phi")}
    conc = torch.empty(k, dtype=torch.float64, device="cuda")
    fm = torch.empty(k, dtype=torch.float64, device="cuda")
    g = torch.empty(k, n, dtype=torch.float64, device="cuda")
    p = lambda t: C.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
    ctx.check(ctx.lib.ngrtd_frac_conv(ctx.h, sid, 0, p(d["tau"]), p(d["D"]), p(d["bbar"]), p(d["Phi"]), None, 0,
                                      None, 0.0, None, 0.0, k, p(conc), p(g), p(fm), _lib.MEM_DEVICE), "frac")
    torch.cuda.synchronize()
    assert rel(conc.cpu().numpy(), z["conc_CFC12_300"]) <= RT_C
    assert g_ok(g.cpu().numpy(), z["g_300"])
    host = np.empty(k)
    keep = [np.ascontiguousarray(z[key]) for key in ("tau", "D", "bbar", "Phi")]   # alive across the call
    ctx.check(ctx.lib.ngrtd_frac_conv(ctx.h, sid, 0, *[C.c_void_p(a.ctypes.data) for a in keep],
                                      None, 0, None, 0.0, None, 0.0, k, C.c_void_p(host.ctypes.data), None, None,
                                      _lib.MEM_HOST), "frac host")
    assert np.array_equal(host, conc.cpu().numpy())       # deterministic: fixed-order reductions
    st = ctx.lib.ngrtd_frac_conv(ctx.h, sid, 0, p(d["tau"]), p(d["D"]), None, p(d["Phi"]), None, 0, None, 0.0,
                                 None, 0.0, k, p(conc), None, None, _lib.MEM_DEVICE)
    assert st == _lib.NGRTD_EINVAL
    st = ctx.lib.ngrtd_frac_conv(ctx.h, sid, 0, p(d["tau"]), p(d["D"]), p(d["bbar"]), p(d["Phi"]), None, 0, None,
                                 0.0, None, 0.0, k, None, None, None, _lib.MEM_DEVICE)
    assert st == _lib.NGRTD_EINVAL


@pytest.mark.parametrize("key,n,tsh", [("shift", 300, 3.7), ("n2", 2, 0.0)])
def test_frac_shifted_sampling_date_and_shortest_series(golden, key, n, tsh):
    """t_samp past the last index (dtp = floor(t_samp - index[-1]) = 3, :172-173) and N = 2."""
    from noblegas_rtd_mcmc_amd.convolution_integral_utils import tracer_conv_integral
    z = golden("frac_golden.npz")
    df = frame("H3", n, "H3")
    cm = tracer_conv_integral(df, df.index[-1] + tsh)
    cm.update_pars(tau=z["tau"][:4], mod_type="frac_inf_diff", t_half=12.34, D=z["D"][:4], bbar=z["bbar"][:4],
                   Phi_im=z["Phi"][:4])
    got = cm.convolve()
    assert rel(got, z[key + "_conc"]) <= RT_C and rel(cm.FM_mu, z[key + "_fm"]) <= RT_C
