"""GPU tests of the prep-stage ensemble propagation: the drop-in
``noble_gas_utils.ng_parse`` and ``cfc_utils.cfc_ce_corr / sf6_ce_corr`` against the
golden vectors of the reference's own classes (tests/golden/make_golden.py make_prep),
batched over the ensemble and as scalar calls, plus the device-pointer C-ABI path.

Tolerance: rtol 1e-12; He4_ter / He4_del / He3_tu are differences of
nearly equal terms, so their tolerance is rtol 1e-12 of the cancelling operands."""
import ctypes as C

import numpy as np
import pytest

from test_oracle_golden import he_scales

pytestmark = pytest.mark.gpu
RTOL = 1e-12


def close(a, b, rtol=RTOL, atol=0.0):
    a, b = np.asarray(a), np.asarray(b)
    ok = (np.isnan(a) & np.isnan(b)) | (np.isinf(a) & np.isinf(b) & (np.sign(a) == np.sign(b)))
    return ok | (np.abs(a - b) <= atol + rtol * np.abs(b))


def test_ng_parse_he_comps_batched_and_scalar(golden):
    from noblegas_rtd_mcmc_amd import noble_gas_utils as ng
    z = golden("prep_golden.npz")
    scale = he_scales(z)
    ngp = ng.ng_parse({"He4": z["He4"], "He3": z["He3"], "Ne": 1.0}, z["Ae"], z["F"], z["E"], z["T"])
    ngp.He_comps(z["Rterr"])
    names = ["He4_eq", "He4_atm", "He4_ter", "He4_del", "He3_tu"]
    for k, name in enumerate(names):
        assert close(ngp.obs_dict_[name], z["he"][k], atol=RTOL * scale[k]).all(), name
    assert ngp.obs_dict_["Ne"] == 1.0 and "He4_ter" not in ngp.obs_dict     # obs_dict untouched
    for i in (0, 1, 2, 3, 700):                                               # scalar: floats
        p = ng.ng_parse({"He4": float(z["He4"][i]), "He3": float(z["He3"][i])}, float(z["Ae"][i]),
                        float(z["F"][i]), float(z["E"][i]), float(z["T"][i]))
        p.He_comps(float(z["Rterr"][i]))
        assert all(isinstance(p.obs_dict_[n], float) for n in names)
        assert close([p.obs_dict_[n] for n in names], z["he"][:, i], atol=RTOL * scale[:, i]).all()
    # constant Rterr broadcast (prep.py:341 Rterr_c)
    c = ng.ng_parse({"He4": z["He4"], "He3": z["He3"]}, z["Ae"], z["F"], z["E"], z["T"])
    c.He_comps(2.0e-8)
    from oracle import prep as oprep
    ref = oprep.he_comps(z["He4"], z["He3"], z["Ae"], z["F"], z["E"], z["T"], 2.0e-8)
    assert close(c.obs_dict_["He3_tu"], ref["He3_tu"], atol=RTOL * scale[4]).all()


def test_cfc_ce_corr_batched_matches_reference(golden):
    from noblegas_rtd_mcmc_amd import cfc_utils
    z = golden("prep_golden.npz")
    E, T, Ae, F, S = z["E"], z["T"], z["Ae"], z["F"], z["S"]
    c = cfc_utils.cfc_ce_corr(cfc_num=[11, 12, 113], E=E, T=T, Ae=Ae, F=F, S=S)
    with pytest.raises(TypeError):
        c.ce_exc_conc_cfc(z["z_in"].T)          # self.P is None until lapse_rate_atm, as the reference
    assert close(c.equil_air_conc_cfc(z["cmeas"].T), z["cfc_air"].T).all()
    assert close(c.P, z["p_atm"]).all()
    assert close(c.equil_aq_conc_cfc(z["z_in"].T), z["cfc_aq"].T).all()
    assert close(c.ce_exc_conc_cfc(z["z_in"].T), z["cfc_exc"].T).all()
    assert close(c.solubility_cfc(), z["cfc_sol"].T).all()
    assert close(c.vapor_pressure_atm(), z["pv_atm"]).all()
    assert close(c.lapse_rate_atm(), z["p_atm"]).all()


def test_sf6_ce_corr_batched_matches_reference(golden):
    from noblegas_rtd_mcmc_amd import cfc_utils
    z = golden("prep_golden.npz")
    s = cfc_utils.sf6_ce_corr(E=z["E"], T=z["T"], Ae=z["Ae"], F=z["F"], S=z["S"])
    assert close(s.equil_air_conc_sf6(z["sf6_meas"]), z["sf6_air"]).all()
    assert close(s.equil_aq_conc_sf6(z["sf6_z"]), z["sf6_aq"]).all()
    assert close(s.ce_exc_conc_sf6(z["sf6_z"]), z["sf6_exc"]).all()
    assert close(s.solubility_sf6(), z["sf6_sol"]).all()


def test_cfc_scalar_calls_like_reference(golden):
    from noblegas_rtd_mcmc_amd import cfc_utils
    z = golden("prep_golden.npz")
    for i in (0, 2, 5, 1100):
        c = cfc_utils.cfc_ce_corr(cfc_num=[11, 12, 113], E=float(z["E"][i]), T=float(z["T"][i]),
                                  Ae=float(z["Ae"][i]), F=float(z["F"][i]), S=float(z["S"][i]))
        r = c.equil_air_conc_cfc(z["cmeas"][:, i].copy())
        assert r.shape == (3,) and close(r, z["cfc_air"][:, i]).all()
        assert isinstance(c.P, float)
        s = cfc_utils.sf6_ce_corr(E=float(z["E"][i]), T=float(z["T"][i]), Ae=float(z["Ae"][i]),
                                  F=float(z["F"][i]), S=float(z["S"][i]))
        v = s.equil_air_conc_sf6(float(z["sf6_meas"][i]))
        assert isinstance(v, float) and close(v, z["sf6_air"][i])
    # one CFC only, and update_pars (cfc_utils.py:144-150)
    c = cfc_utils.cfc_ce_corr(cfc_num=[12], E=2900., T=5., Ae=0.01, F=0.5)
    c.update_pars(T=float(z["T"][7]), E=float(z["E"][7]), Ae=float(z["Ae"][7]), F=float(z["F"][7]))
    c.S = float(z["S"][7])
    assert close(c.ce_exc_conc_cfc(np.array([z["z_in"][1, 7]])), [z["cfc_exc"][1, 7]]).all()


def test_prep_device_pointers_and_errors(golden):
    """ngrtd_he_comps / ngrtd_cfc_corr on device memory (mem=NGRTD_MEM_DEVICE), and the
    argument checks (status < 0, message set)."""
    import torch
    from noblegas_rtd_mcmc_amd import _lib
    z = golden("prep_golden.npz")
    ctx = _lib.Context.get(0)
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    n = z["E"].size
    d = {k: torch.from_numpy(np.ascontiguousarray(z[k])).cuda() for k in ("He4", "He3", "Ae", "F", "E", "T", "Rterr")}
    out = torch.empty(5, n, dtype=torch.float64, device="cuda")
    p = lambda t: C.c_void_p(t.data_ptr())
    ctx.check(ctx.lib.ngrtd_he_comps(ctx.h, *[p(d[k]) for k in ("He4", "He3", "Ae", "F", "E", "T", "Rterr")],
                                     0.0, n, p(out), _lib.MEM_DEVICE), "he_comps")
    torch.cuda.synchronize()
    scale = he_scales(z)
    assert close(out.cpu().numpy(), z["he"], atol=RTOL * scale).all()
    # errors: missing inputs, bad species, ce_exc without P
    st = ctx.lib.ngrtd_he_comps(ctx.h, None, None, None, None, None, None, None, 0.0, 4, p(out), _lib.MEM_DEVICE)
    assert st == _lib.NGRTD_EINVAL
    ids = (C.c_int32 * 1)(7)
    x = torch.ones(n, dtype=torch.float64, device="cuda")
    st = ctx.lib.ngrtd_cfc_corr(ctx.h, 0, ids, 1, p(d["E"]), p(d["T"]), p(d["Ae"]), p(d["F"]), None, None, p(x), n,
                                p(out), _lib.MEM_DEVICE)
    assert st == _lib.NGRTD_EINVAL and b"species" in ctx.lib.ngrtd_last_error(ctx.h)
    ids = (C.c_int32 * 1)(3)
    st = ctx.lib.ngrtd_cfc_corr(ctx.h, 2, ids, 1, p(d["E"]), p(d["T"]), p(d["Ae"]), p(d["F"]), None, None, p(x), n,
                                p(out), _lib.MEM_DEVICE)
    assert st == _lib.NGRTD_EINVAL
    assert ctx.lib.ngrtd_he_comps(ctx.h, *[None] * 7, 0.0, 0, p(out), _lib.MEM_DEVICE) == _lib.NGRTD_EINVAL
