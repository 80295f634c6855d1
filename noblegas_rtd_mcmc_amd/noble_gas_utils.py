"""Drop-in for the reference's ``utils/noble_gas_utils.py`` CE model, evaluated on the GPU.

Same names, arguments and return shapes as the reference:

    ng = noble_gas_fun(gases=['Ne','Ar','Kr','Xe'], E=E, T=T, Ae=Ae, F=F, P='lapse_rate')
    ng.ce_exc(add_eq_conc=True)   # -> {'Ne': ..., 'Ar': ..., ...}

Every compute method goes through ``ngrtd_ce_forward`` (include/ngrtd.h).  Scalars give
floats like the reference; numpy arrays for E/T/Ae/F (and P/S) are evaluated element-wise
in ONE device launch and give arrays -- the batched form the reference's posterior-
predictive loops (ng_interp/noble_gas_mcmc.py:648-653) need.
"""
import ctypes as C

import numpy as np

from . import _lib
from .spec import J_flux  # noqa: F401  (re-exported: utils/noble_gas_utils.py:335-348)

# utils/noble_gas_utils.py:38-73 (Porcelli et al. 2002 dry-air mixing ratios)
atm_std = {'N2': 0.781, 'O2': 0.209, 'Ar': 9.34e-3, 'CO2': 3.7e-4, 'Ne': 1.818e-5, 'He': 5.24e-6,
           'CH4': 1.5e-6, 'Kr': 1.14e-6, 'H2': 7e-7, 'N2O': 3e-7, 'CO': 1e-7, 'Xe': 8.7e-8, 'Rn': 6e-20,
           'He3': 5.24e-6 * 0.000140 / 100, 'He4': 5.24e-6,
           'Ne20': 1.818e-5 * 90.50 / 100, 'Ne21': 1.818e-5 * 0.268 / 100, 'Ne22': 1.818e-5 * 9.23 / 100,
           'Ar36': 9.34e-3 * 0.3364 / 100, 'Ar38': 9.34e-3 * 0.0632 / 100, 'Ar40': 9.34e-3 * 99.60 / 100,
           'Kr78': 1.14e-6 * 0.3469 / 100, 'Kr80': 1.14e-6 * 2.2571 / 100, 'Kr82': 1.14e-6 * 11.523 / 100,
           'Kr83': 1.14e-6 * 11.477 / 100, 'Kr84': 1.14e-6 * 57.00 / 100, 'Kr86': 1.14e-6 * 17.398 / 100,
           'Xe124': 8.7e-8 * 0.0951 / 100, 'Xe126': 8.7e-8 * 0.0887 / 100, 'Xe128': 8.7e-8 * 1.919 / 100,
           'Xe129': 8.7e-8 * 26.44 / 100, 'Xe130': 8.7e-8 * 4.070 / 100, 'Xe131': 8.7e-8 * 21.22 / 100,
           'Xe132': 8.7e-8 * 26.89 / 100, 'Xe134': 8.7e-8 * 10.430 / 100, 'Xe136': 8.7e-8 * 8.857 / 100}

_GAS_ID = {"He": 0, "Ne": 1, "Ar": 2, "Kr": 3, "Xe": 4}


def _ce_call(what, p_mode, E, T, Ae, F, P, S, gases, device=0):
    """One ngrtd_ce_forward launch over broadcast arrays; returns ([n][G] or [n], shape)."""
    arrs = np.broadcast_arrays(*[np.asarray(x if x is not None else 0.0, dtype=np.float64)
                                 for x in (E, T, Ae, F, P, S)])
    shape = arrs[0].shape
    flat = [np.ascontiguousarray(a.ravel()) for a in arrs]
    n = flat[0].size
    ctx = _lib.Context.get(device)
    scalar = what in ("vapor_pressure", "pressure")
    ids = (C.c_int32 * max(1, len(gases)))(*[_GAS_ID[g[0:2]] for g in gases] or [0])
    out = np.empty(n if scalar else (n, len(gases)))
    ptr = [a.ctypes.data_as(C.c_void_p) for a in flat]
    if P is None:
        ptr[4] = None
    if S is None:
        ptr[5] = None
    ctx.check(ctx.lib.ngrtd_ce_forward(ctx.h, _lib.CE_WHAT[what], p_mode, *ptr, n, ids, len(gases),
                                       out.ctypes.data_as(C.c_void_p), _lib.MEM_HOST), "ngrtd_ce_forward")
    return out, shape


def _unwrap(v, shape):
    return float(v.reshape(-1)[0]) if shape == () else v.reshape(shape)


class noble_gas_fun:
    """utils/noble_gas_utils.py:75-261 on the GPU (same constructor and methods)."""

    def __init__(self, gases, E, T, Ae, F, P, S=0.0):
        self.gases = gases
        self.E = E
        self.T = T
        self.Ae = Ae
        self.F = F
        self.S = S
        self.P = self.parse_P(P)
        self.obs_dict = None
        self.err_dict = None

    def parse_P(self, P):
        """:91-100 -- '1atm', 'lapse_rate' or a pressure in GPa."""
        if isinstance(P, str) and P == '1atm':
            return 0.000101325
        elif isinstance(P, str) and P == 'lapse_rate':
            return self.lapse_rate()
        else:
            return P

    def _p_mode(self):
        return _lib.P_MODE["given"]

    def lapse_rate(self):
        """:103-113 -- pressure [GPa] at elevation self.E."""
        v, shape = _ce_call("pressure", _lib.P_MODE["lapse_rate"], self.E, 0.0, 0.0, 0.0, None, None, [])
        return _unwrap(v, shape)

    def solubility(self, gas):
        """:117-180 -- Henry coefficient [GPa]."""
        v, shape = _ce_call("solubility", _lib.P_MODE["1atm"], self.E, self.T, self.Ae, self.F, None, self.S, [gas])
        return _unwrap(v[:, 0], shape)

    def vapor_pressure(self):
        """:184-199 -- Antoine vapour pressure [GPa]."""
        v, shape = _ce_call("vapor_pressure", _lib.P_MODE["1atm"], self.E, self.T, 0.0, 0.0, None, None, [])
        return _unwrap(v, shape)

    def _gas_dict(self, what):
        v, shape = _ce_call(what, self._p_mode(), self.E, self.T, self.Ae, self.F, self.P, self.S, list(self.gases))
        return {g: _unwrap(v[:, j], shape) for j, g in enumerate(self.gases)}

    def equil_conc(self):
        """:202-213 -- atmospheric equilibrium concentration [ccSTP/g] (wet pressure)."""
        return self._gas_dict("equil")

    def equil_conc_dry(self):
        """:216-232 -- equilibrium concentration with the dry pressure; T < 0 -> -9999."""
        return self._gas_dict("equil_dry")

    def ce_exc(self, add_eq_conc):
        """:235-253 -- closed-system excess air (+ equilibrium when add_eq_conc)."""
        return self._gas_dict("ce_total" if add_eq_conc else "ce_excess")

    def update_pars(self, T, Ae, F, E):
        """:256-261."""
        self.T = T
        self.Ae = Ae
        self.F = F
        self.E = E
        self.P = self.lapse_rate()


def find_T_lapse(E_lapse, E_lapse_int, lapse_slope):
    """:304-317 -- temperature from elevation on a lapse rate."""
    return (E_lapse - E_lapse_int) / lapse_slope


def F_w(C_i, T, S, E, Ae, F):
    """:266-297 -- fractionation factors relative to Ar (equilibrium from the GPU model)."""
    gases = list(C_i.keys())
    ng_ = noble_gas_fun(gases=gases, E=E, T=T, Ae=Ae, F=F, P='lapse_rate')
    C_i_atm = ng_.equil_conc()
    R_atm = {g: C_i_atm[g] / C_i_atm['Ar'] for g in C_i_atm}
    R_smp = {g: C_i[g] / C_i['Ar'] for g in C_i}
    return {'F_' + g: R_smp[g] / R_atm[g] for g in R_atm}


def _he_comps_call(He4, He3, Ae, F, E, T, Rterr, device=0):
    """One ngrtd_he_comps launch over broadcast arrays -> ([5][n] SoA, shape)."""
    arrs = np.broadcast_arrays(*[np.asarray(x, dtype=np.float64) for x in (He4, He3, Ae, F, E, T, Rterr)])
    shape = arrs[0].shape
    flat = [np.ascontiguousarray(a.ravel()) for a in arrs]
    n = flat[0].size
    ctx = _lib.Context.get(device)
    out = np.empty((len(_lib.HE_OUT), n))
    ptr = [a.ctypes.data_as(C.c_void_p) for a in flat]
    ctx.check(ctx.lib.ngrtd_he_comps(ctx.h, *ptr, 0.0, n, out.ctypes.data_as(C.c_void_p), _lib.MEM_HOST),
              "ngrtd_he_comps")
    return out, shape


class ng_parse:
    """utils/noble_gas_utils.py:380-444 on the GPU.  obs_dict holds one well's
    observations (keys He4, He3, ...); Ae, F, E, T (and the obs values) may be numpy arrays
    of ensemble members, evaluated in one launch (age_modeling_mcmc.prep.py:356-382 loops
    over them one object at a time)."""

    def __init__(self, obs_dict, Ae, F, E, T):
        self.obs_dict = obs_dict
        self.Ae = Ae
        self.F = F
        self.E = E
        self.T = T
        self.obs_dict_ = obs_dict.copy()

    def He_comps(self, Rterr):
        """:394-422 -- adds He4_eq, He4_atm, He4_ter, He4_del, He3_tu to obs_dict_."""
        v, shape = _he_comps_call(self.obs_dict['He4'], self.obs_dict['He3'], self.Ae, self.F, self.E, self.T,
                                  Rterr)
        for k, name in enumerate(_lib.HE_OUT):
            self.obs_dict_[name] = _unwrap(v[k], shape)

    def Ne_del(self):
        """:425-432 -- delta Ne [%] against the wet equilibrium.  (The reference body calls
        ``ng.noble_gas_fun``, a name its module never defines, so it raises NameError there;
        this is the computation it spells out.)"""
        Ne_obs = self.obs_dict_['Ne']
        ng_ = noble_gas_fun(gases=['Ne'], E=self.E, T=self.T, Ae=self.Ae, F=self.F, P='lapse_rate')
        Ne_atm = ng_.equil_conc()['Ne']
        self.obs_dict_['Ne_del'] = (Ne_obs / Ne_atm - 1) * 100
