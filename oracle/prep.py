"""NumPy restatement of the prep-stage ensemble propagation.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  Elementwise over ensemble members,
same association order as the reference:

* ``he_comps``  -- ng_parse.He_comps, utils/noble_gas_utils.py:394-422 (4He/3He mass
                   balance on the CE model with P='lapse_rate', S=0)
* ``cfc_*``     -- cfc_ce_corr / sf6_ce_corr, utils/cfc_utils.py:25-306
"""
import numpy as np

from . import ce as oce

HE_OUT = ("He4_eq", "He4_atm", "He4_ter", "He4_del", "He3_tu")

# utils/cfc_utils.py:74 (cfc_dict) and :214-219 (solubility_sf6)
CFC_COEF = {11: (-136.2685, 206.1150, 57.2805, -.148598, 0.095114, -0.0163396),
            12: (-124.4395, 185.4299, 51.6383, -0.149779, 0.094668, -0.0160043),
            113: (-136.129, 206.475, 55.8957, -0.02754, 0.006033, 0,),
            "SF6": (-98.7264000, 142.803, 38.8746, 0.0268696, -0.0334407, 0.0070843)}


def _f(x):
    return np.asarray(x, dtype=np.float64)


def he_comps(He4_obs, He3_obs, Ae, F, E, T, Rterr):
    """noble_gas_utils.py:394-422 -> dict of the obs_dict_ entries it adds."""
    He4_obs, He3_obs, Rterr = _f(He4_obs), _f(He3_obs), _f(Rterr)
    P = oce.lapse_rate(E)                                                  # parse_P('lapse_rate')
    He4_eq = oce.equil_conc(["He"], _f(T), P)["He"]                         # :402
    He4_atm = oce.ce_exc(["He"], E, T, Ae, F, P="lapse_rate", add_eq_conc=True)["He"]   # :404
    with np.errstate(all="ignore"):
        He4_ter = He4_obs - He4_atm                                         # :405
        He4_del = 100 * (He4_ter / He4_atm)                                 # :408
        Ratm = 1.384e-6
        S = 0.0
        CF = 4.021e14 / (1 - S)
        He3_trit = He3_obs - (He4_obs - He4_ter) * Ratm + He4_eq * Ratm * (1 - 0.983) - He4_ter * Rterr
        TU = He3_trit * CF
    return {"He4_eq": He4_eq, "He4_atm": He4_atm, "He4_ter": He4_ter, "He4_del": He4_del, "He3_tu": TU}


def vapor_pressure_atm(T):
    """cfc_utils.py:34-51 (identical in sf6_ce_corr :181-196)."""
    T = _f(T)
    A = np.where(T <= 99.0, 8.07131, 8.14019)
    B = np.where(T <= 99.0, 1730.63, 1810.94)
    C = np.where(T <= 99.0, 233.426, 244.485)
    with np.errstate(all="ignore"):
        P = 10 ** (A - (B / (C + T)))
        P = P / 760. * 101325
        P_vapor = P / 1.0e9
        return P_vapor / 0.000101325


def lapse_rate_atm(E):
    """cfc_utils.py:53-62."""
    with np.errstate(all="ignore"):
        return (1 - .0065 * _f(E) / 288.15) ** 5.2561


def solubility(sp, T, S=0.0):
    """cfc_utils.py:64-84 (CFC) / :208-221 (SF6), elementwise over T."""
    a_1, a_2, a_3, b_1, b_2, b_3 = CFC_COEF[sp]
    T_k = _f(T) + 273.15
    with np.errstate(all="ignore"):
        return np.exp(a_1 + a_2 * (100 / T_k) + a_3 * np.log(T_k / 100)
                      + _f(S) * (b_1 + b_2 * (T_k / 100) + b_3 * (T_k / 100) ** 2))


def equil_air_conc(sp, C_meas, E, T, Ae, F, S=0.0):
    """cfc_utils.py:86-106 / :229-249 (SF6 * 0.001).  Ae in ccSTP/g (x1000, :30)."""
    Ae = _f(Ae) * 1000.
    Ki = solubility(sp, T, S)
    with np.errstate(all="ignore"):
        P_da = lapse_rate_atm(E) - vapor_pressure_atm(T)
        molar_volume = 22414.1
        C_meas, F = _f(C_meas), _f(F)
        z_i = (C_meas + ((C_meas * F * (Ae / molar_volume)) / (Ki * P_da))) / (Ki * P_da + (Ae / molar_volume))
        return z_i * 0.001 if sp == "SF6" else z_i


def equil_aq_conc(sp, z_i, E, T, S=0.0):
    """cfc_utils.py:108-124 / :264-278 (SF6 / 0.001)."""
    Ki = solubility(sp, T, S)
    with np.errstate(all="ignore"):
        P_da = lapse_rate_atm(E) - vapor_pressure_atm(T)
        C = Ki * _f(z_i) * P_da
        return C / 0.001 if sp == "SF6" else C


def ce_exc_conc(sp, z_i, P, T, Ae, F, S=0.0):
    """cfc_utils.py:126-142 / :280-296 (SF6 x 1000); P = self.P [atm]."""
    P_vapor = vapor_pressure_atm(T)
    K = solubility(sp, T, S)
    z_i, F = _f(z_i), _f(F)
    with np.errstate(all="ignore"):
        C_eq = K * z_i * (_f(P) - P_vapor)
        Ae = _f(Ae) * 1000. / 22414 / 1e-12
        if sp == "SF6":
            return 1000 * ((1 - F) * Ae * (z_i * 1e-12)) / (1 + F * Ae * ((z_i * 1e-12 / C_eq)))
        return ((1 - F) * Ae * (z_i * 1e-12)) / (1 + F * Ae * ((z_i * 1e-12 / C_eq)))
