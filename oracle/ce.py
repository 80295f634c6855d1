"""NumPy restatement of the Closed-Equilibrium (CE) noble-gas model.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  Follows utils/noble_gas_utils.py of
the reference operation-for-operation (same association order) so that, evaluated
elementwise on float64 arrays, it reproduces the reference to ~1 ulp per operation.
"""
import numpy as np

# utils/noble_gas_utils.py:38-73 (only the entries the CE path reads)
ATM_STD = {"He": 5.24e-6, "Ne": 1.818e-5, "Ar": 9.34e-3, "Kr": 1.14e-6, "Xe": 8.7e-8}
GASES = ("He", "Ne", "Ar", "Kr", "Xe")

# utils/noble_gas_utils.py:138-142 (Crovetto 1981 solubility coefficients)
SOL = {"He": (-0.00953, 0.107722, 0.001969, -0.043825),
       "Ne": (-7.259, 6.95, -1.3826, 0.0538),
       "Ar": (-9.52, 8.83, -1.8959, 0.0698),
       "Kr": (-6.292, 5.612, -0.8881, -0.0458),
       "Xe": (-3.902, 2.439, 0.3863, -0.221)}
# utils/noble_gas_utils.py:145-149 (Setchenow coefficients)
SETCH = {"He": (-10.081, 15.1068, 4.8127),
         "Ne": (-11.9556, 18.4062, 5.5464),
         "Ar": (-10.6951, 16.7513, 4.9551),
         "Kr": (-9.9787, 15.7619, 4.6181),
         "Xe": (-14.5524, 22.5255, 6.7513)}


def _f(x):
    return np.asarray(x, dtype=np.float64)


def lapse_rate(E):
    """noble_gas_utils.py:103-113 -- pressure [GPa] from elevation [m]."""
    E = _f(E)
    return ((1 - .0065 * E / 288.15) ** 5.2561) * 0.000101325


def parse_P(P, E):
    """noble_gas_utils.py:91-100."""
    if isinstance(P, str) and P == "1atm":
        return np.broadcast_to(_f(0.000101325), np.shape(E)).astype(np.float64)
    if isinstance(P, str) and P == "lapse_rate":
        return lapse_rate(E)
    return _f(P)


def solubility(gas, T, S=0.0):
    """noble_gas_utils.py:117-180 -- Henry coefficient K [GPa] (elementwise over T)."""
    gas = gas[0:2]
    T = _f(T)
    S = _f(S)
    T_k = T + 273.15
    G1, G2, G3 = SETCH[gas]
    with np.errstate(all="ignore"):
        setch = G1 + (G2 / (.01 * T_k)) + (G3 * np.log(.01 * T_k))
        gamma = np.where(T < 65., np.exp(S * setch), 1.)
        A0, A1, A2, A3 = SOL[gas]
        x = .001 * T_k
        if gas == "He":
            ln_F_He = A0 + (A1 / x) + (A2 / x ** 2) + (A3 / x ** 3)
            F = np.exp(ln_F_He)
            Frac_He_gas = 5.24e-6 / 9.31e-3
            a0, a1, a2, a3 = SOL["Ar"]
            X_Ar_water = 1. / (np.exp(a0 + (a1 / x) + (a2 / x ** 2) + (a3 / x ** 3))) * 9.31e-3
            X_he_water = F * Frac_He_gas * X_Ar_water
            K_h = 5.24e-6 / X_he_water
            K = gamma * K_h
        else:
            ln_K = A0 + (A1 / x) + (A2 / x ** 2) + (A3 / x ** 3)
            K_h = np.exp(ln_K)
            K = gamma * K_h
    return K


def vapor_pressure(T):
    """noble_gas_utils.py:184-199 -- Antoine equation, GPa."""
    T = _f(T)
    A = np.where(T <= 99.0, 8.07131, 8.14019)
    B = np.where(T <= 99.0, 1730.63, 1810.94)
    C = np.where(T <= 99.0, 233.426, 244.485)
    with np.errstate(all="ignore"):
        P = 10 ** (A - (B / (C + T)))
        P = P / 760. * 101325
        return P / 1.0e9


def equil_conc(gases, T, P, S=0.0):
    """noble_gas_utils.py:202-213 (wet pressure)."""
    out = {}
    for gas in gases:
        K_i = solubility(gas, T, S)
        p_i = ATM_STD[gas] * P
        with np.errstate(all="ignore"):
            x_i = p_i / K_i
            out[gas] = x_i * (22414. / 18.)
    return out


def equil_conc_dry(gases, T, P, S=0.0):
    """noble_gas_utils.py:216-232 (dry pressure; T<0 -> -9999 sentinel)."""
    T = _f(T)
    p_vapor = vapor_pressure(T)
    out = {}
    for gas in gases:
        K_i = solubility(gas, T, S)
        with np.errstate(all="ignore"):
            p_i = ATM_STD[gas] * (P - p_vapor)
            x_i = p_i / K_i
            out[gas] = np.where(T < 0.0, -9999.0, x_i * (22414. / 18.))
    return out


def ce_exc(gases, E, T, Ae, F, P="lapse_rate", S=0.0, add_eq_conc=True):
    """noble_gas_utils.py:235-253: closed-system excess air.  Returns dict gas -> array."""
    E, T, Ae, F = _f(E), _f(T), _f(Ae), _f(F)
    Pv = parse_P(P, E)
    C_eq = equil_conc_dry(gases, T, Pv, S)
    out = {}
    for gas in gases:
        z_i = ATM_STD[gas]
        with np.errstate(all="ignore"):
            C_ex = ((1 - F) * Ae * z_i) / (1 + ((F * Ae * z_i) / C_eq[gas]))
            out[gas] = C_ex + C_eq[gas] if add_eq_conc else C_ex
    return out


def ce_exc_wrapper(theta, gases=("Ne", "Ar", "Kr", "Xe")):
    """ng_interp/noble_gas_mcmc.py:205-213: theta=[log10 Ae, log10 F, E, T] -> conc[G]."""
    Ae_log, F_log, E, T = theta
    Ae, F = 10 ** Ae_log, 10 ** F_log
    r = ce_exc(list(gases), E, T, Ae, F, P="lapse_rate", add_eq_conc=True)
    return np.array([r[g] for g in gases])


def J_flux(Del, rho_r, rho_w, U, Th, phi):
    """noble_gas_utils.py:335-348: He accumulation rate [ccSTP/g/yr]."""
    PU = 1.19e-13
    PTh = 2.88e-14
    return Del * rho_r / rho_w * (U * PU + Th * PTh) * ((1 - phi) / phi)
