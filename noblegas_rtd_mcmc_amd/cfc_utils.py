"""Drop-in for the reference's ``utils/cfc_utils.py`` (CFC / SF6 excess-air and
recharge-condition correction), evaluated on the GPU through ``ngrtd_cfc_corr``.

Same classes, constructor arguments, methods and return shapes as the reference:

    c = cfc_ce_corr(cfc_num=[11, 12, 113], E=E, T=T, Ae=Ae, F=F)
    c.equil_air_conc_cfc(C_meas)      # aqueous pmol/kg -> pptv, [len(cfc_num)]
    sf6_ce_corr(E=E, T=T, Ae=Ae, F=F).equil_air_conc_sf6(C_meas)

E, T, Ae, F (and S) may be numpy arrays of ensemble members (shape [...]); C_meas / z_i
then carry the species on their LAST axis ([..., len(cfc_num)] for CFCs, [...] for SF6)
and every member is evaluated in one launch -- the loop of age_modeling_mcmc.prep.py:
247-305 in a single call.  Scalars give what the reference gives (numpy arrays of
len(cfc_num) for CFCs, floats for SF6).
"""
import ctypes as C

import numpy as np

from . import _lib


def _call(what, species, E, T, Ae, F, S, P, x, device=0):
    """One ngrtd_cfc_corr launch.  x: [..., ns] (or None).  Returns (out [ns][n] or [n], shape)."""
    ns = len(species)
    base = np.broadcast_arrays(*[np.asarray(v if v is not None else 0.0, dtype=np.float64)
                                 for v in (E, T, Ae, F, S, P)])
    shape = base[0].shape
    if x is not None:
        xa = np.asarray(x, dtype=np.float64)
        if species == ("SF6",):
            xa = xa.reshape(xa.shape + (1,))      # sf6_ce_corr takes one value per member
        shape = np.broadcast_shapes(shape, xa.shape[:-1])
        xa = np.broadcast_to(xa, shape + (ns,))
        xs = np.ascontiguousarray(np.moveaxis(xa.reshape(-1, ns), 1, 0))   # [ns][n]
    base = [np.ascontiguousarray(np.broadcast_to(b, shape).ravel()) for b in base]
    n = base[0].size
    ctx = _lib.Context.get(device)
    scalar = what in ("vapor_pressure_atm", "lapse_rate_atm")
    out = np.empty(n if scalar else (ns, n))
    ptr = [b.ctypes.data_as(C.c_void_p) for b in base]
    if S is None:
        ptr[4] = None
    if P is None:
        ptr[5] = None
    xp = xs.ctypes.data_as(C.c_void_p) if x is not None else None
    ids = (C.c_int32 * max(1, ns))(*[_lib.CFC_SPECIES[s] for s in species] or [0])
    ctx.check(ctx.lib.ngrtd_cfc_corr(ctx.h, _lib.CFC_WHAT[what], ids, ns, *ptr, xp, n,
                                     out.ctypes.data_as(C.c_void_p), _lib.MEM_HOST), "ngrtd_cfc_corr")
    return out, shape


def _scalar(v, shape):
    return float(v.reshape(-1)[0]) if shape == () else v.reshape(shape)


def _species(v, shape):
    # [ns][n] -> [..., ns] (a [ns] array for scalar parameters, like the reference)
    return np.moveaxis(v, 0, 1).reshape(shape + (v.shape[0],))


class _ce_corr:
    """Shared state of cfc_ce_corr / sf6_ce_corr (cfc_utils.py:26-32, :165-172)."""
    _species_list = ()

    def _need_P(self):
        if self.P is None:
            # the reference computes C_eq with self.P = None here and raises TypeError
            raise TypeError("unsupported operand type(s) for -: 'NoneType' and 'float' "
                            "(self.P is set by lapse_rate_atm / equil_air_conc / update_pars)")

    def vapor_pressure_atm(self):
        """:34-51 / :181-196 -- Antoine vapour pressure [atm]."""
        v, shape = _call("vapor_pressure_atm", (), self.E, self.T, None, None, None, None, None)
        return _scalar(v, shape)

    def lapse_rate_atm(self):
        """:53-62 / :198-206 -- pressure at elevation E [atm]; sets self.P."""
        v, shape = _call("lapse_rate_atm", (), self.E, self.T, None, None, None, None, None)
        self.P = _scalar(v, shape)
        return self.P

    def update_pars(self, T, E, Ae, F):
        """:144-150 / :298-304."""
        self.T = T
        self.E = E
        self.Ae = Ae * 1000
        self.F = F
        self.vapor_pressure_atm()
        self.lapse_rate_atm()

    def _solubility(self):
        v, shape = _call("solubility", self._species_list, self.E, self.T, self.Ae, self.F, self.S, None, None)
        return v, shape

    def _conv(self, what, x, P=None):
        return _call(what, self._species_list, self.E, self.T, self.Ae, self.F, self.S, P, x)


class cfc_ce_corr(_ce_corr):
    """utils/cfc_utils.py:25-151 on the GPU."""

    def __init__(self, cfc_num, E, T, Ae, F, S=0.0):
        self.cfc = cfc_num
        self.E = E
        self.T = T
        self.Ae = Ae * 1000.
        self.F = F
        self.S = S
        self.P = None
        self._species_list = tuple(cfc_num)

    def solubility_cfc(self):
        """:64-84 -- K [mol atm^-1 kg^-1] per CFC."""
        v, shape = self._solubility()
        return _species(v, shape)

    def equil_air_conc_cfc(self, C_meas):
        """:86-106 -- aqueous pmol/kg -> atmospheric mixing ratio [pptv]."""
        self.lapse_rate_atm()
        v, shape = self._conv("equil_air", C_meas)
        return _species(v, shape)

    def equil_aq_conc_cfc(self, z_i):
        """:108-124 -- mixing ratio [pptv] -> aqueous equilibrium [pmol/kg]."""
        self.lapse_rate_atm()
        v, shape = self._conv("equil_aq", z_i)
        return _species(v, shape)

    def ce_exc_conc_cfc(self, z_i):
        """:126-142 -- excess-air concentration [mol/kg] at self.P."""
        self._need_P()
        v, shape = self._conv("ce_exc", z_i, P=self.P)
        return _species(v, shape)


class sf6_ce_corr(_ce_corr):
    """utils/cfc_utils.py:160-306 on the GPU."""
    _species_list = ("SF6",)

    def __init__(self, E, T, Ae, F, S=0.0):
        self.E = E
        self.T = T
        self.Ae = Ae * 1000.
        self.F = F
        self.S = S
        self.P = None

    def solubility_sf6(self):
        """:208-221."""
        v, shape = self._solubility()
        return _scalar(v[0], shape)

    def equil_air_conc_sf6(self, C_meas):
        """:229-249 -- aqueous -> pptv."""
        self.lapse_rate_atm()
        v, shape = self._conv("equil_air", C_meas)
        return _scalar(v[0], shape)

    def equil_aq_conc_sf6(self, z_i):
        """:264-278 -- pptv -> aqueous [fmol/kg]."""
        self.lapse_rate_atm()
        v, shape = self._conv("equil_aq", z_i)
        return _scalar(v[0], shape)

    def ce_exc_conc_sf6(self, z_i):
        """:280-296 -- excess air [fmol/kg] at self.P."""
        self._need_P()
        v, shape = self._conv("ce_exc", z_i, P=self.P)
        return _scalar(v[0], shape)
