"""ctypes binding of libngrtd.so (include/ngrtd.h).

This is the only way the package reaches the device: there is no CPU fallback.  If the
library is missing (not built) or no GPU is visible, every compute entry raises.
"""
import ctypes as C
import os
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# NGRTD_LIB selects an instrumented build (tools/section_probe.py); default: the product library
LIB_PATH = os.environ.get("NGRTD_LIB") or os.path.join(_HERE, "libngrtd.so")

NGRTD_OK, NGRTD_EINVAL, NGRTD_EDEVICE, NGRTD_ENOMEM, NGRTD_ESTATE = 0, -1, -2, -3, -4
MEM_HOST, MEM_DEVICE = 0, 1
MAX_GASES, MAX_TRACERS, ROLE_COUNT = 5, 8, 17
MOD_NONE = -1
CE_WHAT = {"ce_total": 0, "ce_excess": 1, "equil_dry": 2, "equil": 3, "solubility": 4,
           "vapor_pressure": 5, "pressure": 6}
P_MODE = {"lapse_rate": 0, "1atm": 1, "given": 2}
HE_OUT = ("He4_eq", "He4_atm", "He4_ter", "He4_del", "He3_tu")       # enum ngrtd_he_out
CFC_SPECIES = {11: 0, 12: 1, 113: 2, "SF6": 3}                      # enum ngrtd_cfc_species
CFC_WHAT = {"equil_air": 0, "equil_aq": 1, "ce_exc": 2, "solubility": 3, "vapor_pressure_atm": 4,
            "lapse_rate_atm": 5}
WANT_LIKE, WANT_PRIOR, WANT_JACOBIAN, EXACT_RTD = 1, 2, 4, 8
DISP_WIDE, DISP_LANE = 16, 32
TUNE_TARGET = {None: 0, "none": 0, "scaling": 1, "lambda": 2}       # enum ngrtd_tune_target

_dp = C.POINTER(C.c_double)
_i32p = C.POINTER(C.c_int32)
_i64p = C.POINTER(C.c_int64)


class TracerDesc(C.Structure):
    _fields_ = [("series_id", C.c_int32), ("accum", C.c_int32), ("t_half", C.c_double), ("J", C.c_double),
                ("is_cfc12", C.c_int32), ("is_sf6", C.c_int32)]


class DemczState(C.Structure):
    """ngrtd_demcz_state: device pointers + the host-side counters of a DEMetropolisZ run."""
    _fields_ = [("lamb", C.c_void_p), ("scaling", C.c_void_p), ("n_acc_tune", C.c_void_p), ("hist", C.c_void_p),
                ("hist_cap", C.c_int64), ("hist_len", C.c_int64), ("hist_lo", C.c_int64),
                ("steps_done", C.c_int64), ("n_tune", C.c_int64), ("tune_interval", C.c_int32),
                ("tune_target", C.c_int32), ("drop_fraction", C.c_double), ("seed", C.c_uint64),
                ("chain0", C.c_int64), ("n_chains_total", C.c_int64), ("S", C.c_void_p),
                ("theta_u", C.c_void_p), ("tr_kind", C.c_int32 * ROLE_COUNT), ("tr_a", C.c_double * ROLE_COUNT),
                ("tr_b", C.c_double * ROLE_COUNT), ("per_well", C.c_int32), ("n_wells_total", C.c_int32),
                ("well0", C.c_int64), ("accept_log", C.c_void_p)]


class ModelDesc(C.Structure):
    _fields_ = [
        ("n_wells", C.c_int32), ("n_params", C.c_int32), ("role_index", C.c_int32 * ROLE_COUNT),
        ("flags", C.c_int32),
        ("ce_enabled", C.c_int32), ("ce_n_gases", C.c_int32), ("ce_gas_ids", C.c_int32 * MAX_GASES),
        ("ce_obs", _dp), ("ce_sd", _dp), ("ce_E_min", _dp),
        ("ce_E_max", C.c_double), ("ce_logA_min", C.c_double), ("ce_logA_max", C.c_double),
        ("ce_logF_min", C.c_double), ("ce_logF_max", C.c_double),
        ("ce_b_min", C.c_double), ("ce_b_max", C.c_double), ("ce_m_mu", C.c_double), ("ce_m_sd", C.c_double),
        ("ce_nu_min", C.c_double), ("ce_nu_max", C.c_double),
        ("ce_beta_a", C.c_double * 5), ("ce_beta_b", C.c_double * 5),
        ("rtd_enabled", C.c_int32), ("n_tracers", C.c_int32), ("mod_type1", C.c_int32), ("mod_type2", C.c_int32),
        ("tracers", TracerDesc * MAX_TRACERS),
        ("rtd_obs", _dp), ("rtd_sd", _dp),
        ("tau1_lo", C.c_double), ("tau1_hi", C.c_double), ("tau2_lo", C.c_double), ("tau2_hi", C.c_double),
        ("f1_lo", C.c_double), ("f1_hi", C.c_double),
        ("eta1_lo", C.c_double), ("eta1_hi", C.c_double), ("eta2_lo", C.c_double), ("eta2_hi", C.c_double),
        ("D1_lo", C.c_double), ("D1_hi", C.c_double), ("D2_lo", C.c_double), ("D2_hi", C.c_double),
        ("J_mu", C.c_double), ("J_sd", C.c_double), ("thalf_lo", C.c_double), ("thalf_hi", C.c_double),
        ("thalf_a", C.c_double), ("thalf_b", C.c_double), ("lamsf6_sd", C.c_double),
        ("rtd_nu_min", C.c_double), ("rtd_nu_max", C.c_double), ("rtd_nu_a", C.c_double), ("rtd_nu_b", C.c_double),
    ]


# name -> (restype, argtypes): exactly the functions declared in include/ngrtd.h
PROTOTYPES = {
    "ngrtd_abi_version": (C.c_int, []),
    "ngrtd_create": (C.c_int, [C.POINTER(C.c_void_p), C.c_int]),
    "ngrtd_destroy": (C.c_int, [C.c_void_p]),
    "ngrtd_last_error": (C.c_char_p, [C.c_void_p]),
    "ngrtd_set_stream": (C.c_int, [C.c_void_p, C.c_void_p]),
    "ngrtd_synchronize": (C.c_int, [C.c_void_p]),
    "ngrtd_set_profiling": (C.c_int, [C.c_void_p, C.c_int]),
    "ngrtd_ce_forward": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                   C.c_void_p, C.c_void_p, C.c_int64, _i32p, C.c_int32, C.c_void_p, C.c_int32]),
    "ngrtd_he_comps": (C.c_int, [C.c_void_p] + [C.c_void_p] * 7 + [C.c_double, C.c_int64, C.c_void_p, C.c_int32]),
    "ngrtd_cfc_corr": (C.c_int, [C.c_void_p, C.c_int32, _i32p, C.c_int32] + [C.c_void_p] * 7
                       + [C.c_int64, C.c_void_p, C.c_int32]),
    "ngrtd_series_create": (C.c_int, [C.c_void_p, _dp, _dp, C.c_int64, C.c_double, _i32p]),
    "ngrtd_series_destroy": (C.c_int, [C.c_void_p, C.c_int32]),
    "ngrtd_conv": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p,
                             C.c_void_p, C.c_double, C.c_void_p, C.c_double, C.c_int64, C.c_void_p, C.c_int32]),
    "ngrtd_rtd_weights": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32, C.c_double, C.c_double, C.c_double,
                                    C.c_void_p, C.c_int32]),
    "ngrtd_frac_conv": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32] + [C.c_void_p] * 5
                        + [C.c_int64, C.c_void_p, C.c_double, C.c_void_p, C.c_double, C.c_int64]
                        + [C.c_void_p] * 3 + [C.c_int32]),
    "ngrtd_conv_dot": (C.c_int, [C.c_void_p, C.c_int32, C.c_void_p, C.c_double, C.c_int32, C.c_double,
                                 C.c_void_p, C.c_int32]),
    "ngrtd_plan_create": (C.c_int, [C.c_void_p, C.POINTER(ModelDesc), C.c_int64, C.POINTER(C.c_void_p)]),
    "ngrtd_plan_destroy": (C.c_int, [C.c_void_p]),
    "ngrtd_logp": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_int32]),
    "ngrtd_logp_n": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_int64]),
    "ngrtd_plan_region_ms": (C.c_int, [C.c_void_p, C.POINTER(C.c_float)]),
    "ngrtd_forward": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, C.c_int32]),
    "ngrtd_plan_kernel_stats": (C.c_int, [C.c_void_p, _dp, _i64p, C.c_int32, C.c_int32]),
    "ngrtd_plan_info": (C.c_int, [C.c_void_p, C.c_int64, _i64p, C.c_int32]),
    "ngrtd_demcz_run": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_int64, C.c_void_p,
                                  C.c_void_p, C.c_void_p, C.c_void_p]),
    "ngrtd_logp_units": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_int32]),
    "ngrtd_pymc3_backward": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_int32, C.c_int64, _i32p,
                                       _dp, _dp]),
    "ngrtd_fm_log": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64]),
    "ngrtd_surrogate_check": (C.c_int, [_dp, C.c_int32, C.c_int64, C.c_double, _dp, _dp]),
    "ngrtd_c0_check": (C.c_int, [C.c_double, C.c_double, _dp, _i32p, _i32p, _dp]),
    "ngrtd_epm_window_check": (C.c_int, [C.c_double, C.c_double, C.c_double, C.c_int32, _i32p]),
    "ngrtd_comm_unique_id": (C.c_int, [C.c_char_p, C.c_void_p]),
    "ngrtd_comm_create": (C.c_int, [C.c_void_p, C.c_char_p, C.c_void_p, C.c_int32, C.c_int32, C.POINTER(C.c_void_p)]),
    "ngrtd_comm_destroy": (C.c_int, [C.c_void_p]),
    "ngrtd_logp_gather_n": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_int64, C.c_void_p, C.c_void_p,
                                      C.c_int64]),
}


class NgrtdError(RuntimeError):
    pass


_lib = None
_lib_lock = threading.Lock()


def load():
    """Load libngrtd.so (raises if it has not been built)."""
    global _lib
    with _lib_lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise NgrtdError("libngrtd.so not found at %s: build it with "
                                 "`python -c 'import __graft_entry__ as g; g.build()'`" % LIB_PATH)
            # One HIP runtime per process: torch bundles its own libamdhip64.so.7 (same
            # soname as /opt/rocm's).  Import torch first so libngrtd binds to that copy;
            # loading /opt/rocm's first leaves torch unable to see the GPU.
            try:
                import torch  # noqa: F401
            except ImportError:
                pass
            lib = C.CDLL(LIB_PATH)
            for name, (res, args) in PROTOTYPES.items():
                fn = getattr(lib, name)
                fn.restype = res
                fn.argtypes = args
            if lib.ngrtd_abi_version() != 1:
                raise NgrtdError("libngrtd ABI mismatch")
            _lib = lib
    return _lib


def dptr(a):
    """double* of a contiguous float64 numpy array (or None)."""
    if a is None:
        return None
    return a.ctypes.data_as(_dp)


class Context:
    """One ngrtd_ctx per (process, device); created lazily, re-created after fork()."""
    _instances = {}

    def __init__(self, device=0):
        self.lib = load()
        self.device = device
        h = C.c_void_p()
        st = self.lib.ngrtd_create(C.byref(h), int(device))
        if st != NGRTD_OK:
            raise NgrtdError("ngrtd_create(device=%d) failed with status %d (no GPU visible?)" % (device, st))
        self.h = h
        self.pid = os.getpid()

    @classmethod
    def get(cls, device=0):
        key = (os.getpid(), device)
        ctx = cls._instances.get(key)
        if ctx is None:
            ctx = cls(device)
            cls._instances[key] = ctx
        return ctx

    def check(self, status, what=""):
        if status != NGRTD_OK:
            msg = self.lib.ngrtd_last_error(self.h)
            raise NgrtdError("%s failed (status %d): %s" % (what, status, msg.decode() if msg else ""))

    _stream = None

    def set_stream(self, stream_handle):
        """Enqueue on this hipStream_t from now on (skipped when it is already the ctx stream)."""
        h = int(stream_handle)
        if h == self._stream:
            return
        self.check(self.lib.ngrtd_set_stream(self.h, C.c_void_p(h)), "ngrtd_set_stream")
        self._stream = h

    def synchronize(self):
        self.check(self.lib.ngrtd_synchronize(self.h), "ngrtd_synchronize")

    def set_profiling(self, on):
        self.check(self.lib.ngrtd_set_profiling(self.h, int(bool(on))), "ngrtd_set_profiling")

    def series_create(self, c_by_age, idx_by_age, dtp):
        c = np.ascontiguousarray(c_by_age, dtype=np.float64)
        i = np.ascontiguousarray(idx_by_age, dtype=np.float64)
        sid = C.c_int32()
        self.check(self.lib.ngrtd_series_create(self.h, dptr(c), dptr(i), c.shape[0], float(dtp), C.byref(sid)),
                   "ngrtd_series_create")
        return sid.value

    def series_destroy(self, sid):
        self.check(self.lib.ngrtd_series_destroy(self.h, int(sid)), "ngrtd_series_destroy")
