"""Model specifications for the batched log-probability engine.

A ``ModelSpec`` describes one log-prob workload: L wells, an optional CE (noble gas)
block, an optional RTD (tracer convolution) block, and the per-(walker, well) parameter
layout.  It is the data-only mirror of the reference's two PyMC3 models:

* CE block  -- ng_interp/noble_gas_mcmc.py:184-267 (priors, T=(E-b)/m, StudentT over
  the gases, parameter bounds at :117-147).
* RTD block -- age_ens_runs_mcmc/run_age_mcmc_utils.py:275-397 (conv_mcmc.
  build_mcmc_model_joint_sT) with the prior/obs keywords of run_age_mcmc.py:100-224.

Parameters are the PyMC3 free random variables in their natural (untransformed) space,
laid out per (walker, well) in ``ModelSpec.roles`` order; the batched theta is
structure-of-arrays ``theta[P][L][W]`` (float64) so that a wavefront reading one role for
64 consecutive walkers issues one coalesced load.
"""
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np

GAS_IDS = {"He": 0, "Ne": 1, "Ar": 2, "Kr": 3, "Xe": 4}
MOD_IDS = {"piston": 0, "exponential": 1, "exp_pist_flow": 2, "dispersion": 3}
ACCUM_IDS = {None: 0, False: 0, "3He": 1, "4He": 2, "SF6": 3}

# Parameter roles (must match include/ngrtd.h NGRTD_ROLE_*)
ROLES = ("Ae_beta", "F_beta", "E_beta", "m", "b_beta", "nu_ce_beta",
         "tau1", "tau2", "f1", "eta1", "eta2", "D1", "D2", "J", "thalf_cfc_beta", "lamsf6",
         "nu_rtd_beta")
ROLE_IDS = {r: i for i, r in enumerate(ROLES)}
CE_ROLES = ROLES[:6]
# reference parameter-name -> role (run_age_mcmc.py:147-196 par_names)
RTD_PARNAME_TO_ROLE = {"tau1": "tau1", "tau2": "tau2", "f1": "f1", "eta1": "eta1", "eta2": "eta2",
                       "D1": "D1", "D2": "D2", "J": "J", "thalf_cfc": "thalf_cfc_beta",
                       "lamsf6": "lamsf6"}


def J_flux(Del, rho_r, rho_w, U, Th, phi):
    """utils/noble_gas_utils.py:335-348."""
    PU = 1.19e-13
    PTh = 2.88e-14
    return Del * rho_r / rho_w * (U * PU + Th * PTh) * ((1 - phi) / phi)


# run_age_mcmc_utils.py:90-91 default log10 J for He4_ter when J is not sampled
LOG10_J_HE4_DEFAULT = float(np.log10(J_flux(Del=1., rho_r=2700, rho_w=1000, U=3.0, Th=10.0, phi=0.05)))
# run_age_mcmc.py:182 prior mean of the sampled log10 J
LOG10_J_PRIOR_MU = float(np.log10(J_flux(Del=1., rho_r=2700, rho_w=1000, U=3.7, Th=10.2, phi=0.05)))


@dataclass
class Series:
    """One tracer input series, held age-first.

    ``c_by_age[k]`` = the C_t value of age k (= ``np.flip(C_t.to_numpy().ravel())``,
    convolution_integral_utils.py:336); ``idx_by_age[k]`` = the flipped C_t index (the
    4He/SF6 accumulation multiplies it, :323/:331); ``dtp`` =
    ``floor(t_samp - C_t.index[-1])`` (:172).
    """
    c_by_age: np.ndarray
    idx_by_age: Optional[np.ndarray] = None
    dtp: float = 0.0

    def __post_init__(self):
        self.c_by_age = np.ascontiguousarray(self.c_by_age, dtype=np.float64)
        if self.idx_by_age is None:
            self.idx_by_age = np.arange(len(self.c_by_age), dtype=np.float64)
        self.idx_by_age = np.ascontiguousarray(self.idx_by_age, dtype=np.float64)
        if self.idx_by_age.shape != self.c_by_age.shape:
            raise ValueError("series index/value length mismatch")
        self.dtp = float(self.dtp)

    @property
    def n(self):
        return int(self.c_by_age.shape[0])

    @classmethod
    def from_reference_frame(cls, values, index, t_samp):
        """Build from the reference's DataFrame layout (oldest age first)."""
        values = np.asarray(values, dtype=np.float64).ravel()
        index = np.asarray(index)
        return cls(np.flip(values).copy(), np.flip(index.astype(np.float64)).copy(),
                   float(np.floor(t_samp - index[-1])))

    def reference_frame(self):
        """(values, index, t_samp) in the reference's DataFrame order."""
        idx = np.flip(self.idx_by_age)
        return np.flip(self.c_by_age).copy(), idx.copy(), float(idx[-1] + self.dtp)


@dataclass
class Tracer:
    """One tracer of the RTD likelihood (ForwardMod, run_age_mcmc_utils.py:52-79, with
    the per-tracer convolution kwargs of run_age_mcmc.py:205-224)."""
    name: str
    series: Series
    t_half: Optional[float] = None          # H3/He3: 12.34 yr
    rad_accum: Optional[str] = None         # None | '3He' | '4He' | 'SF6'
    log10_J: Optional[float] = None         # fixed log10 J when 'J' is not sampled
    J_sf6: float = 0.0                      # rad_accum='SF6' zero-order rate

    @property
    def lam(self):
        return float(-1 * np.log(0.5) / self.t_half) if self.t_half else 0.0


@dataclass
class CEBlock:
    """CE noble-gas model + StudentT likelihood (noble_gas_mcmc.py:184-267)."""
    obs: np.ndarray                                   # [L][G]
    sd: np.ndarray                                    # [L][G]
    E_min: np.ndarray                                 # [L]  well_elev - 10 (:142)
    gases: Sequence[str] = ("Ne", "Ar", "Kr", "Xe")   # :109
    E_max: float = 3300.0                             # :143
    logA_min: float = float(np.log10(1.0e-4))         # :134
    logA_max: float = float(np.log10(1.0e-1))         # :135
    logF_min: float = float(np.log10(1.0e-1))         # :138
    logF_max: float = float(np.log10(1.0e+1))         # :139
    b_min: float = 3354.0 - abs(-146.0) * 2.5         # :128-131
    b_max: float = 3354.0 + abs(-146.0) * 2.5
    m_mu: float = -146.0                              # :118
    m_sd: float = 17.0                                # :119
    nu_min: float = 1.0                               # :250
    nu_max: float = 30.0
    beta_Ae: tuple = (2.0, 2.0)                       # :224-226, :237, :249
    beta_F: tuple = (2.0, 2.0)
    beta_E: tuple = (2.0, 4.0)
    beta_b: tuple = (2.0, 2.5)
    beta_nu: tuple = (2.0, 0.1)

    def __post_init__(self):
        self.obs = np.ascontiguousarray(self.obs, dtype=np.float64)
        self.sd = np.ascontiguousarray(self.sd, dtype=np.float64)
        self.E_min = np.ascontiguousarray(self.E_min, dtype=np.float64)
        self.gases = tuple(self.gases)
        G = len(self.gases)
        if self.obs.ndim != 2 or self.obs.shape[1] != G or self.sd.shape != self.obs.shape:
            raise ValueError("CE obs/sd must be [L][G]")
        if self.E_min.shape != (self.obs.shape[0],):
            raise ValueError("CE E_min must be [L]")


@dataclass
class RTDBlock:
    """RTD convolution model + StudentT likelihood (run_age_mcmc_utils.py:275-397)."""
    tracers: List[Tracer]
    obs: np.ndarray                        # [L][K]
    sd: np.ndarray                         # [L][K]
    mod_type1: str = "exponential"
    mod_type2: Optional[str] = None
    par_names: Sequence[str] = ("tau1",)   # reference par_names without 'f2'
    tau1: tuple = (1.0, 1000.0)            # run_age_mcmc.py:145-146
    tau2: tuple = (50.0, 15000.0)          # :151-152
    f1: tuple = (0.01, 0.99)               # :155-156
    eta1: tuple = (1.0, 5.0)               # :161-162
    eta2: tuple = (1.0, 5.0)
    D1: tuple = (0.01, 2.00)               # :171-172
    D2: tuple = (0.01, 2.0)
    J_mu: float = LOG10_J_PRIOR_MU         # :182
    J_sd: float = 0.33                     # :183
    thalf: tuple = (5.0, 35.0)             # :189-190
    beta_thalf: tuple = (2.0, 2.0)         # run_age_mcmc_utils.py:334
    lamsf6_sd: float = 0.5 / 3             # :343
    nu_min: float = 5.0                    # :291-292
    nu_max: float = 30.0
    beta_nu: tuple = (2.0, 0.1)

    def __post_init__(self):
        self.obs = np.ascontiguousarray(self.obs, dtype=np.float64)
        self.sd = np.ascontiguousarray(self.sd, dtype=np.float64)
        self.par_names = tuple(p for p in self.par_names if p != "f2")
        K = len(self.tracers)
        if self.obs.ndim != 2 or self.obs.shape[1] != K or self.sd.shape != self.obs.shape:
            raise ValueError("RTD obs/sd must be [L][K]")
        for m in (self.mod_type1,) + ((self.mod_type2,) if self.mod_type2 else ()):
            if m not in MOD_IDS:
                raise ValueError("unsupported mod_type %r" % m)
        for p in self.par_names:
            if p not in RTD_PARNAME_TO_ROLE:
                raise ValueError("unknown RTD parameter %r" % p)
        ns = {t.series.n for t in self.tracers}
        if len(ns) != 1:
            raise ValueError("all tracers of one RTD block must share the series length N")
        for t in self.tracers:
            if "thalf_cfc" in self.par_names and t.name == "CFC12" and t.rad_accum:
                raise ValueError("per-walker CFC12 decay with accumulation is not a reference case")

    @property
    def n_ages(self):
        return self.tracers[0].series.n


@dataclass
class ModelSpec:
    """A full per-walker log-prob: sum over wells of CE and/or RTD terms."""
    n_wells: int
    ce: Optional[CEBlock] = None
    rtd: Optional[RTDBlock] = None
    include_prior: bool = True
    include_like: bool = True
    jacobian: bool = False             # add PyMC3 transform log|J| (parity unpinned)
    exact_rtd: bool = False            # no channel-sum surrogate: exact sums on the matrix cores
    # a dispersion component's age sum: "auto" (plans of <= 256 units across the lanes of the
    # wide kernel, larger ones one lane per unit), "wide" or "lane" (ngrtd.h NGRTD_DISP_*)
    disp_geometry: str = "auto"
    roles: List[str] = field(default_factory=list)

    def __post_init__(self):
        if self.ce is None and self.rtd is None:
            raise ValueError("ModelSpec needs a CE and/or an RTD block")
        roles = []
        if self.ce is not None:
            if self.ce.obs.shape[0] != self.n_wells:
                raise ValueError("CE block well count mismatch")
            roles += list(CE_ROLES)
        if self.rtd is not None:
            if self.rtd.obs.shape[0] != self.n_wells:
                raise ValueError("RTD block well count mismatch")
            roles += ["tau1", "nu_rtd_beta"]
            for p in self.rtd.par_names:
                r = RTD_PARNAME_TO_ROLE[p]
                if r not in roles:
                    roles.append(r)
        if not self.roles:
            self.roles = roles
        elif sorted(self.roles) != sorted(roles):
            raise ValueError("roles %r do not match the blocks (%r)" % (self.roles, roles))

    @property
    def n_params(self):
        return len(self.roles)

    def well(self, l):
        """The one-well model of well l (what the reference builds per well:
        run_age_mcmc.py:122-231, noble_gas_mcmc.py:95-104)."""
        import dataclasses
        ce = rtd = None
        if self.ce is not None:
            ce = dataclasses.replace(self.ce, obs=self.ce.obs[l:l + 1], sd=self.ce.sd[l:l + 1],
                                     E_min=self.ce.E_min[l:l + 1])
        if self.rtd is not None:
            rtd = dataclasses.replace(self.rtd, obs=self.rtd.obs[l:l + 1], sd=self.rtd.sd[l:l + 1])
        return dataclasses.replace(self, n_wells=1, ce=ce, rtd=rtd, roles=list(self.roles))

    def role_index(self):
        idx = [-1] * len(ROLES)
        for i, r in enumerate(self.roles):
            idx[ROLE_IDS[r]] = i
        return idx

    def theta_soa(self, theta_wlp):
        """[W][L][P] (or [W][L*P]) natural-space params -> SoA [P][L][W]."""
        t = np.asarray(theta_wlp, dtype=np.float64)
        W = t.shape[0]
        t = t.reshape(W, self.n_wells, self.n_params)
        return np.ascontiguousarray(np.transpose(t, (2, 1, 0)))

    def theta_wlp(self, theta_soa):
        t = np.asarray(theta_soa, dtype=np.float64)
        return np.ascontiguousarray(np.transpose(t, (2, 1, 0)))
