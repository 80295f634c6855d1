#!/usr/bin/env python3
"""Freeze the reference's own PyMC3 DEMetropolisZ acceptance statistics as a fixture.

Run in the build container only (needs /root/reference):

    python tests/golden/make_pymc3_accept.py

The reference ships 22 traces of its published RTD runs
(age_ens_runs_mcmc/conv_traces/*.netcdf, written by az.to_netcdf at
run_age_mcmc_utils.py:425 after mc.sample(..., step=DEMetropolisZ) at :407-417).  PyMC3
3.11.2's DEMetropolisZ.astep records the stat ``accept`` = exp(logp(q) - logp(q0)) of every
proposal, where logp is the model's log-density in PyMC3's TRANSFORMED space (interval /
logodds / log transforms, with their log-Jacobians); for an accepted step q is the next
draw.  So for every accepted transition t-1 -> t of a chain

    log(accept[t]) = logp(x_t) - logp(x_{t-1})                                   (*)

pins the reference's transformed-space RTD log-prob of that run at its own series length
(N = 25 256, the full C_in_dict), its priors, Jacobians, Student-t and every tracer's
convolution -- up to what the traces do not hold:

* the observation error sigma_k = std(ens) + mu_k * perr (run_age_mcmc_utils.py:353-356):
  ens_dict.pk is missing (.MISSING_LARGE_BLOBS), so one sigma per tracer is FITTED here by
  least squares over the run's transitions (thousands of equations, <= 4 unknowns);
  mu_k = mean(ens) IS in the trace (observed_data/like);
* the tau1 prior bounds of runs that predate run_age_mcmc.py:145-146's U(1, 1000) (their
  tau1 draws reach 5000): (a, b) is chosen from a grid of round values with the same fit.

Transitions are kept only where the natural-space draws determine the transformed-space
log-prob to better than 1e-10: the trace stores x = backward(u) rounded to float64, and a
logodds variable within 1e-6 of 0 or 1 (nu_ of Beta(2, 0.1) often sits at 1 - 2^-52) or an
interval variable within 1e-6 (relative) of a bound loses the digits of u that PyMC3's
log-Jacobian and Beta term use.  Up to ``MAX_T`` of the remaining transitions per trace are
drawn with a fixed seed.

The fit uses the CPU oracle (oracle/vectorized.py, the restatement pinned to the
reference's own convolve() by conv_golden.npz).  Output: tests/golden/pymc3_accept.npz
(per trace: the two natural-space states of every kept transition in the engine's role
order, log(accept), mu, the fitted sigma and bounds) and pymc3_accept_fit.json (the fit
report DESIGN.md quotes).
"""
import glob
import json
import os
import sys

import numpy as np
from scipy.optimize import least_squares
from scipy.special import gammaln

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, REPO)
REF = os.environ.get("NGRTD_REFERENCE", "/root/reference")
TRACES = os.path.join(REF, "age_ens_runs_mcmc", "conv_traces")
MAX_T = int(os.environ.get("NGRTD_ACCEPT_MAX_T", "1000"))
COND = 1e-6

from noblegas_rtd_mcmc_amd import trace as _trace            # noqa: E402
from noblegas_rtd_mcmc_amd import workloads as wl            # noqa: E402
from noblegas_rtd_mcmc_amd.spec import ModelSpec, RTDBlock   # noqa: E402
from oracle import vectorized as ov                          # noqa: E402
from oracle import stats as st                               # noqa: E402

# candidate tau1 prior bounds for the runs whose draws leave U(1, 1000)
TAU1_A = (1.0, 0.0, 0.1, 0.5, 2.0, 5.0, 10.0)
TAU1_B = (100.0, 200.0, 250.0, 300.0, 400.0, 500.0, 600.0, 700.0, 750.0, 800.0, 900.0, 1000.0, 1200.0,
          1500.0, 2000.0, 2500.0, 3000.0, 4000.0, 5000.0, 6000.0, 7500.0, 8000.0, 10000.0, 15000.0,
          20000.0, 25000.0, 50000.0)


def parse_name(path):
    """PLM1.CFC12.SF6.H3.He4_ter.exp_pist_flow-piston.123.netcdf -> (well, tracers, mod1, mod2, savenum)
    (run_age_mcmc_utils.py trace_name: well.tracers.mod_type1[-mod_type2].savenum)."""
    parts = os.path.basename(path)[:-len(".netcdf")].split(".")
    well, savenum, model = parts[0], parts[-1], parts[-2]
    tracers = tuple(parts[1:-2])
    mods = model.split("-")
    return well, tracers, mods[0], (mods[1] if len(mods) > 1 else None), savenum


def make_spec(tracers, mod1, mod2, savenum, mu, sd, tau1=(1.0, 1000.0)):
    """The run's RTD model (run_age_mcmc.py:140-224) on the full shipped series, one well,
    PyMC3's transformed-space log-prob (Jacobians on)."""
    pn = wl.model_par_names(mod1, mod2, "" if savenum == "0" else savenum)
    rtd = RTDBlock(tracers=[wl.tracer(t, None) for t in tracers], obs=np.asarray(mu, float)[None, :],
                   sd=np.asarray(sd, float)[None, :], mod_type1=mod1, mod_type2=mod2, par_names=pn,
                   tau1=tuple(tau1))
    return ModelSpec(n_wells=1, rtd=rtd, jacobian=True)


def states_from_trace(t, spec):
    """Natural-space draws [chain][draw][P] in spec.roles order."""
    post = t["posterior"]
    name = {"tau1": "tau1", "tau2": "tau2", "f1": "f1", "eta1": "eta1", "eta2": "eta2", "D1": "D1", "D2": "D2",
            "J": "J", "thalf_cfc_beta": "thalf_cfc_", "lamsf6": "lamsf6", "nu_rtd_beta": "nu_"}
    return np.stack([np.asarray(post[name[r]][1], dtype=np.float64) for r in spec.roles], axis=-1)


def well_conditioned(x, spec, tau1):
    """[..., P] -> bool: every transformed variable is far enough from its bounds that the
    float64 natural value pins u (see the module docstring)."""
    r = spec.rtd
    ok = np.ones(x.shape[:-1], bool)
    for i, role in enumerate(spec.roles):
        v = x[..., i]
        if role in ("nu_rtd_beta", "thalf_cfc_beta"):
            ok &= (v > COND) & (1.0 - v > COND)
        elif role in ("tau1", "tau2", "f1", "eta1", "eta2", "D1", "D2"):
            if role == "tau1" and tau1 is None:           # bounds not chosen yet
                continue
            lo, hi = tau1 if role == "tau1" else getattr(r, role)
            ok &= (v - lo > COND * (hi - lo)) & (hi - v > COND * (hi - lo))
        elif role == "lamsf6":
            ok &= v > 0
    return ok


def oracle_parts(spec, X):
    """For states X [n][P]: (nu, concentrations [K][n]) from the oracle."""
    th = spec.theta_soa(X[:, None, :])                       # [P][1][n]
    r = spec.rtd
    nu = th[spec.roles.index("nu_rtd_beta"), 0] * (r.nu_max - r.nu_min) + r.nu_min
    conc = np.zeros((len(r.tracers), X.shape[0]))
    for k in range(len(r.tracers)):
        conc[k] = _conc_one(spec, th, k)
    return nu, conc


def _conc_one(spec, th, k):
    """Tracer k's ForwardMod output for every state, through oracle.vectorized's own
    composition (run_age_mcmc_utils.py:81-163), chunked over states."""
    r = spec.rtd
    t = r.tracers[k]
    p = {role: th[i, 0] for i, role in enumerate(spec.roles)}
    names = r.par_names
    out = np.zeros(th.shape[2])
    step = 256
    for s in range(0, th.shape[2], step):
        sl = slice(s, s + step)
        q = {kk: v[sl] for kk, v in p.items()}
        lam = ov._rtd.thalf_2_lambda(t.t_half) if t.t_half else 0.0
        if "thalf_cfc" in names and t.name == "CFC12":
            lam = ov._rtd.thalf_2_lambda(q["thalf_cfc_beta"] * (r.thalf[1] - r.thalf[0]) + r.thalf[0])
        if "J" in names:
            J = 10 ** q["J"]
        elif t.name == "He4_ter":
            J = 10 ** ov._rtd.J_he4_default()
        else:
            J = 10 ** 0.0
        f1 = q["f1"] if "f1" in names else 1.0
        f2 = 1 - q["f1"] if "f1" in names else 0.0
        c = f1 * ov.convolve_batch(t, q["tau1"], r.mod_type1, lam, q.get("eta1"), q.get("D1"), J)
        if r.mod_type2:
            c = c + f2 * ov.convolve_batch(t, q["tau2"], r.mod_type2, lam, q.get("eta2"), q.get("D2"), J)
        else:
            c = c + f2 * 0.0
        if t.name == "SF6":
            c = c * (1 + (q["lamsf6"] if "lamsf6" in names else False))
        out[sl] = c
    return out


def like_terms(mu, conc, nu, sd):
    """Sum over tracers of the Student-t log-density without its -log(sigma) constant."""
    K = len(mu)
    np.seterr(all="ignore")
    c0 = gammaln((nu + 1.0) / 2.0) - gammaln(nu / 2.0) - 0.5 * np.log(nu * np.pi)
    s = K * c0
    for k in range(K):
        z = (mu[k] - conc[k]) / sd[k]
        s = s - (nu + 1.0) / 2.0 * np.log1p(z * z / nu)
    return s


def fit_sigma(d_obs, prior0, prior1, nu0, nu1, conc0, conc1, mu):
    """Least-squares sigma per tracer for d_obs = dprior + dlike(sigma)."""
    dprior = prior1 - prior0

    def res(logsd):
        sd = np.exp(logsd)
        return d_obs - dprior - (like_terms(mu, conc1, nu1, sd) - like_terms(mu, conc0, nu0, sd))

    best = None
    for scale in (0.02, 0.1, 0.3, 1.0, 3.0, 10.0):
        x0 = np.log(np.abs(mu) * scale + 1e-300)
        try:
            f = least_squares(res, x0, method="lm", xtol=1e-15, ftol=1e-15, gtol=1e-15, max_nfev=4000)
        except Exception:
            continue
        if best is None or f.cost < best.cost:
            best = f
    r = res(best.x)
    return np.exp(best.x), r


def process(path, rng):
    well, tracers, mod1, mod2, savenum = parse_name(path)
    t = _trace.from_netcdf(path)
    mu = np.asarray(t["observed_data"]["like"][1], dtype=np.float64)
    spec = make_spec(tracers, mod1, mod2, savenum, mu, np.abs(mu) * 0.1)
    X = states_from_trace(t, spec)                                           # [3][10000][P]
    acc = np.asarray(t["sample_stats"]["accepted"][1]).astype(bool)
    a = np.asarray(t["sample_stats"]["accept"][1], dtype=np.float64)
    tau_lo, tau_hi = float(X[..., 0].min()), float(X[..., 0].max())
    # bound candidates: the published U(1, 1000) first; other grid values only if draws leave it
    cands = [(1.0, 1000.0)] + [(aa, bb) for aa in TAU1_A for bb in TAU1_B
                               if aa < tau_lo and bb > tau_hi and (aa, bb) != (1.0, 1000.0)]
    cands = [c for c in cands if c[0] < tau_lo and c[1] > tau_hi]
    # transitions: accepted steps t >= 1 (the draw before t = 0 is the discarded last tune draw)
    ch, dr = np.nonzero(acc[:, 1:])
    dr = dr + 1
    x1, x0 = X[ch, dr], X[ch, dr - 1]
    d_obs = np.log(a[ch, dr])
    keep0 = np.isfinite(d_obs)
    # conditioning of every variable but tau1 (its bounds are a candidate: checked per candidate below)
    ok = keep0 & well_conditioned(x0, spec, None) & well_conditioned(x1, spec, None)
    idx = np.nonzero(ok)[0]
    sel = np.sort(rng.choice(idx, size=min(MAX_T, len(idx)), replace=False))
    x0, x1, d_obs, chs, drs = x0[sel], x1[sel], d_obs[sel], ch[sel], dr[sel]
    # concentrations do not depend on the priors: once for all candidates
    nu0, conc0 = oracle_parts(spec, x0)
    nu1, conc1 = oracle_parts(spec, x1)
    results = []
    for cand in cands:
        sp = make_spec(tracers, mod1, mod2, savenum, mu, np.abs(mu) * 0.1, tau1=cand)
        good = well_conditioned(x0, sp, cand) & well_conditioned(x1, sp, cand)
        import dataclasses
        ps = dataclasses.replace(sp, include_like=False)
        p0 = ov.log_prob_vec(ps, sp.theta_soa(x0[:, None, :]))
        p1 = ov.log_prob_vec(ps, sp.theta_soa(x1[:, None, :]))
        g = good & np.isfinite(p0) & np.isfinite(p1)
        sd, r = fit_sigma(d_obs[g], p0[g], p1[g], nu0[g], nu1[g], conc0[:, g], conc1[:, g], mu)
        results.append((float(np.max(np.abs(r))), cand, sd, g))
    results.sort(key=lambda z: z[0])
    maxres, cand, sd, g = results[0]
    second = results[1][0] if len(results) > 1 else None
    return dict(name=os.path.basename(path), well=well, tracers=tracers, mod1=mod1, mod2=mod2, savenum=savenum,
                mu=mu, sd=sd, tau1=cand, x0=x0[g], x1=x1[g], d=d_obs[g], chain=chs[g], draw=drs[g],
                roles=list(spec.roles), maxres=maxres, second=second, n_acc=int(acc[:, 1:].sum()),
                n_kept=int(g.sum()), rmsres=None)


def main():
    paths = sorted(glob.glob(os.path.join(TRACES, "*.netcdf")))
    only = os.environ.get("NGRTD_ACCEPT_ONLY")
    if only:
        paths = [p for p in paths if only in os.path.basename(p)]
    rng = np.random.default_rng(20260418)
    out, report = {}, {}
    for i, p in enumerate(paths):
        r = process(p, rng)
        key = "t%02d" % i
        out[key + "_x0"] = r["x0"]
        out[key + "_x1"] = r["x1"]
        out[key + "_dlogp"] = r["d"]
        out[key + "_chain_draw"] = np.stack([r["chain"], r["draw"]]).astype(np.int32)
        out[key + "_mu"] = r["mu"]
        out[key + "_sd"] = r["sd"]
        out[key + "_tau1"] = np.array(r["tau1"])
        report[key] = {k: (list(v) if isinstance(v, tuple) else v) for k, v in r.items()
                       if k in ("name", "well", "tracers", "mod1", "mod2", "savenum", "roles", "maxres", "second",
                                "n_acc", "n_kept", "tau1")}
        report[key]["sd"] = r["sd"].tolist()
        report[key]["mu"] = r["mu"].tolist()
        print("%-62s kept %4d/%5d  max|res| %.2e (next bound candidate %s)  tau1 %s  sd %s" % (
            r["name"], r["n_kept"], r["n_acc"], r["maxres"], "%.2e" % r["second"] if r["second"] is not None else "-",
            r["tau1"], np.array2string(r["sd"], precision=6)), flush=True)
    if only:
        return
    np.savez_compressed(os.path.join(HERE, "pymc3_accept.npz"), **out)
    with open(os.path.join(HERE, "pymc3_accept_fit.json"), "w") as f:
        json.dump(report, f, indent=1)


if __name__ == "__main__":
    main()
