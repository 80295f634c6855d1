"""Device-resident DE-MC (ngrtd_demc_run): proposal kernel + log-prob kernel with the
Metropolis accept in its per-walker reduction.  Checked against a NumPy restatement of
the same step (same counter-based random numbers, log-probs from the parity-tested
LogProb), for invariants, and statistically on the c1 posterior."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

M64 = (1 << 64) - 1


def mix(z):
    z = (z + 0x9E3779B97F4A7C15) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def key(seed, step):
    return mix((mix(seed) + step) & M64)


def unit(h):
    return ((h >> 11) + 0.5) * (1.0 / 9007199254740992.0)


def numpy_step(x, lp, lp_fn, lamb, scaling, seed, step):
    """One step of ngrtd_demc_run restated (csrc/ngrtd_kernels.hpp demc_partners,
    demc_propose_rows_kernel / demc_propose_kernel, demc_decide); x [R][W]."""
    R, W = x.shape
    k = key(seed, step)
    k1, k2, k3 = mix((k + 1) & M64), mix((k + 2) & M64), mix((k + 3) & M64)
    prop = np.empty_like(x)
    for w in range(W):
        hp = mix((k1 + w) & M64)
        r1 = (w + 1 + (hp >> 32) % (W - 1)) % W
        r2 = (r1 + 1 + (hp & 0xFFFFFFFF) % (W - 2)) % W
        if r2 == w:
            r2 = (r2 + 1) % W
        if r2 == r1:
            r2 = (r2 + 1) % W
        for r in range(R):
            e = r * W + w
            eps = (2.0 * unit(mix((k2 + e) & M64)) - 1.0) * scaling
            prop[r, w] = x[r, w] + lamb * (x[r, r1] - x[r, r2]) + eps
    lpp = lp_fn(prop)
    out_x, out_lp, acc = x.copy(), lp.copy(), np.zeros(W, bool)
    for w in range(W):
        logu = np.log(unit(mix((k3 + w) & M64)))
        if (lpp[w] - lp[w]) > logu and lpp[w] == lpp[w]:
            acc[w] = True
            out_x[:, w] = prop[:, w]
            out_lp[w] = lpp[w]
    return out_x, out_lp, acc


@pytest.mark.parametrize("kind", ["joint", "ce_only"])
def test_demc_matches_numpy_restatement(kind):
    import torch
    from noblegas_rtd_mcmc_amd import workloads as wl
    from noblegas_rtd_mcmc_amd.engine import LogProb
    from noblegas_rtd_mcmc_amd.spec import ModelSpec
    spec = wl.c4_spec(L=4, N=300)
    if kind == "ce_only":                  # no RTD block: generic kernels + demc_accept_kernel
        spec = ModelSpec(n_wells=4, ce=spec.ce)
    W = 40
    th0 = wl.sample_prior(spec, W, np.random.default_rng(5))
    lp = LogProb(spec, max_walkers=W)
    P, L = th0.shape[0], th0.shape[1]
    fn = lambda v: lp(np.ascontiguousarray(v.reshape(P, L, W)), soa=True)
    x = torch.from_numpy(th0).cuda()
    lpv = lp(x).clone()
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    acc = torch.zeros(W, dtype=torch.int32, device="cuda")
    lamb, scaling, seed = 0.02, 1e-5, 987654321
    lp.demc(x, lpv, 3, lamb, scaling, seed, step0=11, n_accepted=cnt, accepted=acc)
    rx, rlp = th0.reshape(P * L, W), fn(th0.reshape(P * L, W))
    total = 0
    for s in range(3):
        rx, rlp, racc = numpy_step(rx, rlp, fn, lamb, scaling, seed, 11 + s)
        total += int(racc.sum())
    assert np.array_equal(x.cpu().numpy().reshape(P * L, W), rx)
    assert np.array_equal(lpv.cpu().numpy(), rlp)
    assert np.array_equal(acc.cpu().numpy().astype(bool), racc)
    assert int(cnt.item()) == total and 0 < total < 3 * W
    lp.close()


def test_demc_unstaged_proposal_large_w():
    """W > 8192: a row of theta no longer fits the proposal kernel's LDS staging
    (demc_propose_rows_kernel), so ngrtd_demc_run takes the gather kernel
    (demc_propose_kernel); same step, bitwise."""
    import torch
    from noblegas_rtd_mcmc_amd import workloads as wl
    from noblegas_rtd_mcmc_amd.engine import LogProb
    from noblegas_rtd_mcmc_amd.spec import ModelSpec
    spec = ModelSpec(n_wells=1, ce=wl.c4_spec(L=1, N=300).ce)
    W = 8200
    th0 = wl.sample_prior(spec, W, np.random.default_rng(8))
    lp = LogProb(spec, max_walkers=W)
    P, L = th0.shape[0], th0.shape[1]
    fn = lambda v: lp(np.ascontiguousarray(v.reshape(P, L, W)), soa=True)
    x = torch.from_numpy(th0).cuda()
    lpv = lp(x).clone()
    lamb, scaling, seed = 0.05, 1e-4, 4242
    lp.demc(x, lpv, 1, lamb, scaling, seed, step0=3)
    rx, rlp, _ = numpy_step(th0.reshape(P * L, W), fn(th0.reshape(P * L, W)), fn, lamb, scaling, seed, 3)
    assert np.array_equal(x.cpu().numpy().reshape(P * L, W), rx)
    assert np.array_equal(lpv.cpu().numpy(), rlp)
    lp.close()


def test_demc_invariants_c4():
    """lamb = scaling = 0: every proposal is the current state, so every step accepts and
    nothing moves; after a real run the tracked logp equals a fresh evaluation."""
    import torch
    from noblegas_rtd_mcmc_amd import workloads as wl
    from noblegas_rtd_mcmc_amd.engine import LogProb
    spec = wl.c4_spec(L=8, N=1200)
    W = 256
    th0 = wl.sample_prior(spec, W, np.random.default_rng(6))
    lp = LogProb(spec, max_walkers=W)
    x = torch.from_numpy(th0).cuda()
    lpv = lp(x).clone()
    lp0 = lpv.clone()
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    lp.demc(x, lpv, 4, 0.0, 0.0, 1, n_accepted=cnt)
    fin = torch.isfinite(lp0)
    assert torch.equal(x, torch.from_numpy(th0).cuda())
    assert torch.equal(lpv[fin], lp0[fin])
    assert int(cnt.item()) >= 4 * int(fin.sum())
    cnt.zero_()
    lp.demc(x, lpv, 25, 0.3, 1e-3, 2, n_accepted=cnt)
    assert torch.equal(lpv, lp(x))
    assert 0 < int(cnt.item()) < 25 * W
    lp.close()


def test_c1_torch_sampler_path():
    """The torch-op DEMetropolis path stays available (sampler="torch")."""
    from noblegas_rtd_mcmc_amd.noble_gas_mcmc import CEModel
    from noblegas_rtd_mcmc_amd.workloads import field_data
    m = CEModel(field_data()["obs"], ["PLM1"], max_walkers=64)
    res = m.sample(nwalkers=32, tune=40, draws=20, seed=3, tune_interval=20, sampler="torch")
    assert res["samples"].shape[0] == 20 and 0.0 < res["accept_rate"] < 1.0
