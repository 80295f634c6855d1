"""Device-resident DEMetropolisZ (ngrtd_demcz_run): the proposal kernel (with the history
append) + the log-prob kernel with the Metropolis decision and the PyMC3 tuning in its
per-walker reduction.  Checked bitwise against sampler.DEMetropolisZ (torch ops, same
counter-based random numbers, log-probs from the parity-tested LogProb), for
invariants, and statistically: the stationary distribution of a prior-only plan against
the analytic prior moments, the c1 CE posterior against the reference's summaries."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _same(a, b):
    import torch
    return torch.equal(a, b) or bool(((a == b) | (torch.isnan(a) & torch.isnan(b))).all())


@pytest.mark.parametrize("per_well", [True, False])
@pytest.mark.parametrize("kind", ["joint", "ce_only", "joint_transformed", "bmm_transformed", "bmm", "epm",
                                  "epm_piston", "epm_transformed", "joint_c4_transformed", "joint_l3",
                                  "joint_123", "epm_123_transformed", "bmm_123", "rtd_only_123_transformed"])
def test_device_demcz_matches_torch_bitwise(kind, per_well):
    """Tuning (every 4 steps), stop_tuning's history drop and the draws: device chains ==
    torch chains, bit for bit.  joint / bmm / epm / epm_piston / joint_transformed /
    epm_transformed / joint_c4_transformed run one launch per step (logp_fused_kernel forms the
    proposal, appends the history, decides and commits); ce_only: the generic kernels +
    demc_accept_kernel; bmm_transformed: the proposal kernel + the log-prob kernel pair.
    *_transformed: PyMC3's logodds / interval / log space, the plan adds the Jacobian.
    joint_c4_transformed: the c4 shape (64 wells, 8 walkers per block), 520 chains: the last
    block is partial.  *_123: savenum 123 (the per-unit CFC12 half-life in the single launch).  joint_l3: 3 wells, so a block holds 170 walkers (510 of its 512 unit
    slots) and the walker-major unit mapping of the multi-step launch leaves a ragged tail.
    per_well: every (walker, well) its own chain (the default; the per-unit decision inside
    the multi-step launch, or the per-unit proposal / log-prob / accept kernels) or one chain
    per walker."""
    import dataclasses
    import torch
    from noblegas_rtd_mcmc_amd import workloads as wl
    from noblegas_rtd_mcmc_amd.engine import LogProb
    from noblegas_rtd_mcmc_amd.sampler import DEMetropolisZ, DeviceDEMetropolisZ, Transform
    from noblegas_rtd_mcmc_amd.spec import ModelSpec
    spec = wl.c4_spec(L=4, N=300)
    if kind == "ce_only":
        spec = ModelSpec(n_wells=4, ce=spec.ce)
    if kind == "bmm_transformed":
        spec = wl.c4_spec(L=2, N=1200, mod_type1="exp_pist_flow", mod_type2="piston",
                          par_names=("tau1", "tau2", "f1", "eta1", "lamsf6"))
    if kind == "bmm":
        spec = wl.c4_spec(L=4, N=1200, mod_type1="exponential", mod_type2="piston", par_names=("tau1", "tau2", "f1"))
    if kind in ("epm", "epm_transformed"):
        spec = wl.c4_spec(L=4, N=1200, mod_type1="exp_pist_flow", par_names=("tau1", "eta1"))
    if kind == "epm_piston":
        spec = wl.c4_spec(L=4, N=1200, mod_type1="exp_pist_flow", mod_type2="piston",
                          par_names=("tau1", "tau2", "f1", "eta1"))
    if kind == "joint_c4_transformed":
        spec = wl.c4_spec(L=64, N=1200)
    if kind == "joint_l3":      # 3 wells: 170 walkers per block (510 units), not a power of two
        spec = wl.c4_spec(L=3, N=300)
    if kind in ("joint_123", "epm_123_transformed", "bmm_123", "rtd_only_123_transformed"):
        # savenum 123 (J, thalf_cfc, lamsf6 sampled): the single-launch LW instances
        m1 = "exp_pist_flow" if kind.startswith("epm") else "exponential"
        m2 = "piston" if kind.startswith("bmm") else None
        pn = ("tau1",) + (("tau2", "f1") if m2 else ()) + (("eta1",) if m1 == "exp_pist_flow" else ()) + \
            ("J", "thalf_cfc", "lamsf6")
        spec = wl.c4_spec(L=4, N=1200, mod_type1=m1, mod_type2=m2, par_names=pn)
        if kind.startswith("rtd_only"):
            keep = [0, 1, 2, 4]
            r = spec.rtd
            spec = ModelSpec(n_wells=4, rtd=dataclasses.replace(r, tracers=[r.tracers[i] for i in keep],
                                                                 obs=r.obs[:, keep], sd=r.sd[:, keep]))
    if kind.endswith("transformed"):
        spec = dataclasses.replace(spec, jacobian=True)
    W = 520 if kind == "joint_c4_transformed" else 200 if kind == "joint_l3" else 40
    th0 = wl.sample_prior(spec, W, np.random.default_rng(5))
    lp = LogProb(spec, max_walkers=W)
    x0 = torch.from_numpy(th0).cuda()
    kw = dict(tune_interval=4, seed=987654321)
    dev = DeviceDEMetropolisZ(lp, per_well=per_well, **kw).run(x0, tune=12, draws=8)
    tf = Transform.from_spec(spec) if spec.jacobian else None
    f = (lambda t: lp.units(t)) if per_well else (lambda t: lp(t))
    ref = DEMetropolisZ(f, transform=tf, per_well=per_well, **kw).run(x0, tune=12, draws=8)
    for k in ("x", "lp", "samples", "logp", "accepted", "accept", "lamb", "scaling"):
        assert _same(dev[k], ref[k]), k
    assert 0 < int(dev["accepted"].sum()) < dev["accepted"].numel()
    lp.close()


SHAPES = ["rtd4_exponential", "rtd4_exp_pist_flow", "rtd4_exponential-piston", "rtd4_exp_pist_flow-piston",
          "rtd4_exponential_123", "rtd4_exp_pist_flow_123", "rtd4_exponential-piston_123",
          "rtd4_exp_pist_flow-piston_123", "rtd1_exponential", "rtd1_exp_pist_flow", "ce_only", "joint_bmm",
          "joint_epm_bmm"]


def _shape_spec(shape, L=4, N=1200):
    """The reference's own model shapes: its RTD-only model over 4 tracers (CFC12, SF6, H3,
    He4_ter; run_age_mcmc.py) or 1 (H3), savenum 0 or 123, its CE-only model (Ne, Ar, Kr, Xe;
    noble_gas_mcmc.py), and the joint c4 BMMs; N ages of the input series (the reference's
    runs: 25 256)."""
    import dataclasses
    from noblegas_rtd_mcmc_amd import workloads as wl
    from noblegas_rtd_mcmc_amd.spec import ModelSpec
    if shape == "ce_only":
        base = wl.c4_spec(L=L, N=300)
        keep = [1, 2, 3, 4]
        c = base.ce
        return ModelSpec(n_wells=L, ce=dataclasses.replace(c, obs=c.obs[:, keep], sd=c.sd[:, keep],
                                                           gases=tuple(c.gases[i] for i in keep)))
    if shape.startswith("joint"):
        m1 = "exp_pist_flow" if "epm" in shape else "exponential"
        return wl.c4_spec(L=L, N=N, mod_type1=m1, mod_type2="piston",
                          par_names=("tau1", "tau2", "f1") + (("eta1",) if m1 == "exp_pist_flow" else ()))
    kind, model = shape.split("_", 1)
    sv = model.endswith("_123")
    model = model[:-4] if sv else model
    m1, _, m2 = model.partition("-")
    pn = ("tau1",) + (("tau2", "f1") if m2 else ()) + (("eta1",) if m1 == "exp_pist_flow" else ()) + \
        (("J", "thalf_cfc", "lamsf6") if sv else ())
    base = wl.c4_spec(L=L, N=N, mod_type1=m1, mod_type2=m2 or None, par_names=pn)
    keep = [0, 1, 2, 4] if kind == "rtd4" else [2]
    r = base.rtd
    return ModelSpec(n_wells=L, rtd=dataclasses.replace(r, tracers=[r.tracers[i] for i in keep], obs=r.obs[:, keep],
                                                        sd=r.sd[:, keep]))


@pytest.mark.parametrize("jac", [False, True])
@pytest.mark.parametrize("shape", SHAPES)
def test_single_launch_step_reference_shapes(shape, jac):
    """The reference's own sampled models run ONE launch per chunk of steps (the lane-chain
    dz_chain_kernel for the RTD-only and CE-only models; logp_fused_kernel's BMM instances in
    PyMC3's transformed space for the joint BMMs), per-well chains: device == torch
    (sampler.DEMetropolisZ over ngrtd_logp_units) bit for bit through tuning, stop_tuning and
    the draws, with walkers not a multiple of the block."""
    import dataclasses
    import torch
    from noblegas_rtd_mcmc_amd import workloads as wl
    from noblegas_rtd_mcmc_amd.engine import LogProb
    from noblegas_rtd_mcmc_amd.sampler import DEMetropolisZ, DeviceDEMetropolisZ, Transform
    spec = dataclasses.replace(_shape_spec(shape), jacobian=jac)
    W = 301
    x0 = torch.from_numpy(wl.sample_prior(spec, W, np.random.default_rng(17))).cuda()
    lp = LogProb(spec, max_walkers=W)
    kw = dict(tune_interval=4, seed=4242, per_well=True)
    lp.ctx.set_profiling(True)
    lp.kernel_stats(reset=True)
    dev = DeviceDEMetropolisZ(lp, **kw).run(x0, tune=12, draws=8)
    lp.ctx.set_profiling(False)
    ks = lp.kernel_stats(reset=True)
    assert ks["fused"][1] == 1, ks            # one launch for the 20 steps (a chunk of <= 256)
    tf = Transform.from_spec(spec) if jac else None
    ref = DEMetropolisZ(lambda t: lp.units(t), transform=tf, **kw).run(x0, tune=12, draws=8)
    for k in ("x", "lp", "samples", "logp", "accepted", "accept", "lamb", "scaling"):
        assert _same(dev[k], ref[k]), k
    assert 0 < int(dev["accepted"].sum()) < dev["accepted"].numel()
    lp.close()


@pytest.mark.parametrize("model", ["exponential", "exp_pist_flow"])
def test_lane_chain_launch_geometry_independent(model):
    """The lane-chain step launches only the waves its chains need (ngrtd_dzc.hip: 3 chains in one
    64-lane block, 70 in one 128-lane block, 600 in 512-lane blocks): a chain's draws do not
    depend on that geometry -- the first 3 chains of the 70- and 600-chain runs equal the 3-chain
    run bit for bit (1 well: a chain's random streams and history are keyed by its index alone)."""
    import dataclasses
    import torch
    from noblegas_rtd_mcmc_amd import workloads as wl
    from noblegas_rtd_mcmc_amd.engine import LogProb
    from noblegas_rtd_mcmc_amd.sampler import DeviceDEMetropolisZ
    spec = dataclasses.replace(wl.rtd_only_spec(L=1, N=1200, mod_type1=model), jacobian=True)
    x0 = torch.from_numpy(wl.sample_prior(spec, 600, np.random.default_rng(5))).cuda()
    kw = dict(tune_interval=4, seed=99, per_well=True)
    outs = {}
    for W in (3, 70, 600):
        lp = LogProb(spec, max_walkers=W)
        lp.ctx.set_profiling(True)
        lp.kernel_stats(reset=True)
        outs[W] = DeviceDEMetropolisZ(lp, **kw).run(x0[..., :W].contiguous(), tune=12, draws=8)
        assert lp.kernel_stats(reset=True)["fused"][1] == 1   # the lane-chain launch: one for the 20 steps
        lp.close()
    for W in (70, 600):
        for k in ("samples", "logp", "accepted", "lamb", "scaling"):
            assert _same(outs[W][k][..., :3], outs[3][k]), (W, k)
    assert 0 < int(outs[600]["accepted"].sum()) < outs[600]["accepted"].numel()


@pytest.mark.parametrize("jac", [True, False])
@pytest.mark.parametrize("shape", ["rtd4_exp_pist_flow_123", "rtd4_exp_pist_flow-piston_123", "rtd4_exp_pist_flow",
                                   "rtd1_exp_pist_flow", "joint_epm_bmm"])
def test_single_launch_step_full_series(shape, jac):
    """The reference's own exp_pist_flow runs at their series length N = 25 256 step in ONE
    launch (the lane-chain step for the RTD-only model, logp_fused_kernel's step for the joint
    BMM) on the windowed channel table (ngrtd.hip epm_window), 3 wells x 67 walkers: device ==
    torch (sampler.DEMetropolisZ over ngrtd_logp_units, itself the windowed single launch) bit
    for bit through tuning, stop_tuning and the draws."""
    import dataclasses
    import torch
    from noblegas_rtd_mcmc_amd import workloads as wl
    from noblegas_rtd_mcmc_amd.engine import LogProb
    from noblegas_rtd_mcmc_amd.sampler import DEMetropolisZ, DeviceDEMetropolisZ, Transform
    spec = dataclasses.replace(_shape_spec(shape, L=3, N=25256), jacobian=jac)
    W = 67
    x0 = torch.from_numpy(wl.sample_prior(spec, W, np.random.default_rng(29))).cuda()
    lp = LogProb(spec, max_walkers=W)
    kw = dict(tune_interval=4, seed=25256, per_well=True)
    lp.ctx.set_profiling(True)
    lp.kernel_stats(reset=True)
    dev = DeviceDEMetropolisZ(lp, **kw).run(x0, tune=12, draws=8)
    lp.ctx.set_profiling(False)
    ks = lp.kernel_stats(reset=True)
    assert ks["fused"][1] == 1 and ks["rtd"][1] == 0 and ks["unit"][1] == 0, ks
    tf = Transform.from_spec(spec) if jac else None
    ref = DEMetropolisZ(lambda t: lp.units(t), transform=tf, **kw).run(x0, tune=12, draws=8)
    for k in ("x", "lp", "samples", "logp", "accepted", "accept", "lamb", "scaling"):
        assert _same(dev[k], ref[k]), k
    assert 0 < int(dev["accepted"].sum()) < dev["accepted"].numel()
    lp.close()


@pytest.mark.parametrize("jac", [False, True])
@pytest.mark.parametrize("shape", ["rtd4_exponential", "rtd4_exponential_123", "rtd1_exponential"])
def test_lane_chain_step_exact_fallback(shape, jac):
    """The lane-chain step's exact matrix-core fallback (dzc_exact: its tiles read the tau rows
    of every lane of the wave from LDS): a tau1 prior U(0.05, 3) puts many proposals inside
    the prior but below the surrogate's reach (tau < 1/2), so waves take the fallback every
    step.  Device chains == torch chains bit for bit, one launch, and states below 1/2 are
    visited (their proposals went through the fallback)."""
    import dataclasses
    import torch
    from noblegas_rtd_mcmc_amd import workloads as wl
    from noblegas_rtd_mcmc_amd.engine import LogProb
    from noblegas_rtd_mcmc_amd.sampler import DEMetropolisZ, DeviceDEMetropolisZ, Transform
    base = _shape_spec(shape)
    spec = dataclasses.replace(base, rtd=dataclasses.replace(base.rtd, tau1=(0.05, 3.0)), jacobian=jac)
    W = 301
    x0 = torch.from_numpy(wl.sample_prior(spec, W, np.random.default_rng(23))).cuda()
    lp = LogProb(spec, max_walkers=W)
    kw = dict(tune_interval=4, seed=5151, per_well=True)
    lp.ctx.set_profiling(True)
    lp.kernel_stats(reset=True)
    dev = DeviceDEMetropolisZ(lp, **kw).run(x0, tune=12, draws=8)
    lp.ctx.set_profiling(False)
    ks = lp.kernel_stats(reset=True)
    assert ks["fused"][1] == 1, ks
    tf = Transform.from_spec(spec) if jac else None
    ref = DEMetropolisZ(lambda t: lp.units(t), transform=tf, **kw).run(x0, tune=12, draws=8)
    for k in ("x", "lp", "samples", "logp", "accepted", "accept", "lamb", "scaling"):
        assert _same(dev[k], ref[k]), k
    tau = dev["samples"][:, spec.roles.index("tau1")]
    assert int((tau < 0.5).sum()) > 0 and int((tau >= 0.5).sum()) > 0
    lp.close()


@pytest.mark.parametrize("per_well", [True, False])
@pytest.mark.parametrize("jac", [False, True])
def test_device_demcz_step_modes_bitwise(jac, per_well):
    """Every device step schedule gives the same chains bit for bit at the c4 shape (520
    chains: 65 walker blocks, the last partial): the multi-step launch (default: up to 256
    steps per launch, each block running its chains through them), one step per launch
    (NGRTD_DZ_CHUNK=1), chunks of 3 (launch boundaries between the tune steps and across
    stop_tuning's history drop at step 8) and the proposal kernel + log-prob kernel pair
    (NGRTD_DZ_MODE=pair)."""
    import dataclasses
    import os
    import torch
    from noblegas_rtd_mcmc_amd import workloads as wl
    from noblegas_rtd_mcmc_amd.engine import LogProb
    from noblegas_rtd_mcmc_amd.sampler import DeviceDEMetropolisZ
    spec = wl.c4_spec(L=64, N=1200)
    if jac:
        spec = dataclasses.replace(spec, jacobian=True)
    W = 520
    x0 = torch.from_numpy(wl.sample_prior(spec, W, np.random.default_rng(15))).cuda()
    lp = LogProb(spec, max_walkers=W)
    res = {}
    modes = {"fused": ("fused", "256"), "pair": ("pair", "256"), "chunk1": ("fused", "1"), "chunk3": ("fused", "3")}
    try:
        for mode, (m, ch) in modes.items():
            os.environ["NGRTD_DZ_MODE"] = m
            os.environ["NGRTD_DZ_CHUNK"] = ch
            res[mode] = DeviceDEMetropolisZ(lp, tune_interval=4, seed=99, per_well=per_well).run(x0, tune=8, draws=6)
    finally:
        for k in ("NGRTD_DZ_MODE", "NGRTD_DZ_CHUNK"):
            os.environ.pop(k, None)
    for mode in ("pair", "chunk1", "chunk3"):
        for k in ("x", "lp", "samples", "logp", "accepted", "accept", "lamb", "scaling"):
            assert _same(res[mode][k], res["fused"][k]), (mode, k)
    if jac:
        assert 0 < int(res["fused"]["accepted"].sum()) < res["fused"]["accepted"].numel()
    lp.close()


def test_device_demcz_many_blocks_chunks_bitwise():
    """More walker blocks than CUs (8200 chains at the c4 shape: 1025 blocks, the last
    partial; W not a multiple of the 32-wide layout tiles): the multi-step launch (one chunk)
    equals one step per launch bit for bit, and the caller's [P][L][W] state comes back in
    its own layout (the walker-major scratch copy is transposed in and out)."""
    import os
    import torch
    from noblegas_rtd_mcmc_amd import workloads as wl
    from noblegas_rtd_mcmc_amd.engine import LogProb
    from noblegas_rtd_mcmc_amd.sampler import DeviceDEMetropolisZ
    spec = wl.c4_spec(L=64, N=1200)
    W = 8200
    x0 = torch.from_numpy(wl.sample_prior(spec, W, np.random.default_rng(21))).cuda()
    lp = LogProb(spec, max_walkers=W)
    res = {}
    try:
        for ch in ("256", "1"):
            os.environ["NGRTD_DZ_CHUNK"] = ch
            res[ch] = DeviceDEMetropolisZ(lp, tune_interval=3, seed=5).run(x0, tune=4, draws=3)
    finally:
        os.environ.pop("NGRTD_DZ_CHUNK", None)
    for k in ("x", "lp", "samples", "logp", "accepted", "accept", "lamb", "scaling"):
        assert _same(res["256"][k], res["1"][k]), k
    # the final state is the last draw, in the caller's layout
    assert _same(res["256"]["x"], res["256"]["samples"][-1])
    # the log-prob of the returned state is the chains' current log-prob
    assert _same(lp.units(res["256"]["x"].contiguous()), res["256"]["lp"])   # per-well chains: [L][W]
    lp.close()


def test_device_demcz_split_calls_and_shard_offsets():
    """A run split over two calls equals one call; a walker block with chain0 / the
    ensemble size equals the same chains of the whole-ensemble run."""
    import torch
    from noblegas_rtd_mcmc_amd import workloads as wl
    from noblegas_rtd_mcmc_amd.engine import LogProb
    from noblegas_rtd_mcmc_amd.sampler import DeviceDEMetropolisZ
    spec = wl.c4_spec(L=2, N=300)
    W = 64
    th0 = torch.from_numpy(wl.sample_prior(spec, W, np.random.default_rng(9))).cuda()
    lp = LogProb(spec, max_walkers=W)
    s = DeviceDEMetropolisZ(lp, tune_interval=5, seed=11, per_well=False)
    x, l, z = s.start(th0, 10, 20)
    lp.demcz(x, l, 20, z)
    x2, l2, z2 = s.start(th0, 10, 20)
    lp.demcz(x2, l2, 7, z2)
    lp.demcz(x2, l2, 13, z2)
    assert torch.equal(x, x2) and torch.equal(l, l2) and torch.equal(z.hist, z2.hist)
    assert z.c.hist_len == 20 and z.c.steps_done == 20 and z.c.hist_lo == 9
    # shard [24, 64) of the same ensemble
    lpb = LogProb(spec, max_walkers=W)
    sb = DeviceDEMetropolisZ(lpb, tune_interval=5, seed=11, chain0=24, n_chains_total=W, per_well=False)
    xb, lb, zb = sb.start(th0[..., 24:].contiguous(), 10, 20)
    lpb.demcz(xb, lb, 20, zb)
    assert torch.equal(xb, x[..., 24:]) and torch.equal(lb, l[24:])
    with pytest.raises(Exception):          # the history is full
        lp.demcz(x, l, 1, z)
    lp.close()
    lpb.close()


def test_per_well_run_equals_single_well_runs():
    """Per-well chains: a run of all L wells equals L independent runs of one well each
    (ModelSpec.well(l), well0 = l), chain for chain and bit for bit -- the reference's
    structure, one PyMC3 model per well (run_age_mcmc.py:122-231).  Also for a walker-block
    shard (chain0) of the L-well run, and through the pair schedule."""
    import dataclasses
    import os
    import torch
    from noblegas_rtd_mcmc_amd import workloads as wl
    from noblegas_rtd_mcmc_amd.engine import LogProb
    from noblegas_rtd_mcmc_amd.sampler import DeviceDEMetropolisZ
    L, W = 5, 96
    spec = dataclasses.replace(wl.c4_spec(L=L, N=1200), jacobian=True)
    x0 = torch.from_numpy(wl.sample_prior(spec, W, np.random.default_rng(31))).cuda()
    kw = dict(tune_interval=4, seed=77)
    lp = LogProb(spec, max_walkers=W)
    full = DeviceDEMetropolisZ(lp, **kw).run(x0, tune=10, draws=6)
    assert tuple(full["logp"].shape) == (6, L, W) and tuple(full["lamb"].shape) == (L, W)
    for l in range(L):
        lpl = LogProb(spec.well(l), max_walkers=W)
        one = DeviceDEMetropolisZ(lpl, well0=l, n_wells_total=L, **kw).run(x0[:, l:l + 1].contiguous(), tune=10,
                                                                           draws=6)
        assert torch.equal(one["x"][:, 0], full["x"][:, l]), l
        assert torch.equal(one["samples"][:, :, 0], full["samples"][:, :, l]), l
        for k in ("logp", "accepted", "accept", "lp", "lamb", "scaling"):
            assert torch.equal(one[k][..., 0, :] if one[k].dim() > 1 else one[k], full[k][..., l, :]), (l, k)
        if l == L - 1:      # a well range past the run's wells is refused (streams would collide)
            with pytest.raises(Exception, match="outside the run"):
                DeviceDEMetropolisZ(lpl, well0=L, n_wells_total=L, **kw).run(x0[:, l:l + 1].contiguous(), 2, 1)
        lpl.close()
    # a walker-block shard of the L-well run
    lpb = LogProb(spec, max_walkers=W)
    sh = DeviceDEMetropolisZ(lpb, chain0=40, n_chains_total=W, **kw).run(x0[..., 40:].contiguous(), tune=10, draws=6)
    assert torch.equal(sh["samples"], full["samples"][..., 40:]) and torch.equal(sh["logp"], full["logp"][..., 40:])
    # the proposal / per-unit log-prob / accept kernels give the same chains
    os.environ["NGRTD_DZ_MODE"] = "pair"
    try:
        pair = DeviceDEMetropolisZ(lp, **kw).run(x0, tune=10, draws=6)
    finally:
        os.environ.pop("NGRTD_DZ_MODE", None)
    for k in ("x", "lp", "samples", "logp", "accepted", "accept", "lamb", "scaling"):
        assert _same(pair[k], full[k]), k
    assert 0 < int(full["accepted"].sum()) < full["accepted"].numel()
    lp.close()
    lpb.close()


@pytest.mark.parametrize("L", [1, 3, 5, 7, 48, 100, 300])
def test_ragged_walker_major_sweep(L):
    """The multi-step launch's walker-major unit mapping over ragged blocks (WB = 512 // L
    walkers per block, WB L < 512 unit slots used; W not a multiple of WB): device == torch
    bit for bit for W in {1, 63, 65, 1025}, per-well chains in PyMC3's transformed space
    and one chain per walker in the natural space -- the class of bug da34ef9 fixed (L = 3)."""
    import dataclasses
    import torch
    from noblegas_rtd_mcmc_amd import workloads as wl
    from noblegas_rtd_mcmc_amd.engine import LogProb
    from noblegas_rtd_mcmc_amd.sampler import DEMetropolisZ, DeviceDEMetropolisZ, Transform
    base = wl.c4_spec(L=L, N=300)
    for per_well, jac in ((True, True), (False, False)):
        spec = dataclasses.replace(base, jacobian=jac)
        lp = LogProb(spec, max_walkers=1025)
        tf = Transform.from_spec(spec) if jac else None
        f = (lambda t: lp.units(t)) if per_well else (lambda t: lp(t))
        for W in (1, 63, 65, 1025):
            x0 = torch.from_numpy(wl.sample_prior(spec, W, np.random.default_rng(L * 1000 + W))).cuda()
            kw = dict(tune_interval=3, seed=L + W, per_well=per_well)
            dev = DeviceDEMetropolisZ(lp, **kw).run(x0, tune=6, draws=4)
            ref = DEMetropolisZ(f, transform=tf, **kw).run(x0, tune=6, draws=4)
            for k in ("x", "lp", "samples", "logp", "accepted", "accept", "lamb", "scaling"):
                assert _same(dev[k], ref[k]), (L, W, per_well, k)
        lp.close()


def test_prior_only_recovers_analytic_moments():
    """include_like=False: the stationary distribution of the chains must be the priors
    (Beta, Normal, Uniform).  4096 chains start from exact prior draws and run PyMC3's
    defaults (transformed space, lambda tuning every 100 steps, 90 % history drop) for
    1000 + 6000 steps; their final states are independent draws, so their means and
    variances must sit within 4 Monte-Carlo standard errors of the analytic values.
    (DE-MC-Z's proposals depend on each chain's own recent past, so the kernel is only
    asymptotically invariant: on CPU, 8-D Gaussians showed a -4 SE variance bias after
    1500 draws that fades to ~-1.5 SE by 6000; hence the long draw phase.)"""
    import dataclasses
    import torch
    from scipy import stats
    from noblegas_rtd_mcmc_amd import workloads as wl
    from noblegas_rtd_mcmc_amd.engine import LogProb
    from noblegas_rtd_mcmc_amd.sampler import DeviceDEMetropolisZ
    from noblegas_rtd_mcmc_amd.spec import ModelSpec
    base = wl.c4_spec(L=1, N=300)
    spec = ModelSpec(n_wells=1, ce=base.ce, rtd=base.rtd, include_like=False)
    W = 4096
    c, r = spec.ce, spec.rtd
    dists = {}
    for role in spec.roles:
        if role == "m":
            dists[role] = stats.norm(c.m_mu, c.m_sd)
        elif role == "tau1":
            dists[role] = stats.uniform(r.tau1[0], r.tau1[1] - r.tau1[0])
        else:
            dists[role] = stats.beta(*{"Ae_beta": c.beta_Ae, "F_beta": c.beta_F, "E_beta": c.beta_E,
                                       "b_beta": c.beta_b, "nu_ce_beta": c.beta_nu, "nu_rtd_beta": r.beta_nu}[role])
    th = wl.sample_prior(spec, W, np.random.default_rng(22))
    lp = LogProb(dataclasses.replace(spec, jacobian=True), max_walkers=W)
    res = DeviceDEMetropolisZ(lp, tune_interval=100, seed=5).run(torch.from_numpy(th).cuda(), tune=1000, draws=6000)
    fin = res["x"].cpu().numpy()[:, 0, :]
    for i, role in enumerate(spec.roles):
        d = dists[role]
        mu, var, _, kurt = (float(v) for v in d.stats(moments="mvsk"))
        se_m = np.sqrt(var / W)
        se_v = np.sqrt((kurt + 2.0) * var ** 2 / W)
        assert abs(fin[i].mean() - mu) < 4 * se_m, (role, fin[i].mean(), mu, se_m)
        assert abs(fin[i].var() - var) < 4 * se_v, (role, fin[i].var(), var, se_v)
    assert 0.01 < res["accept_rate"] < 0.95
    lp.close()


def test_demcz_invariants_c4():
    """lamb = scaling = 0: every proposal is the current state (mr = 0 is accepted) and
    nothing moves; after a real run the tracked logp equals a fresh evaluation."""
    import torch
    from noblegas_rtd_mcmc_amd import workloads as wl
    from noblegas_rtd_mcmc_amd.engine import LogProb
    from noblegas_rtd_mcmc_amd.sampler import DeviceDEMetropolisZ
    spec = wl.c4_spec(L=8, N=1200)
    W = 256
    th0 = torch.from_numpy(wl.sample_prior(spec, W, np.random.default_rng(6))).cuda()
    lp = LogProb(spec, max_walkers=W)
    x, l, z = DeviceDEMetropolisZ(lp, lamb=0.0, scaling=0.0, tune=None, seed=1, per_well=False).start(th0, 0, 8)
    l0 = l.clone()
    cnt = torch.zeros(1, dtype=torch.int64, device="cuda")
    lp.demcz(x, l, 4, z, n_accepted=cnt)
    assert torch.equal(x, th0) and torch.equal(l, l0) and int(cnt.item()) == 4 * W
    # a real run in PyMC3's transformed space (natural-space noise pushes the prior draws of
    # the Beta(2, 0.1) nu rows, which sit at ~1 - 1e-9, out of [0, 1]: nothing is accepted)
    import dataclasses
    lpj = LogProb(dataclasses.replace(spec, jacobian=True), max_walkers=W)
    x, l, z = DeviceDEMetropolisZ(lpj, tune_interval=5, seed=2, per_well=False).start(th0, 10, 30)
    cnt.zero_()
    lpj.demcz(x, l, 30, z, n_accepted=cnt)
    assert torch.equal(l, lpj(x))
    assert 0 < int(cnt.item()) < 30 * W
    # per-well chains: the tracked per-unit log-probs equal a fresh ngrtd_logp_units
    x, l, z = DeviceDEMetropolisZ(lpj, tune_interval=5, seed=2).start(th0, 10, 30)
    cnt.zero_()
    alog = torch.zeros((30, 8 * W), dtype=torch.uint8, device="cuda")
    lpj.demcz(x, l, 30, z, accepted_log=alog, n_accepted=cnt)
    assert torch.equal(l, lpj.units(x)) and tuple(l.shape) == (8, W)
    # the per-block accept count (one atomic per block and step) equals the decisions logged
    assert 0 < int(cnt.item()) < 30 * W * 8 and int(cnt.item()) == int(alog.sum())
    lp.close()
    lpj.close()


def test_c1_torch_sampler_path():
    """The torch-op DEMetropolisZ path stays available (sampler="torch")."""
    from noblegas_rtd_mcmc_amd.noble_gas_mcmc import CEModel
    from noblegas_rtd_mcmc_amd.workloads import field_data
    m = CEModel(field_data()["obs"], ["PLM1"], max_walkers=64)
    res = m.sample(nwalkers=32, tune=40, draws=20, seed=3, tune_interval=20, sampler="torch")
    assert res["samples"].shape[0] == 20 and 0.0 < res["accept_rate"] < 1.0


def _ulp_dist(a, b):
    """|a - b| in units of the last place of b (float64 tensors, finite entries)."""
    import torch
    sp = torch.nextafter(b.abs(), torch.full_like(b, float("inf"))) - b.abs()
    return ((a - b).abs() / sp)


def test_fm_log_matches_torch_log():
    """ngrtd_fm_log (the accept draw's table-driven log, sampler.fm_log on CUDA tensors)
    against torch.log on the CPU: <= 1 ulp on random, tiny, huge, near-1 and subnormal
    inputs, and the IEEE specials (0 -> -inf, inf -> inf, x < 0 and NaN -> NaN) exactly;
    a non-float64 tensor is refused."""
    import torch
    from noblegas_rtd_mcmc_amd.sampler import fm_log
    rng = np.random.default_rng(11)
    x = np.concatenate([rng.uniform(0, 1, 4096), 10 ** rng.uniform(-300, 300, 4096), 1 + rng.uniform(-1e-3, 1e-3, 1024),
                        [1.0, 2.0, 0.5, np.nextafter(1.0, 2.0), np.nextafter(1.0, 0.0), 5e-324, 2.2e-308, 1.7e308,
                         1.1102230246251565e-16]])
    got = fm_log(torch.from_numpy(x).cuda()).cpu()
    ref = torch.log(torch.from_numpy(x))
    ok = ref != 0
    assert float(_ulp_dist(got[ok], ref[ok]).max()) <= 1.0
    assert float(got[~ok].abs().max()) == 0.0
    sp = torch.tensor([0.0, -0.0, float("inf"), -1.0, float("nan")], dtype=torch.float64)
    gs = fm_log(sp.cuda()).cpu()
    assert gs[0] == -float("inf") and gs[1] == -float("inf") and gs[2] == float("inf")
    assert torch.isnan(gs[3]) and torch.isnan(gs[4])
    with pytest.raises(TypeError):
        fm_log(torch.ones(4, dtype=torch.float32, device="cuda"))


def test_pymc3_backward_matches_torch_backward():
    """ngrtd_pymc3_backward (the device step's backward transform, Transform.backward on CUDA
    tensors) against the same transform in torch on the CPU (torch.exp): logodds, interval
    and log rows within 2 / 4 / 1 ulp over random u and the edges (0, +-1, +-inf, NaN, |u| up to 800,
    where exp over- and underflows); identity rows bitwise; a non-float64 tensor is refused."""
    import torch
    from noblegas_rtd_mcmc_amd.sampler import Transform
    tf = Transform([Transform.LOGODDS, Transform.INTERVAL, Transform.LOG, Transform.NONE, Transform.INTERVAL],
                   [0.0, 1.0, 0.0, 0.0, 50.0], [0.0, 1000.0, 0.0, 0.0, 15000.0], L=3)
    rng = np.random.default_rng(12)
    W = 4000
    u = rng.normal(0, 4, (5, 3, W))
    u[:, :, :8] = np.array([0.0, 1.0, -1.0, 40.0, -40.0, 700.0, -745.5, 800.0])[None, None, :]
    u[:, :, 8:24] = 10 ** rng.uniform(-300, 2.9, 16) * rng.choice([-1, 1], 16)
    u[:, 0, 24:27] = [np.inf, -np.inf, np.nan]
    ut = torch.from_numpy(u)
    got = tf.backward(ut.cuda()).cpu()
    ref = tf.backward(ut)
    both_nan = torch.isnan(got) & torch.isnan(ref)
    assert bool((both_nan | ~torch.isnan(ref)).all()) and bool((both_nan | ~torch.isnan(got)).all())
    fin = torch.isfinite(ref) & (ref != 0)
    # exp <= 1 ulp; logodds 1 / (1 + e) adds an add and a division; interval s b + (1 - s) a two more
    for row, bound in ((0, 2.0), (1, 4.0), (2, 1.0), (4, 4.0)):
        f = fin[row]
        assert float(_ulp_dist(got[row][f], ref[row][f]).max()) <= bound, row
    same_special = ~fin & ~both_nan
    assert torch.equal(got[same_special], ref[same_special])
    assert _same(got[3], ut[3])
    with pytest.raises(TypeError):
        tf.backward(ut.float().cuda())


GENERIC_PAIRS = [("dispersion", None, ("tau1", "D1")), ("exponential", "exponential", ("tau1", "tau2", "f1")),
                 ("piston", "exponential", ("tau1", "tau2", "f1")), ("dispersion", "piston", ("tau1", "tau2", "f1", "D1")),
                 ("exponential", "dispersion", ("tau1", "tau2", "f1", "D2")),
                 ("exp_pist_flow", "exponential", ("tau1", "tau2", "f1", "eta1"))]


@pytest.mark.parametrize("per_well", [True, False])
@pytest.mark.parametrize("jac", [False, True])
@pytest.mark.parametrize("pair", GENERIC_PAIRS, ids=lambda p: p[0] + ("-" + p[1] if p[1] else ""))
def test_single_launch_step_generic_pairs(pair, jac, per_well):
    """The model pairs of run_age_mcmc.py:61-70 without a specialised instance (dispersion, a
    piston first component, exponential / dispersion seconds, exp_pist_flow-exponential) step in
    ONE launch per chunk on the generic DZ instances (MIX 64 | 8, + 128 for dispersion), on the
    joint c4 shape (5 tracers, 4 wells, 130 walkers: a partial second block): device == torch
    (sampler.DEMetropolisZ over the parity-tested log-prob) bit for bit through tuning,
    stop_tuning and the draws."""
    import dataclasses
    import torch
    from noblegas_rtd_mcmc_amd import workloads as wl
    from noblegas_rtd_mcmc_amd.engine import LogProb
    from noblegas_rtd_mcmc_amd.sampler import DEMetropolisZ, DeviceDEMetropolisZ, Transform
    m1, m2, pn = pair
    spec = dataclasses.replace(wl.c4_spec(L=4, N=1200, mod_type1=m1, mod_type2=m2, par_names=pn), jacobian=jac)
    W = 130
    x0 = torch.from_numpy(wl.sample_prior(spec, W, np.random.default_rng(31))).cuda()
    lp = LogProb(spec, max_walkers=W)
    kw = dict(tune_interval=4, seed=6170, per_well=per_well)
    lp.ctx.set_profiling(True)
    lp.kernel_stats(reset=True)
    dev = DeviceDEMetropolisZ(lp, **kw).run(x0, tune=12, draws=8)
    lp.ctx.set_profiling(False)
    ks = lp.kernel_stats(reset=True)
    # one launch for the 20 steps (+ the start's log-prob launch of the walker chains, lp(x))
    assert ks["fused"][1] == (1 if per_well else 2) and ks["rtd"][1] == 0 and ks["unit"][1] == 0, ks
    tf = Transform.from_spec(spec) if jac else None
    f = (lambda t: lp.units(t)) if per_well else (lambda t: lp(t))
    ref = DEMetropolisZ(f, transform=tf, **kw).run(x0, tune=12, draws=8)
    for k in ("x", "lp", "samples", "logp", "accepted", "accept", "lamb", "scaling"):
        assert _same(dev[k], ref[k]), k
    assert 0 < int(dev["accepted"].sum()) < dev["accepted"].numel()
    lp.close()
