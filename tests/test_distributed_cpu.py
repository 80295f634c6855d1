"""world_size-2 gloo tests of the walker-block sharding + all-gather path (c5) on CPU.
Each rank evaluates its block with the CPU oracle (test-side evaluator)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _spec():
    from noblegas_rtd_mcmc_amd import workloads as wl
    return wl.c4_spec(L=2, N=120)


def _oracle_eval(spec, per_well=False):
    import oracle.models as om

    def f(theta_block):
        return torch.from_numpy(om.log_prob(spec, theta_block.numpy()))

    def fu(theta_block):
        return torch.from_numpy(om.log_prob_units(spec, theta_block.numpy()))
    return fu if per_well else f


def _worker(rank, world, port, W, outdir, per_well=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from noblegas_rtd_mcmc_amd import workloads as wl
        from noblegas_rtd_mcmc_amd.distributed import ShardedLogProb, sharded_demcz
        spec = _spec()
        full = torch.from_numpy(wl.sample_prior(spec, W, np.random.default_rng(5)))
        sh = ShardedLogProb(_oracle_eval(spec), W)
        blk = sh.block(full)
        lp_b, lp_full = sh(blk)
        pos = sh.gather_positions(blk)
        res, lp_tr, acc_tr = sharded_demcz(_oracle_eval(spec, per_well), blk, W, tune=6, draws=4, seed=3,
                                           tune_interval=2, per_well=per_well)
        np.savez(os.path.join(outdir, "r%d.npz" % rank), lp_full=lp_full.numpy(), pos=pos.numpy(),
                 lp_tr=lp_tr.numpy(), acc_tr=acc_tr.numpy(), x=res["x"].numpy(), lp=res["lp"].numpy(),
                 samples=res["samples"].numpy(), lo=sh.lo, hi=sh.hi)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("W,per_well", [(9, False), (16, False), (9, True)])
def test_walker_block_allgather_matches_single_process(tmp_path, W, per_well):
    """Sharded DEMetropolisZ: the union of the two ranks' chains is bitwise the
    single-process run of the whole ensemble (chains draw the random numbers of their
    global index), and the gathered trace log-probs are the same on both ranks.  per_well:
    every (walker, well) its own chain, per-unit log-probs [L][W] (oracle.log_prob_units)."""
    import oracle.models as om
    from noblegas_rtd_mcmc_amd import workloads as wl
    from noblegas_rtd_mcmc_amd.sampler import DEMetropolisZ
    port = _free_port()
    mp.start_processes(_worker, args=(2, port, W, str(tmp_path), per_well), nprocs=2, start_method="spawn")
    r0, r1 = (np.load(tmp_path / ("r%d.npz" % r)) for r in (0, 1))
    spec = _spec()
    full = wl.sample_prior(spec, W, np.random.default_rng(5))
    ref = om.log_prob(spec, full)
    assert np.allclose(r0["lp_full"], ref, rtol=1e-13) and np.array_equal(r0["lp_full"], r1["lp_full"])
    assert np.array_equal(r0["pos"], full) and np.array_equal(r1["pos"], full)
    # blocks tile the ensemble
    assert int(r0["lo"]) == 0 and int(r0["hi"]) == int(r1["lo"]) and int(r1["hi"]) == W
    one = DEMetropolisZ(_oracle_eval(spec, per_well), seed=3, tune_interval=2,
                        per_well=per_well).run(torch.from_numpy(full), tune=6, draws=4)
    assert np.array_equal(np.concatenate([r0["x"], r1["x"]], axis=-1), one["x"].numpy())
    assert np.array_equal(np.concatenate([r0["samples"], r1["samples"]], axis=-1), one["samples"].numpy())
    assert np.array_equal(r0["lp_tr"], one["logp"].numpy()) and np.array_equal(r1["lp_tr"], one["logp"].numpy())
    assert np.array_equal(r0["acc_tr"], one["accepted"].numpy())
    # the final chain log-probs are consistent with the positions
    f = om.log_prob_units if per_well else om.log_prob
    assert np.allclose(f(spec, r1["x"]), r1["lp"], rtol=1e-13)


def test_shard_walkers_partition():
    from noblegas_rtd_mcmc_amd.workloads import shard_walkers
    for W in (1, 7, 2048, 2049):
        for G in (1, 2, 3, 8):
            spans = [shard_walkers(W, r, G) for r in range(G)]
            assert spans[0][0] == 0 and spans[-1][1] == W
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))


def _step_loop_worker(rank, world, port, W_total, outdir):
    """bench.py's per-step function (distributed.LogpStepLoop) on gloo: each rank's block
    of ONE seeded ensemble, evaluated into the padded block buffer, then one all-gather."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle.models as om
        from noblegas_rtd_mcmc_amd import workloads as wl
        from noblegas_rtd_mcmc_amd.distributed import LogpStepLoop
        spec = _spec()
        full = wl.sample_prior(spec, W_total, np.random.default_rng(34568))
        loop = LogpStepLoop(None, W_total, "cpu")
        blk = np.ascontiguousarray(full[:, :, loop.lo:loop.hi])

        def evaluate(out):
            out.copy_(torch.from_numpy(om.log_prob(spec, blk)))
        loop.evaluate = evaluate
        g1 = loop.step().clone()
        g2 = loop.step().clone()
        loop.evaluate_n = lambda out, k: (_ for _ in ()).throw(AssertionError("world > 1 must gather per step"))
        assert torch.equal(loop.run(2).nan_to_num(), g1.nan_to_num())   # (padding is NaN)
        # run()'s two-deep pipeline (CPU tensors on gloo: async all-gathers, not host-staged):
        # the block buffers alternate, every step evaluates and gathers, the hook brackets each
        # evaluation, and the latest gathered vector is the ensemble's
        seen, hooks = [], []
        loop.evaluate = lambda out: seen.append(out.data_ptr()) or evaluate(out)
        last = loop.run(5, hook=lambda i, before: hooks.append((i, before)))
        assert seen == [loop.outs[i % 2].data_ptr() for i in range(5)] and loop.outs[0].data_ptr() != loop.outs[1].data_ptr()
        assert hooks == [(i, b) for i in range(5) for b in (True, False)]
        assert last is loop.gathers[0] and torch.equal(loop.gathers[1].nan_to_num(), g1.nan_to_num())
        assert torch.equal(last.nan_to_num(), g1.nan_to_num())
        # gather="region" (bench.py's default for N > 1): k evaluations -- ONE evaluate_n call --
        # then one all-gather, into gathers[0]
        calls = []
        rl = LogpStepLoop(evaluate, W_total, "cpu", gather="region",
                          evaluate_n=lambda out, k: calls.append(k) or evaluate(out))
        got = rl.run(6)
        assert calls == [6] and got is rl.gathers[0] and torch.equal(got.nan_to_num(), g1.nan_to_num())
        assert torch.equal(rl.ensemble(), loop.ensemble())
        np.savez(os.path.join(outdir, "s%d.npz" % rank), ens=loop.ensemble().numpy(), g1=g1.numpy(),
                 g2=g2.numpy(), lo=loop.lo, hi=loop.hi, per=loop.per)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("W_total", [9, 16])
def test_bench_step_loop_gloo(tmp_path, W_total):
    """Strong (one ensemble split over the ranks, uneven when W is odd) and weak (W per
    rank: W_total = 2 W) sharding both run this function; the gathered ensemble vector on
    every rank equals the single-process log-prob of the whole ensemble."""
    import oracle.models as om
    from noblegas_rtd_mcmc_amd import workloads as wl
    port = _free_port()
    mp.start_processes(_step_loop_worker, args=(2, port, W_total, str(tmp_path)), nprocs=2, start_method="spawn")
    r0, r1 = (np.load(tmp_path / ("s%d.npz" % r)) for r in (0, 1))
    spec = _spec()
    ref = om.log_prob(spec, wl.sample_prior(spec, W_total, np.random.default_rng(34568)))
    assert np.array_equal(r0["ens"], ref) and np.array_equal(r1["ens"], ref)
    assert np.array_equal(r0["g1"], r1["g1"], equal_nan=True) and np.array_equal(r0["g1"], r0["g2"], equal_nan=True)
    assert int(r0["hi"]) == int(r1["lo"]) and int(r1["hi"]) == W_total
    if W_total % 2:                      # the short last block is NaN-padded in the gather
        assert np.isnan(r0["g1"][-1])


def test_step_loop_run_world1_single_call():
    """World 1 with evaluate_n: run(k) makes ONE evaluate_n(out, k) call (bench.py N = 1:
    one ngrtd_logp_n call enqueues the K launches); without it, k step()s."""
    from noblegas_rtd_mcmc_amd.distributed import LogpStepLoop
    calls = []
    loop = LogpStepLoop(lambda out: calls.append(("step", 1)) or out.fill_(1.0), 5, "cpu",
                        evaluate_n=lambda out, k: calls.append(("n", k)) or out.fill_(2.0))
    assert torch.equal(loop.run(7), torch.full((5,), 2.0, dtype=torch.float64)) and calls == [("n", 7)]
    loop.evaluate_n = None
    calls.clear()
    loop.run(3)
    assert calls == [("step", 1)] * 3
