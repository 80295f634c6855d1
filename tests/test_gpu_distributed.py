"""c5 on the GPU: the sharded path with the real HIP kernels and two ranks.

The test box has one MI355X, so both ranks run on cuda:0 over gloo (RCCL refuses two ranks
on one device; the all-gathers go through host memory).  The ranks are separate processes
started by torch.distributed.run as children of this one (never an exec of a process that
touched the GPU).  Checked bitwise against one process evaluating / sampling the whole
ensemble: the gathered log-prob vector (bench.py's LogpStepLoop) and the union of the
ranks' device DEMetropolisZ chains (sharded_demcz(device_sampler=True)).  Then bench.py's
own N > 1 branch runs the same way (--backend gloo --one-device)."""
import dataclasses
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _torchrun(args, timeout=300, nproc=2):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
           "--master-addr", "127.0.0.1", "--master-port", str(_port())] + args
    env = dict(os.environ, OMP_NUM_THREADS=str(max(1, 8 // nproc)))
    return subprocess.run(cmd, check=True, timeout=timeout, env=env, capture_output=True, text=True, cwd=REPO)


@pytest.mark.parametrize("W,L,per_well,nproc", [(2048, 64, 1, 2), (2048, 64, 0, 2), (130, 3, 1, 2),
                                                 (2048, 64, 1, 8)])
def test_ranks_on_gpu_equal_one_process(tmp_path, W, L, per_well, nproc):
    """Strong sharding of one seeded ensemble (c5's partition at N = 2, and c5's exact
    partition: 8 ranks x 256 walkers x 64 wells; W = 130 at L = 3: ragged walker-major
    blocks): the gathered ensemble log-prob == the single-process log-prob, and the ranks'
    device DEMetropolisZ chains == the same chains of the single-process device run, bit for
    bit.  All ranks share the box's one GPU (gloo, host-staged all-gathers)."""
    import torch
    from noblegas_rtd_mcmc_amd import workloads as wl
    from noblegas_rtd_mcmc_amd.engine import LogProb
    from noblegas_rtd_mcmc_amd.sampler import DeviceDEMetropolisZ
    _torchrun([os.path.join(REPO, "tests", "dist_gpu_worker.py"), str(tmp_path), str(W), str(L), str(per_well)],
              nproc=nproc)
    rs = [np.load(tmp_path / ("rank%d.npz" % r)) for r in range(nproc)]
    spec = wl.c4_spec(L=L, N=1200)
    full = torch.from_numpy(wl.sample_prior(spec, W, np.random.default_rng(34568))).cuda()
    lp = LogProb(spec, max_walkers=W)
    ref = lp(full).cpu().numpy()
    assert int(rs[0]["lo"]) == 0 and int(rs[-1]["hi"]) == W
    assert all(int(a["hi"]) == int(b["lo"]) for a, b in zip(rs, rs[1:]))
    for r in rs:
        assert np.array_equal(r["ens"], ref, equal_nan=True)
        assert np.array_equal(r["g1"], r["g2"], equal_nan=True)
    kw = dict(tune_interval=4, seed=2024)
    kw["per_well"] = bool(per_well)
    lpj = LogProb(dataclasses.replace(spec, jacobian=True), max_walkers=W)
    one = DeviceDEMetropolisZ(lpj, **kw).run(full, tune=8, draws=6)
    cat = lambda k: np.concatenate([r[k] for r in rs], axis=-1)   # noqa: E731
    assert np.array_equal(cat("x"), one["x"].cpu().numpy())
    assert np.array_equal(cat("lp"), one["lp"].cpu().numpy())
    assert np.array_equal(cat("samples"), one["samples"].cpu().numpy())
    for r in rs:
        assert np.array_equal(r["lp_tr"], one["logp"].cpu().numpy())
        assert np.array_equal(r["acc_tr"], one["accepted"].cpu().numpy())
    assert 0 < int(one["accepted"].sum()) < one["accepted"].numel()
    lp.close()
    lpj.close()


@pytest.mark.parametrize("nproc", [2, 8])
def test_bench_ranks_one_gpu(nproc, tmp_path):
    """bench.py's N > 1 branch (LogpStepLoop + all-gather, max-over-ranks timing, the
    sampler leg on every rank) end to end on the one GPU: a valid JSON line; nproc = 8 is
    c5's strong partition (8 x 256 walkers of the 2048-walker ensemble)."""
    r = _torchrun(["bench.py", "--gpus", str(nproc), "--steps", "10", "--warmup", "2", "--scaling", "strong",
                   "--backend", "gloo", "--one-device", "--sampler-steps", "16", "--no-cpu-baseline",
                   "--side-out", str(tmp_path / "side.json")], nproc=nproc)
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:] + r.stderr[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == nproc and d["value"] > 0 and d["config"]["walkers_per_gpu"] == 2048 // nproc
    assert d["config"]["one_device"] is True and d["ensemble_finite_frac"] > 0.5
    assert len(lines[0]) < 8000 and "sampler_error" not in d["side"] and d["side"]["sampler"]["transformed"][0] > 0
    full = json.load(open(tmp_path / "side.json"))     # the full record beside the headline
    assert "error" not in full["sampler"] and full["sampler"]["transformed"]["us_per_step"] > 0
    assert full["value"] == d["value"]


def test_rccl_pipeline_world_one(tmp_path):
    """LogpStepLoop's RCCL branch on device tensors, at world size 1 on the one GPU
    (LogpStepLoop(pipeline=True)): 12 steps over 12 different ensembles with two steps in
    flight; every step's gathered vector equals the direct log-prob of its own ensemble bit
    for bit (snapshots taken behind the wait on each gather), as does the sequential step().
    Then the native loop (NativeComm: libngrtd's own RCCL communicator, ngrtd_logp_gather_n)
    over the same buffers, 3 steps per call on each ensemble: both gathered rows equal it."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()), RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0")
    subprocess.run([sys.executable, os.path.join(REPO, "tests", "dist_gpu_pipeline.py"), str(tmp_path), "1000", "8",
                    "12"], check=True, timeout=300, env=env, cwd=REPO)
    z = np.load(tmp_path / "pipeline.npz")
    assert str(z["backend"]) == "nccl"
    direct, snaps = z["direct"], z["snaps"]
    assert np.isfinite(direct).mean() > 0.5 and not np.array_equal(direct[0], direct[1], equal_nan=True)
    for i in range(direct.shape[0]):
        assert np.array_equal(snaps[i], direct[i], equal_nan=True), i
    assert np.array_equal(z["ens"], direct[-1], equal_nan=True)
    assert np.array_equal(z["seq"], direct[-1], equal_nan=True)
    nat = z["native"]                  # [K][2][W]: the native loop's two gathered rows per call
    for i in range(direct.shape[0]):
        assert np.array_equal(nat[i][0], direct[i], equal_nan=True), i
        assert np.array_equal(nat[i][1], direct[i], equal_nan=True), i
