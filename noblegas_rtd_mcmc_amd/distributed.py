"""Multi-GPU ensembles: one process per GPU, walker blocks, RCCL all-gather (c5).

The reference's only parallelism is PyMC3 forking 3 chain processes
(run_age_mcmc_utils.py:416).  Here an ensemble of W_total walkers is split into
contiguous blocks, one per rank (``workloads.shard_walkers``); every rank evaluates its
block with its own GPU plan and the per-block log-prob vectors are exchanged with ONE
``all_gather_into_tensor`` (backend "nccl" = RCCL over xGMI on MI355X, "gloo" in CPU
tests).  The payload is W_total float64 (16 KiB at 2048 walkers): latency-bound, so it is
a single collective per step, never bucketed.

``sharded_demcz`` runs the reference's sampler (DEMetropolisZ: one chain per (walker, well),
or per walker) over the shards: its chains propose from their own histories, so sampling
itself exchanges nothing; the trace's log-probs are gathered once at the end.
"""
import ctypes as C
import os

import torch
import torch.distributed as dist

from .workloads import shard_walkers


def host_staged(group=None, t=None):
    """True when the collective of ``group`` cannot take device tensors directly: the gloo
    backend (CPU rehearsals of the multi-rank path, e.g. several ranks sharing the one GPU of
    a test box -- RCCL refuses two ranks on one device) with a CUDA tensor.  The tensor then
    goes through a host copy around the collective."""
    if not dist.is_initialized() or (t is not None and not t.is_cuda):
        return False
    return dist.get_backend(group) == "gloo"


def all_gather_into(out, buf, group=None):
    """``dist.all_gather_into_tensor(out, buf)``; through host copies when host_staged."""
    if not host_staged(group, buf):
        dist.all_gather_into_tensor(out, buf, group=group)
        return out
    ho = torch.empty(out.shape, dtype=out.dtype)
    dist.all_gather_into_tensor(ho, buf.cpu(), group=group)
    out.copy_(ho)
    return out


def rccl_library_path():
    """The RCCL library torch itself loaded (its bundled librccl.so when present), so that the
    native communicator (ngrtd_comm) shares one RCCL instance with torch.distributed; None:
    the system's librccl.so.1."""
    d = os.path.join(os.path.dirname(torch.__file__), "lib")
    for name in ("librccl.so", "librccl.so.1"):
        path = os.path.join(d, name)
        if os.path.exists(path):
            return path
    return None


class NativeComm:
    """libngrtd's own RCCL communicator (ngrtd_comm) over the ranks of ``group``: rank 0 draws the
    unique id, torch.distributed broadcasts it, every rank joins.  ``gather_n(plan, theta, W,
    bufs, gathers, k)`` runs k steps of LogpStepLoop in native code (ngrtd_logp_gather_n: the
    block's log-prob launch, then ncclAllGather on the communicator's stream, two steps in flight)
    -- no Python, ctypes or torch.distributed call per step."""

    def __init__(self, ctx, group=None):
        from . import _lib
        self.ctx, self.lib = ctx, ctx.lib
        self.rank, self.world = dist.get_rank(group), dist.get_world_size(group)
        path = rccl_library_path()
        self.path = path.encode() if path else None
        obj = [None]
        if self.rank == 0:
            buf = (C.c_uint8 * 128)()
            st = self.lib.ngrtd_comm_unique_id(self.path, buf)
            if st != _lib.NGRTD_OK:
                raise _lib.NgrtdError("ngrtd_comm_unique_id failed (%d)" % st)
            obj = [bytes(buf)]
        dist.broadcast_object_list(obj, src=0, group=group)
        idb = (C.c_uint8 * 128).from_buffer_copy(obj[0])
        h = C.c_void_p()
        ctx.check(self.lib.ngrtd_comm_create(ctx.h, self.path, idb, self.world, self.rank, C.byref(h)), "ngrtd_comm_create")
        self.h = h

    def gather_n(self, plan, theta, W, bufs, gathers, k):
        """bufs: CUDA float64 [2][per], gathers: [2][world per] (contiguous)."""
        per = bufs.shape[1]
        self.ctx.set_stream(torch.cuda.current_stream(theta.device).cuda_stream)
        self.ctx.check(self.lib.ngrtd_logp_gather_n(plan.plan, self.h, C.c_void_p(theta.data_ptr()), int(W), int(per),
                                                    C.c_void_p(bufs.data_ptr()), C.c_void_p(gathers.data_ptr()), int(k)),
                       "ngrtd_logp_gather_n")

    def close(self):
        if getattr(self, "h", None):
            self.lib.ngrtd_comm_destroy(self.h)
            self.h = None


class LogpStepLoop:
    """The per-step work of ``bench.py`` on one rank (and of any caller that shards a
    walker ensemble): the batched log-prob of the rank's walker block, then -- world > 1
    -- ONE all-gather of the per-block log-prob vectors into the ensemble vector.

    ``evaluate(out)`` writes the block's log-probs into ``out`` (a contiguous prefix of a
    block buffer padded to the largest block, so uneven shards gather with one collective).
    Two block buffers and two gathered vectors are allocated once (``outs``, ``gathers``):
    ``run`` alternates them so that a step's all-gather overlaps the next step's
    evaluation.  ``step()`` uses buffer 0 and returns the gathered [per * world] vector;
    ``ensemble()`` the unpadded [W_total] view of the latest one.

    The same function runs under torchrun (RCCL) and in the world-size-2 gloo tests
    (tests/test_distributed_cpu.py), so the bench's multi-GPU step has no untested branch.

    ``pipeline``: None (default) gathers -- and pipelines the gathers of device-side
    collectives -- only when world > 1; True gathers every step through the two-deep
    pipeline at ANY world size (a process group must be initialised), so the async branch
    runs on one GPU with RCCL at world size 1 (tests/test_gpu_distributed.py); False never
    pipelines.

    ``gather``: "step" (default) all-gathers after every evaluation, as above; "region": ``run(k)``
    evaluates k times (one native call with ``evaluate_n``) and all-gathers ONCE, after the last.
    The walker blocks are independent -- each chain decides on its own log-prob, and the
    ensemble vector is needed only where it is consumed (a trace, a check) -- and an RCCL
    all-gather costs ~21 us even at world size 1, twice a c4 log-prob (profiles/r06d_gather_per_step.jsonl:
    32 vs 10.6 us per step), so bench.py gathers once per timed region.
    """

    def __init__(self, evaluate, W_total, device, dtype=torch.float64, group=None, evaluate_n=None, pipeline=None,
                 gather="step"):
        if gather not in ("step", "region"):
            raise ValueError('gather must be "step" or "region"')
        self.evaluate = evaluate
        self.evaluate_n = evaluate_n      # optional: evaluate_n(out, k) = k evaluations in one call
        self.gather = gather
        self.group = group
        self.W_total = int(W_total)
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.lo, self.hi = shard_walkers(self.W_total, self.rank, self.world)
        self.per = (self.W_total + self.world - 1) // self.world
        if pipeline and not dist.is_initialized():
            raise ValueError("LogpStepLoop(pipeline=True) needs an initialised process group")
        self.pipeline = pipeline
        # gather every step: several ranks, or a forced pipeline (world 1 included)
        self.collective = self.world > 1 or bool(pipeline)
        nb = 2 if self.collective else 1
        # the two block buffers and the two gathered vectors as rows of one tensor each (the
        # native loop, gather_n, takes them as [2][per] / [2][world per])
        self.bufs2 = torch.full((nb, self.per), float("nan"), dtype=dtype, device=device)
        self.bufs = [self.bufs2[i] for i in range(nb)]
        self.outs = [b[: self.hi - self.lo] for b in self.bufs]
        self.gathers2 = torch.empty((nb, self.per * self.world), dtype=dtype, device=device) if self.collective else None
        self.gathers = [self.gathers2[i] for i in range(nb)] if self.collective else self.bufs
        self.buf, self.out, self.gathered = self.bufs[0], self.outs[0], self.gathers[0]
        # optional: gather_n(k) = k steps of the two-deep pipeline in native code (NativeComm)
        self.gather_n = None

    def step(self):
        self.evaluate(self.outs[0])
        if self.collective:
            all_gather_into(self.gathers[0], self.bufs[0], group=self.group)
        self.gathered = self.gathers[0]
        return self.gathered

    def run(self, k, hook=None):
        """k steps.  World 1 with ``evaluate_n`` (and no per-step hook): one call enqueues the
        k evaluations.  World > 1 with device-side collectives: two steps in flight -- step i
        evaluates into block buffer i % 2 while step i - 1's all-gather (async_op, the
        collective's own stream) still runs; step i's gather starts once its evaluation has
        (the collective waits on the current stream), and step i + 2's evaluation waits for it
        (``work.wait()``: a stream dependency, no host sync) because it reuses the buffer.
        Otherwise (host-staged gloo rehearsals) k sequential ``step()``s.  ``hook(i, before)``
        runs around step i's evaluation (bench.py's event sampling)."""
        k = int(k)
        if not self.collective and self.evaluate_n is not None and hook is None:
            self.evaluate_n(self.out, k)
            return self.gathered
        if self.collective and self.gather == "region":
            # k evaluations of the block (one native call when possible), then ONE all-gather
            if self.evaluate_n is not None and hook is None:
                self.evaluate_n(self.outs[0], k)
            else:
                for i in range(k):
                    if hook:
                        hook(i, True)
                    self.evaluate(self.outs[0])
                    if hook:
                        hook(i, False)
            if k:
                all_gather_into(self.gathers[0], self.bufs[0], group=self.group)
                self.gathered = self.gathers[0]
            return self.gathered
        if self.collective and self.gather_n is not None and hook is None and self.pipeline is not False:
            self.gather_n(k)
            if k:
                self.gathered = self.gathers[(k - 1) & 1]
            return self.gathered
        if not self.collective or self.pipeline is False or host_staged(self.group, self.bufs[0]):
            for i in range(k):
                if hook:
                    hook(i, True)
                self.evaluate(self.outs[0])
                if hook:
                    hook(i, False)
                if self.collective:
                    all_gather_into(self.gathers[0], self.bufs[0], group=self.group)
            self.gathered = self.gathers[0]
            return self.gathered
        works = [None, None]
        for i in range(k):
            s = i & 1
            if works[s] is not None:
                works[s].wait()
            if hook:
                hook(i, True)
            self.evaluate(self.outs[s])
            if hook:
                hook(i, False)
            works[s] = dist.all_gather_into_tensor(self.gathers[s], self.bufs[s], group=self.group, async_op=True)
        for w in works:
            if w is not None:
                w.wait()
        if k:
            self.gathered = self.gathers[(k - 1) & 1]
        return self.gathered

    def ensemble(self):
        if not self.collective:
            return self.out
        return torch.cat([self.gathered[r * self.per: r * self.per + (lambda s: s[1] - s[0])(
            shard_walkers(self.W_total, r, self.world))] for r in range(self.world)])


class ShardedLogProb:
    """Evaluate a rank's walker block and all-gather the ensemble log-prob."""

    def __init__(self, evaluate_block, W_total, group=None):
        self.evaluate_block = evaluate_block
        self.W_total = int(W_total)
        self.group = group
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.lo, self.hi = shard_walkers(self.W_total, self.rank, self.world)
        self.per = (self.W_total + self.world - 1) // self.world

    def block(self, theta_full):
        """This rank's slice [..., lo:hi] of a full-ensemble array."""
        return theta_full[..., self.lo:self.hi].contiguous()

    def __call__(self, theta_block):
        """theta_block [..., W_block] -> (logp_block [W_block], logp_full [W_total])."""
        lp = self.evaluate_block(theta_block)
        return lp, self.gather(lp)

    def gather(self, lp_block):
        if self.world == 1:
            return lp_block
        buf = torch.full((self.per,), float("nan"), dtype=lp_block.dtype, device=lp_block.device)
        buf[: lp_block.shape[0]] = lp_block
        out = torch.empty(self.per * self.world, dtype=lp_block.dtype, device=lp_block.device)
        all_gather_into(out, buf, group=self.group)
        return torch.cat([out[r * self.per: r * self.per + (shard_walkers(self.W_total, r, self.world)[1]
                                                            - shard_walkers(self.W_total, r, self.world)[0])]
                          for r in range(self.world)])

    def gather_positions(self, x_block):
        if self.world == 1:
            return x_block
        lead = x_block.shape[:-1]
        buf = torch.zeros(lead + (self.per,), dtype=x_block.dtype, device=x_block.device)
        buf[..., : x_block.shape[-1]] = x_block
        flat = buf.contiguous().reshape(-1)
        out = torch.empty(self.world * flat.numel(), dtype=x_block.dtype, device=x_block.device)
        all_gather_into(out, flat, group=self.group)
        out = out.reshape((self.world,) + lead + (self.per,))
        parts = []
        for r in range(self.world):
            lo, hi = shard_walkers(self.W_total, r, self.world)
            parts.append(out[r][..., : hi - lo])
        return torch.cat(parts, dim=-1)


def sharded_demcz(log_prob, x_block, W_total, tune, draws, *, per_well, device_sampler=False, group=None, **kw):
    """DEMetropolisZ over an ensemble sharded in walker blocks: every rank runs the chains
    of its block (sampler.DEMetropolisZ on a batched log_prob, or DeviceDEMetropolisZ on an
    engine.LogProb), each chain drawing the random numbers of its GLOBAL index, so the
    union of the shards is bitwise the single-process run of the whole ensemble.  Chains
    are independent (each proposes from its own history), so sampling needs no
    collective at all; the per-draw log-probs and decisions are all-gathered once, at
    the end, for the trace.  ``per_well`` (required, so that the chain structure never
    depends on which backend is picked): True = one chain per (walker, well) (log_prob
    returns [L][W]), False = one chain per walker ([W]).  Returns (result of this rank's
    block, logp [draws, (L,) W_total], accepted [draws, (L,) W_total])."""
    from .sampler import DEMetropolisZ, DeviceDEMetropolisZ
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    lo, hi = shard_walkers(int(W_total), rank, world)
    if x_block.shape[-1] != hi - lo:
        raise ValueError("rank %d owns walkers [%d, %d), got a block of %d" % (rank, lo, hi, x_block.shape[-1]))
    cls = DeviceDEMetropolisZ if device_sampler else DEMetropolisZ
    res = cls(log_prob, chain0=lo, n_chains_total=int(W_total), per_well=bool(per_well), **kw).run(x_block, tune, draws)
    if world == 1:
        return res, res["logp"], res["accepted"]
    per = (int(W_total) + world - 1) // world

    def gather(t, fill):      # [..., W_block] -> [..., W_total] (per-well logs: [draws][L][W])
        lead = t.shape[:-1]
        t2 = t.reshape(-1, t.shape[-1])
        buf = torch.full((t2.shape[0], per), fill, dtype=t.dtype, device=t.device)
        buf[:, : t2.shape[1]] = t2
        out = torch.empty((world * t2.shape[0], per), dtype=t.dtype, device=t.device)
        all_gather_into(out, buf.contiguous(), group=group)
        out = out.view(world, t2.shape[0], per)
        g = torch.cat([out[r, :, : shard_walkers(int(W_total), r, world)[1] - shard_walkers(int(W_total), r, world)[0]]
                       for r in range(world)], dim=1)
        return g.reshape(lead + (int(W_total),))
    return res, gather(res["logp"], float("nan")), gather(res["accepted"].to(torch.float64), 0.0).to(torch.uint8)
