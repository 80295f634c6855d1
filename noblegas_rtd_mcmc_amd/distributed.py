"""Multi-GPU ensembles: one process per GPU, walker blocks, RCCL all-gather (c5).

The reference's only parallelism is PyMC3 forking 3 chain processes
(run_age_mcmc_utils.py:416).  Here an ensemble of W_total walkers is split into
contiguous blocks, one per rank (``workloads.shard_walkers``); every rank evaluates its
block with its own GPU plan and the per-block log-prob vectors are exchanged with ONE
``all_gather_into_tensor`` (backend "nccl" = RCCL over xGMI on MI355X, "gloo" in CPU
tests).  The payload is W_total float64 (16 KiB at 2048 walkers): latency-bound, so it is
a single collective per step, never bucketed.

``exchange="positions"`` additionally all-gathers the walker positions so the DE proposal
of a walker may draw partners from every block (one more all-gather of P*L*W_total
doubles per step); the default ``"logp"`` keeps DE moves inside each block (independent
sub-ensembles, no position traffic).
"""
import math

import torch
import torch.distributed as dist

from .sampler import pymc3_tune
from .workloads import shard_walkers


class LogpStepLoop:
    """The per-step work of ``bench.py`` on one rank (and of any caller that shards a
    walker ensemble): the batched log-prob of the rank's walker block, then -- world > 1
    -- ONE all-gather of the per-block log-prob vectors into the ensemble vector.

    ``evaluate(out)`` writes the block's log-probs into ``out`` (a contiguous prefix of a
    block buffer padded to the largest block, so uneven shards gather with one collective).
    Both the block buffer and the gathered vector are allocated once.  ``step()`` returns
    the gathered [per * world] vector; ``ensemble()`` the unpadded [W_total] view.

    The same function runs under torchrun (RCCL) and in the world-size-2 gloo tests
    (tests/test_distributed_cpu.py), so the bench's multi-GPU step has no untested branch.
    """

    def __init__(self, evaluate, W_total, device, dtype=torch.float64, group=None):
        self.evaluate = evaluate
        self.group = group
        self.W_total = int(W_total)
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.lo, self.hi = shard_walkers(self.W_total, self.rank, self.world)
        self.per = (self.W_total + self.world - 1) // self.world
        self.buf = torch.full((self.per,), float("nan"), dtype=dtype, device=device)
        self.out = self.buf[: self.hi - self.lo]
        self.gathered = (torch.empty(self.per * self.world, dtype=dtype, device=device)
                         if self.world > 1 else self.buf)

    def step(self):
        self.evaluate(self.out)
        if self.world > 1:
            dist.all_gather_into_tensor(self.gathered, self.buf, group=self.group)
        return self.gathered

    def ensemble(self):
        if self.world == 1:
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
        dist.all_gather_into_tensor(out, buf, group=self.group)
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
        dist.all_gather_into_tensor(out, flat, group=self.group)
        out = out.reshape((self.world,) + lead + (self.per,))
        parts = []
        for r in range(self.world):
            lo, hi = shard_walkers(self.W_total, r, self.world)
            parts.append(out[r][..., : hi - lo])
        return torch.cat(parts, dim=-1)


def sharded_de_step_loop(sharded, x_block, tune, draws, seed=123423, scaling=1e-3, tune_interval=100,
                         exchange="logp"):
    """Population DE-MC over a sharded ensemble (see sampler.DEMetropolis).  Every rank
    runs the same number of steps; tuning uses the GLOBAL acceptance rate (all-reduce)."""
    x = x_block.clone()
    Wb = x.shape[-1]
    d = int(x[..., 0].numel())
    lamb = 2.38 / math.sqrt(2 * d)
    g = torch.Generator(device=x.device)
    g.manual_seed(seed + 7919 * sharded.rank)
    lp, lp_full = sharded(x)
    acc_window = 0.0
    kept = []
    for it in range(tune + draws):
        pool = sharded.gather_positions(x) if exchange == "positions" else x
        Wp = pool.shape[-1]
        base = sharded.lo if exchange == "positions" else 0
        idx = torch.arange(Wb, device=x.device) + base
        r1 = (idx + torch.randint(1, Wp, (Wb,), generator=g, device=x.device)) % Wp
        r2 = (r1 + torch.randint(1, Wp - 1, (Wb,), generator=g, device=x.device)) % Wp
        r2 = torch.where(r2 == idx, (r2 + 1) % Wp, r2)
        r2 = torch.where(r2 == r1, (r2 + 1) % Wp, r2)
        eps = (torch.rand(x.shape, generator=g, device=x.device, dtype=x.dtype) * 2 - 1) * scaling
        prop = x + lamb * (pool[..., r1] - pool[..., r2]) + eps
        lp_prop, _ = sharded(prop)
        logu = torch.log(torch.rand((Wb,), generator=g, device=x.device, dtype=lp.dtype))
        acc = ((lp_prop - lp) > logu) & ~torch.isnan(lp_prop)
        x = torch.where(acc, prop, x)
        lp = torch.where(acc, lp_prop, lp)
        acc_window += float(acc.sum())
        if it < tune and (it + 1) % tune_interval == 0:
            t = torch.tensor([acc_window], dtype=torch.float64, device=x.device)
            if sharded.world > 1:
                dist.all_reduce(t, group=sharded.group)
            scaling = pymc3_tune(scaling, float(t) / (tune_interval * sharded.W_total))
            acc_window = 0.0
        if it >= tune:
            kept.append(sharded.gather(lp))
    return x, lp, (torch.stack(kept) if kept else None), scaling
