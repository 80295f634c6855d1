"""One rank of the c5 rehearsal on a one-GPU box (tests/test_gpu_distributed.py): launched
by torch.distributed.run with 2 ranks, both on cuda:0, gloo backend (RCCL refuses two ranks
on one device; distributed.all_gather_into stages the collective through host memory).

Each rank owns its block of ONE seeded c4 ensemble (strong sharding, 2 x W/2 walkers) and
runs, with the real HIP log-prob:
  1. distributed.LogpStepLoop (bench.py's per-step function): its block's log-prob, then
     the all-gather of the ensemble vector;
  2. distributed.sharded_demcz(device_sampler=True): the device DEMetropolisZ chains of its
     block, drawing the random numbers of their global chain indices.
It saves what it saw to <outdir>/rank<r>.npz; the test compares with one process."""
import dataclasses
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    outdir, W, L, per_well = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    import torch
    import torch.distributed as dist
    from noblegas_rtd_mcmc_amd import workloads as wl
    from noblegas_rtd_mcmc_amd.distributed import LogpStepLoop, sharded_demcz
    from noblegas_rtd_mcmc_amd.engine import LogProb
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    rank = dist.get_rank()
    try:
        spec = wl.c4_spec(L=L, N=1200)
        full = wl.sample_prior(spec, W, np.random.default_rng(34568))
        loop = LogpStepLoop(None, W, torch.device("cuda", 0))
        blk = torch.from_numpy(np.ascontiguousarray(full[:, :, loop.lo:loop.hi])).cuda()
        lp = LogProb(spec, max_walkers=loop.hi - loop.lo, device=0)
        run = lp.bind(blk, loop.out)
        loop.evaluate = lambda out: run()
        g1 = loop.step().clone()
        g2 = loop.run(3).clone()
        kw = dict(tune_interval=4, seed=2024)
        kw["per_well"] = bool(per_well)
        # the sampler in PyMC3's transformed space (a plan with the Jacobians)
        lpj = LogProb(dataclasses.replace(spec, jacobian=True), max_walkers=loop.hi - loop.lo, device=0)
        res, lp_tr, acc_tr = sharded_demcz(lpj, blk, W, tune=8, draws=6, device_sampler=True, **kw)
        np.savez(os.path.join(outdir, "rank%d.npz" % rank), ens=loop.ensemble().cpu().numpy(),
                 g1=g1.cpu().numpy(), g2=g2.cpu().numpy(), lo=loop.lo, hi=loop.hi,
                 x=res["x"].cpu().numpy(), lp=res["lp"].cpu().numpy(), samples=res["samples"].cpu().numpy(),
                 lp_tr=lp_tr.cpu().numpy(), acc_tr=acc_tr.cpu().numpy())
        lp.close()
        lpj.close()
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
