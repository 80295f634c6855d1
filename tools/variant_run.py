#!/usr/bin/env python3
"""Run K single-launch log-prob calls of one c4 workload variant (for PMC passes per
variant: tools/gpu_variant_pmc.sh).  Variants: joint, noprior, prioronly, rtd_only,
rtd_bare (no priors, no likelihood), ce_only."""
import dataclasses
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def spec_of(name, L=64):
    from noblegas_rtd_mcmc_amd import workloads
    from noblegas_rtd_mcmc_amd.spec import ModelSpec
    base = workloads.c4_spec(L=L)
    return {
        "joint": lambda: base,
        "noprior": lambda: dataclasses.replace(base, include_prior=False, roles=[]),
        "prioronly": lambda: dataclasses.replace(base, include_like=False, roles=[]),
        "rtd_only": lambda: ModelSpec(n_wells=L, rtd=base.rtd),
        "rtd_bare": lambda: dataclasses.replace(ModelSpec(n_wells=L, rtd=base.rtd), include_prior=False,
                                                include_like=False, roles=[]),
        "ce_only": lambda: ModelSpec(n_wells=L, ce=base.ce),
    }[name]()


def main():
    name = sys.argv[1]
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    import torch
    from noblegas_rtd_mcmc_amd import workloads
    from noblegas_rtd_mcmc_amd.engine import LogProb
    spec = spec_of(name)
    th = torch.from_numpy(workloads.sample_prior(spec, 2048, np.random.default_rng(1))).cuda()
    lp = LogProb(spec, max_walkers=2048)
    out = torch.empty(2048, dtype=torch.float64, device="cuda")
    for _ in range(K):
        lp(th, out=out)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
