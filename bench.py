#!/usr/bin/env python3
"""Headline benchmark: joint CE + RTD-convolution log-likelihood evaluations per second.

Workload (BASELINE.json configs[3]), per GPU: 2048 walkers x 64 wells x
(CE over 5 gases + RTD convolution of 5 tracers over a 1200-year input series,
exponential RTD) in float64.  One step = one full log-prob of the rank's walker block
(theta resident in HBM) + an RCCL all-gather of the per-block log-prob vector (N > 1).
Scaling is weak: every rank owns its own 2048-walker block (c5).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...

Rank 0 prints ONE JSON line; see DESIGN.md 'Measurement' for the roofline accounting.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "log-likelihood evals/sec (CE + RTD-conv), 2048 walkers, 1/2/4/8 MI355X"
FP64_MFMA_PEAK = 78.6e12     # dense FP64 matrix peak, 256 CU x 4 SIMD x 32 FLOP/clk x 2.4 GHz
                             # (tools/ubench_fp64.hip measures 78.3: profiles/r01_ubench_fp64.txt)
FP64_VALU_PEAK = 38.3e12     # v_fma_f64 throughput measured by tools/ubench_fp64.hip (profiles/r01_ubench_fp64.txt)
HBM_PEAK = 8.0e12            # MI355X_MICROARCH.md chip table
PMC_SUMMARY = "r01_pmc.json"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--walkers", type=int, default=2048)
    ap.add_argument("--wells", type=int, default=64)
    ap.add_argument("--ages", type=int, default=1200)
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="bounded CPU-baseline budget")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-overlap", action="store_true", help="N > 1: all-gather on the compute stream")
    ap.add_argument("--event-every", type=int, default=8,
                    help="bracket the kernels of every k-th timed step with HIP events (kernel roofline)")
    return ap.parse_args()


def cpu_baseline(spec, theta, budget_s, workers):
    """The oracle (reference-faithful NumPy per-walker loop) on the host cores, on a
    bounded sample of walkers of the same workload."""
    import multiprocessing as mp
    from oracle import models as om
    t0 = time.perf_counter()
    om.log_prob(spec, theta, walkers=[0])                   # one walker: size the sample
    per = time.perf_counter() - t0
    n = max(workers, int(budget_s / max(per, 1e-6)) * workers)
    idx = [i % theta.shape[2] for i in range(n)]
    chunks = [idx[i::workers] for i in range(workers)]
    ctx = mp.get_context("fork")
    t0 = time.perf_counter()
    with ctx.Pool(workers) as pool:
        pool.starmap(_cpu_chunk, [(spec, theta, c) for c in chunks])
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "evals/s", "cores": workers, "kind": "port",
            "sample": "%d walker log-probs of the same workload (oracle/models.py per-walker loop: "
                      "reference-faithful NumPy CE + convolve per (well, tracer)), %d processes, %.1f s"
                      % (n, workers, dt)}


def _cpu_chunk(spec, theta, walkers):
    from oracle import models as om
    return om.log_prob(spec, theta, walkers=walkers)


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist
    from noblegas_rtd_mcmc_amd import workloads
    from noblegas_rtd_mcmc_amd.engine import LogProb

    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    W = args.walkers
    spec = workloads.c4_spec(L=args.wells, N=args.ages)
    # this rank's walker block of the global ensemble (weak scaling: W per GPU)
    theta_h = workloads.sample_prior(spec, W, np.random.default_rng(34568 + rank))
    theta = torch.from_numpy(theta_h).to(dev)
    lp = LogProb(spec, max_walkers=W, device=local)
    # N > 1: the all-gather of step i runs on a communication stream while step i+1's
    # kernel runs (double-buffered logp / gather buffers); the compute stream reuses a
    # buffer only after the gather that read it has finished.  --no-overlap serialises.
    outs = [torch.empty(W, dtype=torch.float64, device=dev) for _ in range(2)]
    gathered = [torch.empty(W * world, dtype=torch.float64, device=dev) for _ in range(2)]
    overlap = world > 1 and not args.no_overlap
    comm = torch.cuda.Stream(device=dev) if overlap else None
    ready = [torch.cuda.Event() for _ in range(2)]
    freed = [torch.cuda.Event() for _ in range(2)]
    issued = [False, False]
    nstep = [0]

    def step():
        k = nstep[0] % 2
        nstep[0] += 1
        o = outs[k]
        if not overlap:
            lp(theta, out=o)
            if world > 1:
                dist.all_gather_into_tensor(gathered[k], o)
            return
        cur = torch.cuda.current_stream(dev)
        if issued[k]:
            cur.wait_event(freed[k])              # the gather that read outs[k] is done
        lp(theta, out=o)
        ready[k].record(cur)
        comm.wait_event(ready[k])
        with torch.cuda.stream(comm):
            dist.all_gather_into_tensor(gathered[k], o)
            freed[k].record(comm)
        issued[k] = True
    out = outs[0]

    for _ in range(args.warmup):
        step()
    # which kernels does one step launch? (one profiled step after the warm-up)
    lp.ctx.set_profiling(True)
    lp.kernel_stats(reset=True)
    step()
    lp.ctx.set_profiling(False)
    kinds = {k for k, v in lp.kernel_stats(reset=True).items() if v[1]}
    single_kernel = kinds == {"fused"}
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # timed region.  Kernel time for the roofline, measured live with HIP events on the
    # launch stream (torch's current stream, which the plan enqueues on):
    #  * N = 1: one event pair around the whole region; every launch in it is the
    #    single-launch log-prob kernel, so region / steps is its average duration
    #    (back-to-back, as rocprofv3 --kernel-trace sees it);
    #  * N > 1: the all-gather shares the stream, so the kernels of every k-th step are
    #    bracketed by their own event pair (read back after the region, no host syncs).
    lp.kernel_stats(reset=True)
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    for i in range(args.steps):
        sample = (world > 1 or not single_kernel) and i % args.event_every == 0
        if sample:
            lp.ctx.set_profiling(True)
        step()
        if sample:
            lp.ctx.set_profiling(False)
    ev1.record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    ks = lp.kernel_stats(reset=True)
    if world == 1 and single_kernel:
        ks = dict(ks)
        ks["fused"] = (ev0.elapsed_time(ev1), args.steps)
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    assert torch.isfinite(out).any()
    # PCIe-inclusive rate: theta handed over as host memory (staged H2D per call, results
    # copied back) -- reported beside `value`, never as it (DESIGN.md 'Measurement')
    host_staged = None
    if rank == 0:
        hs = max(5, args.steps // 20)
        lp(theta_h, soa=True)
        t1 = time.perf_counter()
        for _ in range(hs):
            lp(theta_h, soa=True)
        host_staged = W * hs / (time.perf_counter() - t1)

    if rank == 0:
        info = lp.info(W)
        U = spec.n_wells * W
        C = info["channels"]
        N = spec.rtd.n_ages
        # dominant kernel: the single-launch log-prob kernel when the plan uses it
        kname = "fused" if ks["fused"][1] else "rtd"
        kms = ks[kname][0] / max(ks[kname][1], 1)
        kfull = {"fused": "logp_fused_kernel", "rtd": "rtd_exp_mfma_kernel" if info["mfma_rows"] else "rtd_conc_kernel"}[kname]
        # committed PMC summary of the same command (tools/gpu_profile.sh -> tools/profile_summary.py)
        pmc = {}
        path = os.environ.get("NGRTD_PMC_SUMMARY") or os.path.join(REPO, "profiles", PMC_SUMMARY)
        if os.path.exists(path):
            with open(path) as f:
                for k, e in json.load(f).items():
                    if kfull in k:
                        pmc = e
        traffic = pmc.get("hbm_bytes_per_launch")   # FETCH_SIZE x 2 (calibrated) + WRITE_SIZE
        if info.get("surrogate"):
            # FP64 work of the launch: PMC-counted FP64 FLOPs per (walker, well) unit of this
            # kernel (SQ_INSTS_VALU_FLOPS_FP64 x 64 lanes, fma = 2) x units
            fpu = pmc.get("fp64_flop_per_unit")
            flops = fpu * U if fpu else None
            flop_src = "PMC fp64_flop_per_unit %s x %d units (%s)" % (
                "%.1f" % fpu if fpu else "n/a", U, os.path.relpath(path, REPO))
        else:
            # exact matrix-core path: one FMA (2 FLOP) per (unit, channel, age >= 1)
            flops = 2.0 * U * C * (N - 1)
            flop_src = "2 * units * channels * (N - 1) (matrix-core Horner)"
        achieved = flops / (kms * 1e-3) if flops else None
        evals_per_s_kernel = W / (kms * 1e-3)
        # algorithmic HBM bytes of the same launch: every theta row read once + logp out
        hbm_bytes = U * 8.0 * len(spec.roles) + (W * 8.0 if kname == "fused" else U * 8.0 * len(spec.rtd.tracers))
        evals = W * world * args.steps
        line = {
            "metric": METRIC,
            "value": evals / dt,
            "unit": "evals/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {"workload": "c4 joint CE+RTD log-prob: %d walkers/GPU x %d wells x (5 gases CE + 5 tracers "
                                   "RTD exponential, N=%d ages)" % (W, args.wells, N),
                       "walkers_per_gpu": W, "wells": args.wells, "gases": 5, "tracers": 5, "ages": N,
                       "parallelism": ("walker blocks per GPU + RCCL all-gather of logp" +
                                       (" (overlapped with the next step's kernel)" if overlap else ""))
                                      if world > 1 else "single GPU"},
            "roofline": {"bound": "mfma", "achieved": achieved / 1e12 if achieved else None,
                         "peak": FP64_MFMA_PEAK / 1e12, "unit": "TFLOP/s",
                         "frac": achieved / FP64_MFMA_PEAK if achieved else None, "traffic": traffic,
                         "kernel": kfull, "kernel_ms": kms, "flop_per_launch": flops, "flop_source": flop_src,
                         "pipe": "FP64 (gfx950 FP64 VALU and MFMA share one pipe; the surrogate path is VALU)",
                         "fp64_valu_peak_measured": FP64_VALU_PEAK / 1e12,
                         "frac_of_fp64_valu_peak": achieved / FP64_VALU_PEAK if achieved else None,
                         # SURVEY.md §8d froze the REFERENCE algorithm's count (2 exp per age at
                         # X = 20, 167 FLOP per walker-well-age + 850 CE): informational only --
                         # the surrogate/Horner rewrite does not execute that work
                         "survey_8d_flop_per_eval": args.wells * (N * 167.0 + 850.0),
                         "survey_8d_equivalent_TFLOPs": evals_per_s_kernel * args.wells * (N * 167.0 + 850.0) / 1e12,
                         "hbm": {"algorithmic_bytes": hbm_bytes, "achieved_GBps": hbm_bytes / (kms * 1e-3) / 1e9,
                                 "peak_GBps": HBM_PEAK / 1e9, "frac": hbm_bytes / (kms * 1e-3) / HBM_PEAK}},
            "host_staged_value": host_staged,
            "kernels_ms": {k: v[0] / max(v[1], 1) for k, v in ks.items()},
            "geometry": info,
        }
        if not args.no_cpu_baseline and world == 1:
            workers = min(16, os.cpu_count() or 1)
            line["cpu_baseline"] = cpu_baseline(spec, theta_h, args.cpu_seconds, workers)
        else:
            line["cpu_baseline"] = None
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
