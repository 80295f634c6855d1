#!/usr/bin/env python3
"""Headline benchmark: joint CE + RTD-convolution log-likelihood evaluations per second.

Workload (BASELINE.json configs[3]): 2048 walkers x 64 wells x (CE over
5 gases + RTD convolution of 5 tracers over a 1200-year input series, exponential RTD)
in float64.  One step = one full batched log-prob of the rank's walker block (theta
resident in HBM), the loop of distributed.LogpStepLoop: LogpStepLoop.run enqueues the K launches
with one native call (ngrtd_logp_n) instead of K Python round trips, and for N > 1 the per-block
log-prob vectors are all-gathered ONCE, after the K-th step, inside the timed region (--gather
region; the blocks are independent, and an all-gather per step (--gather step) costs twice a
step: profiles/r06d_gather_per_step.jsonl).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--scaling weak|strong]
                    [--mod-type1 exponential|exp_pist_flow|piston|dispersion] [--mod-type2 piston|...]
    torchrun --nproc-per-node N bench.py --gpus N ...

--scaling weak (default): every rank owns 2048 walkers of a (2048 N)-walker ensemble.
--scaling strong (c5): ONE 2048-walker ensemble is sharded, 2048 / N walkers per rank.
Either way the ensemble is drawn once from the same seed and each rank takes its
contiguous block (workloads.shard_walkers).  --mod-type1/2 select the other RTD models the
reference published runs of.

Rank 0 prints ONE JSON line; see DESIGN.md §6 for the roofline accounting.
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
FP64_PEAK = 78.6e12          # MI355X FP64 peak (vector and matrix, AMD spec: 256 CU x 128 FLOP/clk x 2.4 GHz)
FP64_VALU_MEASURED = 38.3e12 # v_fma_f64 throughput measured by tools/ubench_fp64.hip (profiles/r01_ubench_fp64.txt)
FP64_MFMA_MEASURED = 78.3e12 # v_mfma_f64_16x16x4f64, same microbenchmark
HBM_PEAK = 8.0e12            # MI355X_MICROARCH.md chip table
PMC_SUMMARIES = ("r06fin2_pmc.json", "r06fin_pmc.json", "r06_pmc.json", "r05_pmc.json", "r04_pmc.json", "r03s2f_pmc.json", "r03s2_pmc.json", "r03_pmc.json", "r02_pmc.json", "r01_pmc.json")   # newest first (tools/gpu_profile.sh)

# the RTD parameters each model adds (run_age_mcmc.py:145-178)
MODEL_PARS = {"exponential": (), "piston": (), "exp_pist_flow": ("eta",), "dispersion": ("D",)}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--walkers", type=int, default=2048, help="walkers per GPU (weak) or in total (strong)")
    ap.add_argument("--wells", type=int, default=64)
    ap.add_argument("--ages", type=int, default=1200)
    ap.add_argument("--scaling", choices=("weak", "strong"), default="weak")
    ap.add_argument("--mod-type1", default="exponential", choices=sorted(MODEL_PARS))
    ap.add_argument("--mod-type2", default=None, choices=sorted(MODEL_PARS))
    ap.add_argument("--cpu-seconds", type=float, default=16.0, help="bounded CPU-baseline budget (both variants)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-exact", action="store_true", help="skip the exact-path (no surrogate) line")
    ap.add_argument("--no-sampler", action="store_true", help="skip the device DEMetropolisZ line")
    ap.add_argument("--no-models", action="store_true",
                    help="skip the published-model / c2 / c3 side lines (N = 1)")
    ap.add_argument("--sampler-steps", type=int, default=256,
                    help="steps of the timed device DEMetropolisZ call (one multi-step launch chunk)")
    ap.add_argument("--sampler-tune", type=int, default=1000,
                    help="untimed tuning steps before the sampler's timed window (its draw phase)")
    ap.add_argument("--event-every", type=int, default=8,
                    help="bracket the kernels of every k-th timed step with HIP events (multi-kernel / N > 1)")
    ap.add_argument("--backend", choices=("nccl", "gloo"), default="nccl",
                    help="torch.distributed backend for N > 1 (nccl = RCCL over xGMI; gloo stages the "
                         "all-gather through host memory: the multi-rank rehearsal on a one-GPU box)")
    ap.add_argument("--one-device", action="store_true",
                    help="every rank uses cuda:0 (rehearsal of the N > 1 path on a one-GPU box; needs --backend gloo)")
    ap.add_argument("--no-reference-runs", action="store_true",
                    help="skip the reference's own sampling runs, timed end to end (N = 1)")
    ap.add_argument("--pipeline", action="store_true",
                    help="gather every step through LogpStepLoop's two-deep async pipeline even at N = 1 (RCCL at "
                         "world size 1: the device-tensor branch of the N > 1 step on a one-GPU box)")
    ap.add_argument("--gather", choices=("region", "step"), default="region",
                    help="N > 1: ONE all-gather of the ensemble log-prob vector per timed region (default: the "
                         "walker blocks are independent) or one per step (two in flight)")
    ap.add_argument("--no-native", action="store_true",
                    help="--gather step: step through torch.distributed's all-gather loop instead of the native one")
    ap.add_argument("--full-line", action="store_true",
                    help="print the full record (every side leg) as the last line instead of the headline "
                         "(the A/B scripts under tools/ parse it)")
    ap.add_argument("--side-out", default=os.path.join(REPO, "gpurun_out", "bench_side.json"),
                    help="file the full record (every side leg) is written to; stdout's last line is the headline")
    return ap.parse_args()


# ------------------------------------------------------------------ the printed line
HEADLINE_MAX_BYTES = 7000     # the driver keeps a bounded stdout tail: the last line must fit well inside it
# the headline keys kept verbatim (the contract's fields + the measured companions of `value`)
HEADLINE_KEYS = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
                 "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "plan_build_ms",
                 "value_amortized_20k", "conv_evals_per_s", "exact_value", "host_staged_value", "ensemble_finite_frac",
                 "kernels_ms",
                 "geometry")


def _r(x, nd=4):
    """x to nd significant figures (None / non-numbers pass through)."""
    if isinstance(x, bool) or not isinstance(x, (int, float)) or x != x or x in (float("inf"), float("-inf")):
        return x
    return float("%.*g" % (nd, x))


def write_side(line, path):
    """The full record -- models, reference_runs, sampler, ce_runs, geometry, cpu_baseline variants --
    as one JSON file beside the bench (None if it cannot be written: the headline never depends on it)."""
    if not path:
        return None
    try:
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        with open(path, "w") as f:
            json.dump(line, f, indent=1)
        return os.path.relpath(path, REPO) if os.path.abspath(path).startswith(REPO) else path
    except OSError:
        return None


def headline(full, side_path=None):
    """The one-line JSON object the driver parses: the contract's fields, roofline, cpu_baseline
    and the exact-path line verbatim (trimmed prose), plus one-line summaries of every side leg
    (their full objects are in `side_path`).  Bounded by HEADLINE_MAX_BYTES."""
    out = {k: full[k] for k in HEADLINE_KEYS if k in full}
    if isinstance(out.get("config"), dict):
        cfg = dict(out["config"])
        if isinstance(cfg.get("rtd_sums"), str) and len(cfg["rtd_sums"]) > 160:
            cfg["rtd_sums"] = cfg["rtd_sums"][:157] + "..."
        out["config"] = cfg
    if isinstance(full.get("exact_roofline"), dict):
        er = full["exact_roofline"]
        out["exact_roofline"] = {k: _r(er.get(k)) for k in ("bound", "achieved", "peak", "unit", "frac", "kernel_ms")}
    cb = full.get("cpu_baseline")
    if isinstance(cb, dict):
        out["cpu_baseline"] = {k: cb.get(k) for k in ("value", "unit", "cores", "kind", "sample")}
        if isinstance(out["cpu_baseline"]["sample"], str) and len(out["cpu_baseline"]["sample"]) > 400:
            out["cpu_baseline"]["sample"] = out["cpu_baseline"]["sample"][:397] + "..."
        if isinstance(cb.get("variants"), dict):
            out["cpu_baseline"]["vectorised_numpy"] = _r(cb["variants"].get("vectorised_numpy"))
    else:
        out["cpu_baseline"] = cb
    side = {"file": side_path}
    models = full.get("models")
    if isinstance(models, dict) and "error" not in models:
        # kernel microseconds per launch of every model line (2048 walkers x 64 wells unless stated)
        side["models_kernel_us"] = {k: _r(1e3 * v["kernel_ms"], 3) for k, v in models.items()
                                    if isinstance(v, dict) and isinstance(v.get("kernel_ms"), (int, float))}
        fr = {k: _r(v["roofline"]["frac"], 3) for k, v in models.items()
              if isinstance(v, dict) and isinstance(v.get("roofline"), dict) and "frac" in v["roofline"]}
        if fr:
            side["models_fp64_frac"] = fr
    elif models is not None:
        side["models"] = models
    for leg in ("reference_runs", "ce_runs"):
        rr = full.get(leg)
        if isinstance(rr, dict) and "error" not in rr:
            s = {"runs": {r["run"]: [_r(r.get("wall_s")), _r(r.get("speedup_vs_reference")), _r(r.get("accept_rate"), 3)]
                          + ([_r(r["speedup_vs_oracle_projection"])] if r.get("speedup_vs_oracle_projection") else [])
                          for r in rr.get("runs", []) if isinstance(r, dict) and "run" in r},
                 "fields": "[wall_s, speedup_vs_reference, accept_rate(, speedup_vs_oracle_projection: runs with no "
                           "shipped reference time)]"}
            for k in ("total_wall_s", "reference_total_s", "reference_total_s_projected"):
                if k in rr:
                    s[k] = _r(rr[k])
            if rr.get("batched_3_wells"):
                s["batched_3_wells"] = [[_r(b.get("wall_s")), _r(b.get("speedup_vs_reference"))]
                                        for b in rr["batched_3_wells"]]
            side[leg] = s
        elif rr is not None:
            side[leg] = {"error": str(rr.get("error"))[:200]} if isinstance(rr, dict) else rr
    samp = full.get("sampler")
    if isinstance(samp, dict):
        side["sampler"] = {k: [_r(v.get("us_per_step")), _r(v.get("accept_rate"), 3)] for k, v in samp.items()
                           if isinstance(v, dict) and "us_per_step" in v}
        side["sampler_fields"] = "[us_per_step, accept_rate]: device DEMetropolisZ, 2048 walkers x 64 wells"
        if "error" in samp:
            side["sampler_error"] = str(samp["error"])[:200]
    out["side"] = side
    # hard bound: drop the largest summaries first if the prose ever grows
    for k in ("models_fp64_frac", "models_kernel_us", "ce_runs", "reference_runs", "sampler"):
        if len(json.dumps(out)) <= HEADLINE_MAX_BYTES:
            break
        side.pop(k, None)
    return out


# savenum digits -> the parameters they sample (run_age_mcmc.py:180-198): 1 log10 J (He4_ter
# production), 2 thalf_cfc (CFC12 half-life), 3 lamsf6 (SF6 contamination); every published
# 4-tracer run is savenum 123 (the shipped conv_traces/*.123.netcdf)
SAVENUM_PARS = {"1": "J", "2": "thalf_cfc", "3": "lamsf6"}


def model_spec(args, savenum=""):
    from noblegas_rtd_mcmc_amd import workloads
    m1, m2 = args.mod_type1, args.mod_type2
    return workloads.c4_spec(L=args.wells, N=args.ages, mod_type1=m1, mod_type2=m2,
                             par_names=workloads.model_par_names(m1, m2, savenum))


# ------------------------------------------------------------------ CPU baseline
def cpu_share():
    """CPUs this job may use: the affinity mask, capped by OMP_NUM_THREADS (the GPU box
    grants a 16-CPU share of a larger machine and says so there; os.cpu_count() reports
    the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    cap = os.environ.get("OMP_NUM_THREADS")
    if cap and cap.isdigit() and int(cap) > 0:
        n = min(n, int(cap))
    return max(1, n)


def _cpu_loop_chunk(spec, theta, walkers):
    from oracle import models as om
    return om.log_prob(spec, theta, walkers=walkers)


def _cpu_vec_chunk(spec, theta, reps):
    from oracle.vectorized import log_prob_vec
    for _ in range(reps):
        log_prob_vec(spec, theta)
    return reps


def cpu_baseline(spec, theta, budget_s, workers):
    """The oracle on the host cores, on a bounded sample of the same workload: (1) the
    reference-faithful per-walker loop (oracle/models.py: NumPy CE + one convolve per
    (well, tracer), as ForwardMod.perform does), (2) the vectorised NumPy variant
    (oracle/vectorized.py: all walkers of a well at once).  One process per CPU."""
    import multiprocessing as mp
    from oracle import models as om
    from oracle.vectorized import log_prob_vec
    os.environ.setdefault("OPENBLAS_NUM_THREADS", "1")
    ctx = mp.get_context("fork")
    W = theta.shape[2]
    # (1) per-walker loop
    t0 = time.perf_counter()
    om.log_prob(spec, theta, walkers=[0])
    per = time.perf_counter() - t0
    n = max(workers, int(0.5 * budget_s / max(per, 1e-6)) * workers)
    idx = [i % W for i in range(n)]
    chunks = [idx[i::workers] for i in range(workers)]
    t0 = time.perf_counter()
    with ctx.Pool(workers) as pool:
        pool.starmap(_cpu_loop_chunk, [(spec, theta, c) for c in chunks])
    dt_loop = time.perf_counter() - t0
    loop_rate = n / dt_loop
    # (2) vectorised: 64-walker slices per call
    Wc = min(64, W)
    sl = np.ascontiguousarray(theta[:, :, :Wc])
    t0 = time.perf_counter()
    log_prob_vec(spec, sl)
    per = time.perf_counter() - t0
    reps = max(1, int(0.5 * budget_s / max(per, 1e-6)))
    t0 = time.perf_counter()
    with ctx.Pool(workers) as pool:
        pool.starmap(_cpu_vec_chunk, [(spec, sl, reps)] * workers)
    dt_vec = time.perf_counter() - t0
    vec_rate = workers * reps * Wc / dt_vec
    return {"value": loop_rate, "unit": "evals/s", "cores": workers, "kind": "port",
            "sample": ("%d walker log-probs of the same workload through the reference-faithful per-walker "
                       "loop (oracle/models.py: NumPy CE + one convolve per (well, tracer)), %d processes, "
                       "%.1f s.  The oracle skips the reference's per-call DataFrame copies and object "
                       "construction (ForwardMod.perform, run_age_mcmc_utils.py:94), so it is faster than the "
                       "reference itself" % (n, workers, dt_loop)),
            "variants": {"per_walker_loop": loop_rate,
                         "vectorised_numpy": vec_rate,
                         "vectorised_sample": "%d calls of %d walkers (oracle/vectorized.py), %d processes, %.1f s"
                                              % (reps * workers, Wc, workers, dt_vec)},
            "cpu_count_machine": os.cpu_count()}


# ------------------------------------------------------------------ main
def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist
    from noblegas_rtd_mcmc_amd import workloads
    from noblegas_rtd_mcmc_amd.distributed import LogpStepLoop
    from noblegas_rtd_mcmc_amd.engine import LogProb

    if args.one_device and args.backend != "gloo" and world > 1:
        raise SystemExit("--one-device needs --backend gloo (RCCL refuses two ranks on one device)")
    gpu = 0 if args.one_device else local
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    if world > 1 or args.pipeline:
        if world == 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29531")
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")

    W_total = args.walkers * world if args.scaling == "weak" else args.walkers
    spec = model_spec(args)
    # ONE ensemble for the whole job (same seed at every N); each rank takes its block
    lo, hi = workloads.shard_walkers(W_total, rank, world)
    theta_full = workloads.sample_prior(spec, W_total, np.random.default_rng(34568))
    theta_h = np.ascontiguousarray(theta_full[:, :, lo:hi])
    del theta_full
    Wb = hi - lo
    theta = torch.from_numpy(theta_h).to(dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    lp = LogProb(spec, max_walkers=Wb, device=gpu)       # plan: tables, surrogate fit + validation, c0 table
    torch.cuda.synchronize()
    plan_build_ms = (time.perf_counter() - t0) * 1e3
    loop = LogpStepLoop(None, W_total, dev, pipeline=True if args.pipeline else None, gather=args.gather)
    fasts = {o.data_ptr(): lp.bind(theta, o) for o in loop.outs}   # one bound launch per block buffer
    fast_n = lp.bind_n(theta, loop.out)
    loop.evaluate = lambda out: fasts[out.data_ptr()]()
    loop.evaluate_n = lambda out, k: fast_n(k)     # N = 1: the K steps in one native call
    # N > 1 over RCCL (device buffers): the K steps -- launch + all-gather, two in flight -- in one
    # native call too (ngrtd_logp_gather_n on libngrtd's own communicator); gloo rehearsals and
    # --no-native keep torch.distributed's loop
    native = None
    if loop.collective and args.gather == "step" and args.backend == "nccl" and not args.no_native:
        from noblegas_rtd_mcmc_amd.distributed import NativeComm
        native = NativeComm(lp.ctx)
        loop.gather_n = lambda k: native.gather_n(lp, theta, Wb, loop.bufs2, loop.gathers2, k)

    # which kernels does one step launch? (one profiled step)
    lp.ctx.set_profiling(True)
    lp.kernel_stats(reset=True)
    loop.step()
    lp.ctx.set_profiling(False)
    kinds = {k for k, v in lp.kernel_stats(reset=True).items() if v[1]}
    single_kernel = kinds == {"fused"}

    # the side lines (outside the timed region, reported beside the headline, never as it)
    # run BEFORE it: the headline region then starts on a GPU that has been busy for
    # seconds, at the clock a long sampling run holds (a 20-step region
    # started from an idle GPU measured slower per launch)
    side = {}
    if world == 1 and not args.no_exact and spec.rtd.mod_type1 == "exponential" and not spec.rtd.mod_type2 \
            and lp.info(Wb).get("surrogate"):
        side.update(exact_line(args, spec, theta, Wb, lp.info(Wb)["channels"], spec.rtd.n_ages))
    if world == 1 and not args.no_models:
        try:
            side["models"] = model_lines(args, gpu)
        except Exception as e:        # noqa: BLE001
            side["models"] = {"error": repr(e)}
    if world == 1 and not args.no_reference_runs:
        try:
            side["reference_runs"] = reference_runs(gpu)
        except Exception as e:        # noqa: BLE001
            side["reference_runs"] = {"error": repr(e)}
        try:
            side["ce_runs"] = ce_runs(gpu)
        except Exception as e:        # noqa: BLE001
            side["ce_runs"] = {"error": repr(e)}
    # device DEMetropolisZ on every rank (its own chains: no collective), max over ranks
    samp = None
    if not args.no_sampler:
        samp, us = {}, {}
        try:                          # a side measurement: never lose the headline line to it
            samp, us = sampler_line(args, spec, lp, theta, gpu)
        except Exception as e:        # noqa: BLE001
            samp = {"error": repr(e)}
        for space in ("transformed", "natural", "transformed_joint"):   # max over ranks (all ranks reach this)
            t = torch.tensor([us.get(space, float("nan"))], dtype=torch.float64, device=dev)
            if world > 1:
                dist.all_reduce(t, op=dist.ReduceOp.MAX) if args.backend == "nccl" else _host_max(t)
            if space in samp and "us_per_step" in samp[space]:
                e = samp[space]
                e["us_per_step"] = float(t.item())
                e["walker_steps_per_s"] = W_total / (float(t.item()) * 1e-6)
                e["chain_steps_per_s"] = e["walker_steps_per_s"] * e["chains"] / Wb
        if "transformed" in samp:
            samp["us_per_step"] = samp["transformed"]["us_per_step"]

    for _ in range(args.warmup):
        loop.step()
    torch.cuda.synchronize()
    # the ensemble vector of an untimed step: the timed steps must reproduce it bit for bit
    ref_ens = loop.step().clone() if loop.collective else loop.out.clone()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # timed region.  Kernel time for the roofline, measured live with HIP events on the
    # launch stream:
    #  * N = 1 and one kernel per step: the event pair ngrtd_logp_n records around its K
    #    launches (LogProb.region_ms), so region / steps is that kernel's average duration
    #    back to back (as rocprofv3 --kernel-trace sees it);
    #  * otherwise the kernels of every k-th step get their own event pairs (read back
    #    after the region, no host syncs inside it).
    lp.kernel_stats(reset=True)
    per_step_events = (loop.collective and args.gather == "step" and native is None) or not single_kernel
    t0 = time.perf_counter()
    if per_step_events:
        def hook(i, before):
            if i % args.event_every == 0:
                lp.ctx.set_profiling(before)
        loop.run(args.steps, hook=hook)
    else:
        loop.run(args.steps)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    ks = dict(lp.kernel_stats(reset=True))
    if not per_step_events and native is None:
        ks["fused"] = (lp.region_ms(), args.steps)
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX) if args.backend == "nccl" else _host_max(t)
        dt = float(t.item())
    last = loop.gathered if loop.collective else loop.out
    if not torch.equal(last.nan_to_num(), ref_ens.nan_to_num()) or \
            not torch.equal(torch.isnan(last), torch.isnan(ref_ens)):
        raise SystemExit("bench: the timed steps' log-probs differ from an untimed evaluation")
    finite_frac = float(torch.isfinite(loop.ensemble()).double().mean())
    if not finite_frac > 0.5:
        raise SystemExit("bench: only %.3f of the ensemble log-probs are finite" % finite_frac)
    if native is not None:
        # the native loop's region holds launches and gathers: the kernel's own duration for the
        # roofline from a burst of event-bracketed launches right after it (outside the timed region)
        ks["gather_region_ms_per_step"] = (lp.region_ms(), args.steps)
        lp.ctx.set_profiling(True)
        lp.kernel_stats(reset=True)
        loop.run(max(10, args.steps // 4))
        torch.cuda.synchronize()
        lp.ctx.set_profiling(False)
        ks["fused"] = lp.kernel_stats(reset=True)["fused"]
        if world > 1:
            dist.barrier()

    if rank == 0:
        line = report(args, spec, lp, ks, dt, world, W_total, Wb, plan_build_ms, theta, theta_h, side)
        line["ensemble_finite_frac"] = finite_frac
        if samp is not None:
            line["sampler"] = samp
        if loop.collective:
            line["config"]["backend"] = args.backend + (" (host-staged all-gather)" if args.backend == "gloo" else "")
            line["config"]["one_device"] = bool(args.one_device)
            line["config"]["pipeline"] = bool(args.pipeline or world > 1)
            line["config"]["gather"] = ("one all-gather of the ensemble log-prob vector per timed region (after its "
                                        "last step, inside the timing)" if args.gather == "region" else
                                        "one all-gather per step, two in flight")
            line["config"]["step_loop"] = ("native (ngrtd_logp_n, then one all-gather)" if args.gather == "region" else
                                           "native (ngrtd_logp_gather_n: libngrtd's RCCL communicator)" if native is not None
                                           else "torch.distributed")
        # the full record (every side leg) goes to a file; stdout's LAST line is the compact
        # headline object the driver parses (<= HEADLINE_MAX_BYTES, tests/test_bench_line_cpu.py)
        side_path = write_side(line, args.side_out)
        print(json.dumps(line if args.full_line else headline(line, side_path)), flush=True)
    if native is not None:
        native.close()
    if dist.is_initialized():
        dist.destroy_process_group()


def _host_max(t):
    """MAX all-reduce through host memory (gloo: the one-GPU rehearsal of N > 1)."""
    import torch.distributed as dist
    h = t.cpu()
    dist.all_reduce(h, op=dist.ReduceOp.MAX)
    t.copy_(h)


def pmc_summary(kfull, instance=None):
    """Committed PMC summary of the same command (tools/gpu_profile.sh -> tools/profile_summary.py):
    the entry of this exact kernel instance when present, else any launch of the kernel."""
    for name in PMC_SUMMARIES:
        path = os.environ.get("NGRTD_PMC_SUMMARY") or os.path.join(REPO, "profiles", name)
        if os.path.exists(path):
            with open(path) as f:
                summ = json.load(f)
            for key in ([instance] if instance else []) + [kfull]:
                for k, e in summ.items():
                    if key in k:
                        return e, os.path.relpath(path, REPO) + (" [%s]" % key)
    return {}, None


def report(args, spec, lp, ks, dt, world, W_total, Wb, plan_build_ms, theta, theta_h, side):
    import torch
    from noblegas_rtd_mcmc_amd.engine import LogProb
    info = lp.info(Wb)
    U = spec.n_wells * Wb
    C = info["channels"]
    N = spec.rtd.n_ages
    kname = "fused" if ks["fused"][1] else "rtd"
    kms = ks[kname][0] / max(ks[kname][1], 1)
    kfull = {"fused": "logp_fused_kernel", "rtd": "rtd_exp_mfma_kernel" if info["mfma_rows"] else "rtd_conc_kernel"}[kname]
    instance = None
    if kname == "fused":
        r = spec.rtd
        mix = (1 if r.mod_type2 == "piston" else 0) | (2 if r.mod_type1 == "exp_pist_flow" else 0)
        full = spec.ce is not None and spec.include_like and spec.include_prior
        instance = "logp_fused_kernel<%d, %s, 2, %d>" % (C, "true" if full else "false", mix)
    pmc, pmc_path = pmc_summary(kfull, instance)
    traffic = pmc.get("hbm_bytes_per_launch")        # FETCH_SIZE x 2 (calibrated) + WRITE_SIZE
    if info.get("surrogate") and pmc.get("fp64_flop_per_unit"):
        # FP64 work of the launch: PMC-counted FP64 FLOPs per (walker, well) unit of this
        # kernel (SQ_INSTS_VALU_FLOPS_FP64 x 64 lanes, fma = 2) x units
        fpu = pmc["fp64_flop_per_unit"]
        flops = fpu * U
        flop_src = "PMC fp64_flop_per_unit %.1f x %d units (%s)" % (fpu, U, pmc_path)
        bound = "fp64_valu"
    else:
        # exact path: one FMA (2 FLOP) per (unit, channel, age >= 1) per geometric component
        ncomp = sum(1 for m in (spec.rtd.mod_type1, spec.rtd.mod_type2) if m in ("exponential", "exp_pist_flow"))
        flops = 2.0 * U * C * (N - 1) * max(ncomp, 1)
        flop_src = "algorithmic: 2 x units x channels x (N - 1) x %d geometric component(s)" % max(ncomp, 1)
        bound = "fp64_mfma" if info["mfma_rows"] else "fp64_valu"
    achieved = flops / (kms * 1e-3)
    hbm_bytes = U * 8.0 * len(spec.roles) + (Wb * 8.0 if kname == "fused" else U * 8.0 * len(spec.rtd.tracers))
    evals = W_total * args.steps
    model = spec.rtd.mod_type1 + ("-" + spec.rtd.mod_type2 if spec.rtd.mod_type2 else "")
    line = {
        "metric": METRIC,
        "value": evals / dt,
        "unit": "evals/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt * 1e3 / args.steps,
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (seeded c4 ensemble; series = shipped C_in_dict.pk x lognormal noise)",
        "config": {"workload": "c4 joint CE+RTD log-prob: %d walkers (%d/GPU) x %d wells x (5 gases CE + 5 tracers "
                               "RTD %s, N=%d ages)" % (W_total, Wb, args.wells, model, N),
                   "walkers_total": W_total, "walkers_per_gpu": Wb, "wells": args.wells, "gases": 5, "tracers": 5,
                   "ages": N, "rtd_model": model,
                   "rtd_sums": {1: "piecewise-Chebyshev surrogate of the exponential channel sums, fitted and "
                                   "validated per plan (max rel err %.2g <= 5e-14); uncovered tau take the exact "
                                   "matrix-core path",
                                2: "exp_pist_flow: exact Horner head of <= 32 ages + piecewise-Chebyshev surrogates "
                                   "of the block tails, fitted and validated per plan (max rel err %.2g <= 5e-14); "
                                   "uncovered tau/eta sum their tails exactly"}.get(
                                       info.get("surrogate"), "exact (no surrogate%s)") % (
                                       info["surrogate_max_rel_err"] if info.get("surrogate") else ""),
                   "parallelism": ("%d walker blocks + RCCL all-gather of logp (%s scaling)" % (world, args.scaling))
                                  if world > 1 else "single GPU"},
        "roofline": {"bound": bound, "achieved": achieved / 1e12, "peak": FP64_PEAK / 1e12, "unit": "TFLOP/s",
                     "frac": achieved / FP64_PEAK, "traffic": traffic, "kernel": kfull, "kernel_ms": kms,
                     "flop_per_launch": flops, "flop_source": flop_src,
                     "peak_source": "MI355X FP64 spec (vector = matrix = 78.6 TFLOP/s)",
                     "frac_of_measured_fp64_valu": achieved / FP64_VALU_MEASURED if bound == "fp64_valu" else None,
                     "hbm": {"algorithmic_bytes": hbm_bytes, "achieved_GBps": hbm_bytes / (kms * 1e-3) / 1e9,
                             "peak_GBps": HBM_PEAK / 1e9, "frac": hbm_bytes / (kms * 1e-3) / HBM_PEAK}},
        "plan_build_ms": plan_build_ms,
        "kernels_ms": {k: v[0] / max(v[1], 1) for k, v in ks.items()},
        "geometry": info,
    }
    # also (walker, well, tracer) convolution evaluations per second
    line["conv_evals_per_s"] = line["value"] * spec.n_wells * len(spec.rtd.tracers)
    line.update({k: v for k, v in side.items() if k != "models"})
    # the reference's run length (run_age_mcmc_utils.py:412-417: tune 10 000 + draws 10 000)
    # with the plan build paid once: W S / (S t_step + plan_build)
    S20k = 20000
    line["value_amortized_20k"] = W_total * S20k / (S20k * dt / args.steps + plan_build_ms * 1e-3)
    if "models" in side:
        line["models"] = side["models"]
    # PCIe-inclusive rate: theta handed over as host memory (staged H2D per call, results
    # copied back) -- reported beside `value`, never as it
    hs = max(5, args.steps // 20)
    lp(theta_h, soa=True)
    t1 = time.perf_counter()
    for _ in range(hs):
        lp(theta_h, soa=True)
    line["host_staged_value"] = Wb * hs / (time.perf_counter() - t1)
    torch.cuda.synchronize()
    if not args.no_cpu_baseline and world == 1:
        line["cpu_baseline"] = cpu_baseline(spec, theta_h, args.cpu_seconds, cpu_share())
    else:
        line["cpu_baseline"] = None
    return line


def sampler_line(args, spec, lp, theta, gpu):
    """The device DEMetropolisZ (ngrtd_demcz_run) on the same walkers, outside the timed
    region: per-step time of ONE call of --sampler-steps steps (the multi-step launch; the
    call's two layout transposes included) in the draw phase, after --sampler-tune (1000)
    tuning steps and stop_tuning: the stationary regime of a reference-length run.  Primary: PyMC3's
    transformed space (a plan with the Jacobians -- the space the reference samples in);
    beside it the natural space on the headline plan.  Reported beside the headline, never
    as it.  Returns (fields, {space: us per step}) -- the caller takes the max over ranks."""
    import dataclasses
    import torch
    from noblegas_rtd_mcmc_amd.engine import LogProb
    n = max(1, args.sampler_steps)
    W = theta.shape[-1]
    out, us = {}, {}
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    lpj = LogProb(dataclasses.replace(spec, jacobian=True), max_walkers=W, device=gpu)
    torch.cuda.synchronize()
    build_ms = (time.perf_counter() - t0) * 1e3
    L = spec.n_wells
    tune = max(0, args.sampler_tune)
    for name, plan, pw in (("transformed", lpj, True), ("natural", lp, True), ("transformed_joint", lpj, False)):
        out[name] = _dz_time(plan, theta, pw, plan is lpj, tune, n)
        us[name] = out[name]["us_per_step"]
    out["transformed"]["plan_build_ms"] = build_ms
    lpj.close()
    # the reference's own sampled models (one launch per chunk of steps: dz_chain_kernel), on
    # the same walkers x wells in PyMC3's transformed space: its RTD-only model (4 tracers,
    # savenum 123, exponential; 1 tracer, savenum 0) and its CE-only model (Ne, Ar, Kr, Xe)
    if int(os.environ.get("WORLD_SIZE", "1")) == 1:
        from noblegas_rtd_mcmc_amd import workloads
        for name, sp in (("rtd_4tracer_123", workloads.rtd_only_spec(L, spec.rtd.n_ages)),
                         ("rtd_4tracer_123_exp_pist_flow", workloads.rtd_only_spec(L, spec.rtd.n_ages,
                                                                                   mod_type1="exp_pist_flow")),
                         ("rtd_1tracer", workloads.rtd_only_spec(L, spec.rtd.n_ages, tracers=("H3",), savenum="")),
                         ("ce_only", workloads.ce_only_spec(L))):
            sp = dataclasses.replace(sp, jacobian=True)
            th = torch.from_numpy(workloads.sample_prior(sp, W, np.random.default_rng(34568))).to(theta.device)
            pl = LogProb(sp, max_walkers=W, device=gpu)
            out[name] = _dz_time(pl, th, True, True, tune, n)
            out[name]["model"] = {"rtd_4tracer_123": "RTD-only, CFC12 SF6 H3 He4_ter, exponential, J/thalf_cfc/lamsf6",
                                  "rtd_4tracer_123_exp_pist_flow": "RTD-only, 4 tracers, exp_pist_flow, savenum 123",
                                  "rtd_1tracer": "RTD-only, H3, exponential, savenum 0",
                                  "ce_only": "CE-only, Ne Ar Kr Xe"}[name]
            pl.close()
            del th
        # generic model pairs (run_age_mcmc.py:61-70 without a specialised instance) on the joint
        # c4 shape: one launch per chunk on the generic DZ instances (MIX 64 | 8, + 128)
        for name, (m1, m2, pn) in (("joint_dispersion", ("dispersion", None, ("tau1", "D1"))),
                                   ("joint_exponential-exponential", ("exponential", "exponential", ("tau1", "tau2", "f1")))):
            sp = dataclasses.replace(workloads.c4_spec(L=L, N=spec.rtd.n_ages, mod_type1=m1, mod_type2=m2, par_names=pn),
                                     jacobian=True)
            th = torch.from_numpy(workloads.sample_prior(sp, W, np.random.default_rng(34569))).to(theta.device)
            pl = LogProb(sp, max_walkers=W, device=gpu)
            out[name] = _dz_time(pl, th, True, True, tune, n)
            out[name]["model"] = "joint CE + 5 tracers, %s, PyMC3 transformed space" % (m1 + ("-" + m2 if m2 else ""))
            pl.close()
            del th
    out["method"] = ("PyMC3 DEMetropolisZ, device-resident (ngrtd_demcz_run: one launch per <= 256 steps, "
                     "each block stepping its own chains); primary = per-well chains (one PyMC3 model per well, "
                     "as the reference runs them) in PyMC3's transformed space")
    out["us_per_step"] = out["transformed"]["us_per_step"]
    return out, us


def _dz_time(plan, theta, pw, transformed, tune, n):
    """Per-step time of ONE ngrtd_demcz_run call of n steps after `tune` tuning steps (the
    timed window is the draw phase, stop_tuning included: the stationary regime of a
    reference-length run, not the first steps of fresh chains), with its acceptance rate."""
    import torch
    from noblegas_rtd_mcmc_amd.sampler import DeviceDEMetropolisZ
    W, L = theta.shape[-1], plan.spec.n_wells
    s = DeviceDEMetropolisZ(plan, tune_interval=100, seed=7, transformed=transformed, per_well=pw)
    x, l, z = s.start(theta, tune, tune + n + 1)
    cnt = torch.zeros(1, dtype=torch.int64, device=theta.device)
    plan.demcz(x, l, tune, z)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    plan.demcz(x, l, n, z, n_accepted=cnt)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / n
    nch = W * (L if pw else 1)
    return {"us_per_step": dt * 1e6, "chains": nch, "chain_steps_per_s": nch / dt, "walker_steps_per_s": W / dt,
            "steps": n, "after_tune_steps": tune, "accept_rate": int(cnt.item()) / float(n * nch),
            "chain": "one per (walker, well)" if pw else "one per walker over its %d wells" % L}


# the RTD models of the reference's published runs (run_age_mcmc.py:61-70),
# without (savenum 0) and with (123: J, thalf_cfc, lamsf6 sampled -- the published
# configuration) the savenum parameters
PUBLISHED_MODELS = (("exponential", None, ""), ("exponential", None, "123"), ("exponential", "piston", ""), ("exponential", "piston", "123"),
                    ("exp_pist_flow", None, ""), ("exp_pist_flow", None, "123"), ("exp_pist_flow", "piston", ""),
                    ("exp_pist_flow", "piston", "123"))
# the other model pairs the reference's driver accepts (run_age_mcmc.py:61-70), on the generic
# single-launch instances (MIX bit 6): piston / dispersion single components, BMMs with an
# exponential / exp_pist_flow / dispersion second component, a piston first component
OTHER_MODELS = (("piston", None, ""), ("piston", None, "123"), ("dispersion", None, ""), ("dispersion", None, "123"),
                ("exponential", "exponential", ""), ("exponential", "exponential", "123"),
                ("exp_pist_flow", "exponential", ""), ("exponential", "exp_pist_flow", ""),
                ("exp_pist_flow", "exp_pist_flow", ""), ("exponential", "dispersion", ""), ("piston", "exponential", ""),
                ("dispersion", "piston", ""))


N_FULL = 25256            # the reference's series length: the whole C_in_dict (run_age_mcmc.py:46,209)
TAU2_HI_EPM2 = 1000.0     # tau2 range of a second exp_pist_flow component's lines at N = 1200
MODEL_PMC_SUMMARIES = ("r06_model_pmc.json", "r05_model_pmc.json")   # tools/gpu_model_pmc.sh + tools/model_pmc_summary.py, newest first


def model_pmc_summary(key):
    """The per-model PMC entry ("model[.savenum]@N") of the committed summary, or ({}, None)."""
    for name in MODEL_PMC_SUMMARIES:
        path = os.environ.get("NGRTD_MODEL_PMC_SUMMARY") or os.path.join(REPO, "profiles", name)
        if os.path.exists(path):
            with open(path) as f:
                summ = json.load(f)
            if key in summ:
                return summ[key], os.path.relpath(path, REPO)
    return {}, None


def fused_instance(m1, m2, sv, C=5):
    """The logp_fused_kernel instance a joint c4-shape plan of this model runs (FULL, C = 5)."""
    lw = 32 if "2" in sv else 0
    if m1 in ("exponential", "exp_pist_flow") and m2 in (None, "piston"):
        mix = (1 if m2 == "piston" else 0) | (2 if m1 == "exp_pist_flow" else 0) | lw
    else:
        mix = 64 | lw | (128 if "dispersion" in (m1, m2) else 0)   # generic; +128: the dispersion instances
    return "logp_fused_kernel<%d, true, 2, %d>" % (C, mix)


def _time_plan(spec, W, gpu, steps, seed=34568, tau2_hi=None):
    """Plan build time and the per-launch time of the plan's log-prob (HIP events on the
    launch stream around `steps` back-to-back launches) on a seeded prior ensemble (tau2 from
    U(50, tau2_hi) instead of its prior when given, as tools/model_pmc.py)."""
    import torch
    from noblegas_rtd_mcmc_amd import workloads
    from noblegas_rtd_mcmc_amd.engine import LogProb
    th = workloads.sample_prior(spec, W, np.random.default_rng(seed))
    if tau2_hi is not None:
        R = {r: i for i, r in enumerate(spec.roles)}
        th[R["tau2"]] = np.random.default_rng(8).uniform(50.0, tau2_hi, th[R["tau2"]].shape)
    th = torch.from_numpy(th).cuda(gpu)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    lp = LogProb(spec, max_walkers=W, device=gpu)
    torch.cuda.synchronize()
    build_ms = (time.perf_counter() - t0) * 1e3
    out = torch.empty(W, dtype=torch.float64, device=th.device)
    run = lp.bind_n(th, out)
    run(5)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    run(steps)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / steps
    finite = float(torch.isfinite(out).double().mean())
    info = lp.info(W)
    lp.close()
    return build_ms, ms, finite, info


def model_lines(args, gpu):
    """Side lines (N = 1, outside the headline's timed region): the RTD models the reference
    published runs of (run_age_mcmc.py:61-70) on the c4 shape, the other
    model pairs its driver accepts (OTHER_MODELS, the generic instances; "published": false), and
    the CE-only (c2) and RTD-only (c3) configurations of BASELINE.json.  Each: plan build,
    kernel time per launch, evals/s, PMC FP64 fraction (committed summary of the same kernel
    instance) and the rate amortised over a 20 000-step run."""
    import argparse as ap
    from noblegas_rtd_mcmc_amd import workloads
    steps = max(50, args.steps)
    W = args.walkers
    res = {}
    base_ms = {("exponential", None): None}
    lines = [(m1, m2, sv, args.ages) for m1, m2, sv in PUBLISHED_MODELS + OTHER_MODELS]
    # the published configuration at the reference's own series length (run_age_mcmc.py:46,209)
    lines += [(m1, m2, sv, N_FULL) for m1, m2, sv in PUBLISHED_MODELS if sv and args.ages != N_FULL]
    # ... and dispersion there (not published; its generic instance stages nothing of the series)
    lines += [("dispersion", None, "123", N_FULL)] if args.ages != N_FULL else []
    for m1, m2, sv, N in lines:
        a = ap.Namespace(wells=args.wells, ages=N, mod_type1=m1, mod_type2=m2)
        spec = model_spec(a, sv)
        # (dispersion sums every age exactly: fewer launches keep the line short)
        n = max(20, steps // 10) if "dispersion" in (m1, m2) else steps
        # a second exp_pist_flow component masks every age of a short series once tau2 (1 - 1/eta2)
        # passes N (the reference's g is then 0 / 0: NaN): tau2 from U(50, 1000) inside its prior
        t2 = TAU2_HI_EPM2 if (m2 == "exp_pist_flow" and N < 15000) else None
        build_ms, ms, finite, info = _time_plan(spec, W, gpu, n, tau2_hi=t2)
        if not sv and N == args.ages:
            base_ms[(m1, m2)] = ms
        inst = fused_instance(m1, m2, sv)
        key = m1 + ("-" + m2 if m2 else "") + ("." + sv if sv else "")
        U = W * args.wells
        e = {"kernel_ms": ms, "evals_per_s": W / (ms * 1e-3), "plan_build_ms": build_ms,
             "value_amortized_20k": W * 20000 / (20000 * ms * 1e-3 + build_ms * 1e-3),
             "finite_frac": finite, "kernel": inst, "surrogate": info.get("surrogate"), "ages": N,
             "sampled": list(spec.rtd.par_names), "savenum": int(sv) if sv else 0,
             "published": (m1, m2, sv) in PUBLISHED_MODELS}
        if t2 is not None:
            e["tau2_sample"] = ("U(50, %g) inside tau2's U(50, 15000) prior: at N = %d a second exp_pist_flow "
                                "component with tau2 (1 - 1/eta2) > N masks every age (NaN, as the reference)" % (t2, N))
        if sv and base_ms.get((m1, m2)) and N == args.ages:
            e["vs_savenum0_kernel"] = ms / base_ms[(m1, m2)]
        if sv and N != args.ages and ("%s.%s" % (m1 + ("-" + m2 if m2 else ""), sv)) in res:
            e["vs_N%d_kernel" % args.ages] = ms / res["%s.%s" % (m1 + ("-" + m2 if m2 else ""), sv)]["kernel_ms"]
        # the model's own PMC summary (tools/gpu_model_pmc.sh: one plan per profiled process)
        mp, mp_path = model_pmc_summary("%s@N%d" % (key, N))
        pmc, pmc_path = (mp, mp_path) if mp else pmc_summary("logp_fused_kernel", inst)
        if mp and mp.get("fp64_flop_per_unit"):
            fl = mp["fp64_flop_per_unit"] * U
            e["roofline"] = {"bound": "fp64_valu", "achieved": fl / (ms * 1e-3) / 1e12, "peak": FP64_PEAK / 1e12,
                             "unit": "TFLOP/s", "frac": fl / (ms * 1e-3) / FP64_PEAK,
                             "traffic": mp.get("hbm_bytes_per_launch"),
                             "lds_bank_conflict_cycles": mp.get("SQ_LDS_BANK_CONFLICT"),
                             "flop_source": "PMC fp64_flop_per_unit %.1f x %d units (%s, this model's launches only)" % (
                                 mp["fp64_flop_per_unit"], U, mp_path)}
        elif int(inst.rsplit(", ", 1)[1].rstrip(">")) & 64:
            # the generic instance runs several models (piston, dispersion, BMM pairs): a PMC
            # summary keyed by kernel instance cannot say which model it counted, so no FLOP rate
            e["roofline"] = None
            e["roofline_note"] = "generic instance shared by %d model pair(s); PMC counts are per instance, not per model" % (
                sum(1 for mm in OTHER_MODELS if fused_instance(*mm) == inst))
        elif pmc.get("fp64_flop_per_unit") and inst in (pmc_path or "") and N == args.ages:
            fl = pmc["fp64_flop_per_unit"] * U
            e["roofline"] = {"bound": "fp64_valu", "achieved": fl / (ms * 1e-3) / 1e12, "peak": FP64_PEAK / 1e12,
                             "unit": "TFLOP/s", "frac": fl / (ms * 1e-3) / FP64_PEAK, "traffic": pmc.get("hbm_bytes_per_launch"),
                             "flop_source": "PMC fp64_flop_per_unit %.1f x %d units (%s)" % (pmc["fp64_flop_per_unit"], U, pmc_path)}
        else:
            e["roofline"] = None
        if not finite >= 0.5:
            # a rate over a workload whose log-probs are mostly NaN / -inf says nothing: no rate
            e["valid"] = False
            e["invalid_reason"] = "finite_frac %.3f < 0.5" % finite
            for k in ("evals_per_s", "value_amortized_20k", "roofline"):
                e[k] = None
        res[key + ("@N%d" % N if N != args.ages else "")] = e
    for name, (spec, _) in (("c2", workloads.c2(W=8)), ("c3", workloads.c3(W=8))):
        build_ms, ms, finite, info = _time_plan(spec, W, gpu, steps, seed=12345 if name == "c2" else 23456)
        res[name] = {"workload": {"c2": "CE log-prob, %d walkers x 3 wells (PLM1, PLM6, PLM7) x 5 gases" % W,
                                  "c3": "RTD log-prob, %d walkers x 4 tracers (CFC12, SF6, H3, He4_ter), exponential, "
                                        "N=1200 shipped series, sampled log10 J" % W}[name],
                     "kernel_ms": ms, "evals_per_s": W / (ms * 1e-3), "plan_build_ms": build_ms,
                     "value_amortized_20k": W * 20000 / (20000 * ms * 1e-3 + build_ms * 1e-3), "finite_frac": finite}
    return res


# The reference's published runs (age_ens_runs_mcmc/conv_traces/*.netcdf):
# (tracers, mod_type1, mod_type2, savenum digits) per well
REFERENCE_RUNS = ((("CFC12",), "exponential", None, ()), (("SF6",), "exponential", None, ()),
                  (("H3",), "exponential", None, ()), (("He4_ter",), "exponential", None, ()),
                  (("CFC12", "SF6", "H3", "He4_ter"), "exponential", None, (1, 2, 3)),
                  (("CFC12", "SF6", "H3", "He4_ter"), "exp_pist_flow", None, (1, 2, 3)),
                  (("CFC12", "SF6", "H3", "He4_ter"), "exponential", "piston", (1, 2, 3)),
                  (("CFC12", "SF6", "H3", "He4_ter"), "exp_pist_flow", "piston", (1, 2, 3)))


# the dispersion models the reference's driver accepts (run_age_mcmc.py:61-70, D ~ U(0.01, 2):
# :170-178) at the published runs' shape -- not among the shipped traces, so no reference time:
# the oracle's per-walker log-prob x the run's 60 000 evaluations stands beside them
DISPERSION_RUNS = ((("CFC12", "SF6", "H3", "He4_ter"), "dispersion", None, (1, 2, 3)),
                   (("CFC12", "SF6", "H3", "He4_ter"), "dispersion", "piston", (1, 2, 3)))


def _oracle_logp_s(spec, theta, reps=3):
    """Seconds per walker log-prob of the reference-faithful per-walker oracle loop
    (oracle/models.py), best of `reps` -- the CPU baseline of a side run (one core)."""
    import oracle.models as om
    best = float("inf")
    for _ in range(reps):
        t0 = time.perf_counter()
        om.log_prob(spec, theta, walkers=[0])
        best = min(best, time.perf_counter() - t0)
    return best


def _run_name(well, tracers, m1, m2, sv):
    return "%s.%s.%s.%s.netcdf" % (well, ".".join(tracers), m1 + ("-" + m2 if m2 else ""),
                                   "".join(str(d) for d in sv) or "0")


def reference_runs(gpu, wells=("PLM1",)):
    """The reference's own runs, end to end: ``conv_mcmc(...).sample_mcmc()`` (the drop-in,
    run_age_mcmc.py:229-231 -> run_age_mcmc_utils.py:407-429) with the reference's arguments --
    1 well, the full series (N = 25 256), DEMetropolisZ in PyMC3's transformed space, 3 chains,
    tune 10 000, draws 10 000, tune_interval 1000, seed 123423 -- for every published model of
    PLM1 (the four single-tracer exponential runs at savenum 0 and the four 4-tracer models at
    savenum 123).  Wall seconds per run include the plan build (tables, surrogates), the
    sampling and the netCDF-4 trace write, beside the shipped trace's own sampling_time (PyMC3,
    3 processes, hardware unrecorded) and acceptance rate.  ens_dict.pk is not shipped: the
    observation mean is the trace's observed_data and sigma the fit of
    tests/golden/make_pymc3_accept.py (the ensemble a two-point [mu - s, mu + s]).  Then the same
    runs for the three published wells batched into ONE call (a 3-well plan, per-well chains:
    3 chains per well)."""
    import dataclasses
    import tempfile
    import torch
    from noblegas_rtd_mcmc_amd import workloads as wl
    from noblegas_rtd_mcmc_amd.run_age_mcmc_utils import conv_mcmc
    from noblegas_rtd_mcmc_amd.sampler import sample_model
    from noblegas_rtd_mcmc_amd.spec import ModelSpec
    fit = {e["name"]: e for e in json.load(open(os.path.join(REPO, "tests", "golden", "pymc3_accept_fit.json"))).values()}
    attrs = json.load(open(os.path.join(REPO, "tests", "golden", "trace_attrs.json")))
    C_in = wl.c_in_dict()
    tmp = tempfile.mkdtemp(prefix="ngrtd_runs_")
    runs, cfg = [], dict(chains=3, tune=10000, draws=10000, seed=123423, tune_interval=1000)

    def kwargs(well, tr, m1, m2, sv):
        e = fit[_run_name(well, tr, m1, m2, sv)]
        perr = wl.OBS_PERR_ALT if (m2 == "piston" and m1 == "exponential") else None
        return e, wl.reference_run_kwargs(well, tr, m1, m2 or False, sv or (0,), e["mu"], e["sd"], perr=perr,
                                         tau1=e["tau1"], C_in=C_in)
    # one untimed short run first: the process's one-time costs (code-object loads of the
    # sampling kernels, first allocations) are not a run's (the first timed run paid ~0.17 s)
    e0 = fit.get(_run_name(wells[0], *REFERENCE_RUNS[0]))
    if e0 is not None:
        tr, m1, m2, sv = REFERENCE_RUNS[0]
        _, (okw, ckw, pkw) = kwargs(wells[0], tr, m1, m2, sv)
        mc = conv_mcmc(wells[0], list(tr), okw, ckw, pkw, tmp, "0", max_walkers=3, device=gpu)
        mc.sample_mcmc(**dict(cfg, tune=20, draws=20))
        mc._lp.close()
    for well in wells:
        for tr, m1, m2, sv in REFERENCE_RUNS:
            name = _run_name(well, tr, m1, m2, sv)
            if name not in fit:
                continue
            e, (okw, ckw, pkw) = kwargs(well, tr, m1, m2, sv)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            mc = conv_mcmc(well, list(tr), okw, ckw, pkw, tmp, "".join(str(d) for d in sv) or "0", max_walkers=3,
                           device=gpu)
            t1 = time.perf_counter()
            mc.build_mcmc_model_joint_sT()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            out = mc.sample_mcmc(**cfg)
            torch.cuda.synchronize()
            t3 = time.perf_counter()
            ref_t = attrs.get(name, {}).get("sampling_time")
            ref_acc = e["n_acc"] / (3.0 * 9999.0)
            runs.append({"run": name[:-len(".netcdf")], "wall_s": t3 - t0, "plan_build_s": t2 - t1,
                         "sample_s": float(out["sampling_time"]), "trace_write_s": (t3 - t2) - float(out["sampling_time"]),
                         "accept_rate": float(out["accept_rate"]), "reference_sampling_time_s": ref_t,
                         "reference_accept_rate": ref_acc, "speedup_vs_reference": (ref_t / (t3 - t0)) if ref_t else None,
                         "posterior_tau1_mean": float(np.mean(out["posterior"]["tau1"])),
                         "logp_evals": 3 * 20000, "steps_per_s": 20000 / float(out["sampling_time"])})
            mc._lp.close()
    # the dispersion models at the same shape (no shipped trace: the oracle's projection beside)
    for well in wells:
        base = fit.get(_run_name(well, ("CFC12", "SF6", "H3", "He4_ter"), "exponential", None, (1, 2, 3)))
        for tr, m1, m2, sv in DISPERSION_RUNS if base else ():
            name = _run_name(well, tr, m1, m2, sv)
            okw, ckw, pkw = wl.reference_run_kwargs(well, tr, m1, m2 or False, sv, base["mu"], base["sd"], C_in=C_in)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            mc = conv_mcmc(well, list(tr), okw, ckw, pkw, tmp, "".join(str(d) for d in sv), max_walkers=3, device=gpu)
            t1 = time.perf_counter()
            lpd = mc.build_mcmc_model_joint_sT()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            out = mc.sample_mcmc(**cfg)
            torch.cuda.synchronize()
            t3 = time.perf_counter()
            sp = mc.spec()
            per = _oracle_logp_s(sp, wl.test_point(sp, 1))
            proj = per * 3 * 20000
            runs.append({"run": name[:-len(".netcdf")], "wall_s": t3 - t0, "plan_build_s": t2 - t1,
                         "sample_s": float(out["sampling_time"]), "trace_write_s": (t3 - t2) - float(out["sampling_time"]),
                         "accept_rate": float(out["accept_rate"]), "reference_sampling_time_s": None,
                         "oracle_logp_s": per, "oracle_projected_s": proj, "speedup_vs_oracle_projection": proj / (t3 - t0),
                         "us_per_step": 1e6 * float(out["sampling_time"]) / 20000,
                         "geometry": "wide (%d partials per unit)" % lpd.info(3)["disp_wide_g"],
                         "posterior_tau1_mean": float(np.mean(out["posterior"]["tau1"])),
                         "logp_evals": 3 * 20000, "steps_per_s": 20000 / float(out["sampling_time"])})
            mc._lp.close()
    # the three published wells in one call: their 1-well specs stacked into a 3-well plan
    batched = []
    for tr, m1, m2, sv in REFERENCE_RUNS:
        names = [_run_name(w, tr, m1, m2, sv) for w in ("PLM1", "PLM6", "PLM7")]
        if not all(n in fit for n in names):
            continue
        specs = []
        for w in ("PLM1", "PLM6", "PLM7"):
            e, (okw, ckw, pkw) = kwargs(w, tr, m1, m2, sv)
            specs.append(conv_mcmc(w, list(tr), okw, ckw, pkw, "", "0").spec())
        r = specs[0].rtd
        rtd = dataclasses.replace(r, obs=np.concatenate([s.rtd.obs for s in specs]),
                                  sd=np.concatenate([s.rtd.sd for s in specs]))
        spec3 = ModelSpec(n_wells=3, rtd=rtd)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        # every chain at PyMC3's test point, as the single runs beside it (sample_mcmc's default start)
        x0 = torch.from_numpy(wl.test_point(spec3, 3)).cuda(gpu)
        res = sample_model(spec3, 3, gpu, x0, 10000, 10000, 123423, 1000, space="transformed")
        from noblegas_rtd_mcmc_amd import trace
        idd = trace.inference_data(res, dataclasses.replace(spec3, jacobian=True), wells=["PLM1", "PLM6", "PLM7"],
                                   observed=spec3.rtd.obs)
        trace.to_netcdf(trace.InferenceData.from_dict(idd), os.path.join(tmp, "batched.netcdf"))
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        ref_t = sum(attrs.get(n, {}).get("sampling_time") or 0.0 for n in names)
        batched.append({"runs": [n[:-len(".netcdf")] for n in names], "start": "test_point",
                        "wall_s": wall, "sample_s": float(res["sampling_time"]),
                        "accept_rate": float(res["accept_rate"]), "reference_sampling_time_s_sum": ref_t,
                        "speedup_vs_reference": ref_t / wall if ref_t else None})
    import shutil
    shutil.rmtree(tmp, ignore_errors=True)
    return {"config": "conv_mcmc(...).sample_mcmc(): 1 well, N = 25 256, DEMetropolisZ (PyMC3's transformed space), "
                      "3 chains, tune 10 000, draws 10 000, tune_interval 1000, seed 123423; wall = plan build + "
                      "sampling + netCDF-4 trace write (after one untimed 40-step warm-up run of the first model)",
            "runs": runs, "batched_3_wells": batched,
            "total_wall_s": sum(r["wall_s"] for r in runs if r["reference_sampling_time_s"]),
            "reference_total_s": sum(r["reference_sampling_time_s"] or 0.0 for r in runs),
            "note": "total_wall_s / reference_total_s over the published runs; the dispersion runs carry the "
                    "oracle's per-walker log-prob x 60 000 (oracle_projected_s) instead"}


def ce_runs(gpu, wells=("PLM1", "PLM6", "PLM7")):
    """The reference's CE inference, end to end at its own shape (ng_interp/noble_gas_mcmc.py:402-424):
    one well per run, DEMetropolisZ(tune_interval=5000), 4 chains, tune 10 000, draws 50 000,
    seed 123423, the prior checks and the InferenceData built (CEModel.sample).  Wall seconds
    include the plan build.  No CE trace is shipped, so the CPU baseline is the oracle's
    per-walker CE log-prob x the run's 240 000 evaluations."""
    import torch
    from noblegas_rtd_mcmc_amd import workloads as wl
    from noblegas_rtd_mcmc_amd.noble_gas_mcmc import CEModel
    obs = wl.field_data()["obs"]
    runs = []
    for w in wells:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        m = CEModel(obs, [w], max_walkers=4, device=gpu)
        res = m.sample(nwalkers=4, tune=10000, draws=50000, seed=123423, tune_interval=5000)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        per = _oracle_logp_s(m.spec, wl.test_point(m.spec, 1))
        proj = per * 4 * 60000
        runs.append({"run": "%s.CE.4chains" % w, "wall_s": wall, "sample_s": float(res["sampling_time"]),
                     "accept_rate": float(res["accept_rate"]), "us_per_step": 1e6 * float(res["sampling_time"]) / 60000,
                     "oracle_logp_s": per, "oracle_projected_s": proj, "speedup_vs_reference": None,
                     "speedup_vs_oracle_projection": proj / wall})
        if m._lp is not None:
            m._lp.close()
    return {"config": "CEModel([well]).sample(): Ne Ar Kr Xe, DEMetropolisZ (PyMC3's transformed space), 4 chains, "
                      "tune 10 000, draws 50 000, tune_interval 5000, seed 123423 (noble_gas_mcmc.py:408-415)",
            "runs": runs, "total_wall_s": sum(r["wall_s"] for r in runs),
            "reference_total_s_projected": sum(r["oracle_projected_s"] for r in runs)}


def exact_line(args, spec, theta, Wb, C, N):
    """The same step with the surrogate switched off (NGRTD_EXACT_RTD): every unit sums
    its channels over all N ages on the matrix cores."""
    import dataclasses
    import torch
    from noblegas_rtd_mcmc_amd.engine import LogProb
    sx = dataclasses.replace(spec, exact_rtd=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    lx = LogProb(sx, max_walkers=Wb, device=theta.device.index)
    torch.cuda.synchronize()
    build_ms = (time.perf_counter() - t0) * 1e3
    out = torch.empty(Wb, dtype=torch.float64, device=theta.device)
    run = lx.bind(theta, out)
    for _ in range(max(3, args.warmup // 4)):
        run()
    n = max(10, args.steps // 4)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(n):
        run()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / n
    U = spec.n_wells * Wb
    flops = 2.0 * U * C * (N - 1)
    info = lx.info(Wb)
    lx.close()
    return {"exact_value": Wb / (ms * 1e-3),
            "exact_roofline": {"bound": "fp64_mfma", "achieved": flops / (ms * 1e-3) / 1e12,
                               "peak": FP64_PEAK / 1e12, "unit": "TFLOP/s",
                               "frac": flops / (ms * 1e-3) / FP64_PEAK, "kernel": "logp_fused_kernel (exact)",
                               "kernel_ms": ms, "flop_per_launch": flops,
                               "flop_source": "algorithmic: 2 x units x channels x (N - 1), v_mfma_f64_16x16x4 Horner",
                               "surrogate": info.get("surrogate"), "plan_build_ms": build_ms}}


if __name__ == "__main__":
    main()
