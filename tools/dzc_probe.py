#!/usr/bin/env python3
"""Per-step time of the lane-chain DEMetropolisZ step (dz_chain_kernel) at the reference's own
run shape -- RTD-only, 1 well, 3 chains, N = 25 256, PyMC3's transformed space -- with the logs
the drop-in's sampler keeps (accepted, lp, accept stat), after 1000 tune steps; NGRTD_DZ_DIAG
selects timing-only variants of the step (wrong results; bits in ngrtd_dzc.hpp).  JSON lines.

    [NGRTD_DZ_DIAG=k] python tools/dzc_probe.py [--tracers 4|1] [--model exponential|exp_pist_flow]
        [--phase draw|tune]"""
import argparse
import dataclasses
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tracers", type=int, default=4)
    ap.add_argument("--model", default="exponential")
    ap.add_argument("--chains", type=int, default=3)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--phase", choices=("draw", "tune"), default="draw",
                    help="time draw-phase steps (after 1000 tune steps) or steps inside the tuning phase")
    ap.add_argument("--sections", action="store_true",
                    help="probe build (tools/section_probe.py): shader-clock cycles per section of a step")
    args = ap.parse_args()
    if args.sections:
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__))))
        import section_probe
        section_probe.build()
        os.environ["NGRTD_LIB"] = section_probe.probe_lib(())
    import torch
    from noblegas_rtd_mcmc_amd import workloads as wl
    from noblegas_rtd_mcmc_amd.engine import LogProb
    from noblegas_rtd_mcmc_amd.sampler import DeviceDEMetropolisZ
    tr = ("CFC12", "SF6", "H3", "He4_ter") if args.tracers == 4 else ("H3",)
    sv = "123" if args.tracers == 4 else ""
    spec = dataclasses.replace(wl.rtd_only_spec(L=1, N=25256, tracers=tr, mod_type1=args.model, savenum=sv), jacobian=True)
    W = args.chains
    th = torch.from_numpy(wl.test_point(spec, W)).cuda()
    lp = LogProb(spec, max_walkers=W)
    n = args.steps
    s = DeviceDEMetropolisZ(lp, tune_interval=1000, seed=7, transformed=True, per_well=True)
    n_tune = 1000 if args.phase == "draw" else 1000 + 2 * n
    x, l, z = s.start(th, n_tune, 1000 + 2 * n + 1)
    lp.demcz(x, l, 1000, z)
    acc = torch.empty((n, W), dtype=torch.uint8, device="cuda")
    lpl = torch.empty((n, W), dtype=torch.float64, device="cuda")
    arl = torch.empty((n, W), dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    lp.demcz(x, l, n, z, accepted_log=acc, logp_log=lpl, accept_log=arl)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / n
    res = {"diag": int(os.environ.get("NGRTD_DZ_DIAG", "0")), "tracers": args.tracers, "model": args.model,
           "phase": args.phase, "chains": W, "us_per_step": dt * 1e6}
    if args.sections:   # the last launch's sums, wave 0 (the chains' wave)
        import ctypes as C
        from noblegas_rtd_mcmc_amd import _lib
        rd = _lib.load().ngrtd_probe_read_dzc
        rd.argtypes = [C.c_void_p, C.c_int64]
        buf = np.zeros(16, dtype=np.uint64)
        assert rd(buf.ctypes.data, buf.size) == 0
        ns = max(int(buf[6]), 1)
        names = ("schedule_append", "proposal", "partner_rows", "args_theta", "rtd_like", "decision_logs")
        res["cycles_per_step"] = {k: float(buf[i]) / ns for i, k in enumerate(names)}
        res["cycles_per_step"]["total"] = float(buf[:6].sum()) / ns
        res["launch_steps"] = ns
    print(json.dumps(res))
    lp.close()


if __name__ == "__main__":
    main()
