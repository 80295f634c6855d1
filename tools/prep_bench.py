#!/usr/bin/env python3
"""Prep-stage ensemble propagation benchmark: the He ensembles of
age_modeling_mcmc.prep.py:356-397 (50 000 CE posterior members x wells x 8 Rterr passes of
ng_parse.He_comps) and the CFC / SF6 pptv ensembles (:247-305), on device memory through
ngrtd_he_comps / ngrtd_cfc_corr, timed with HIP events.  Both kernels are elementwise and
HBM-bound; the line reports achieved GB/s of their algorithmic bytes (He_comps: 7 inputs +
5 outputs = 96 B per member; CFC x3: 7 + 3 outputs... see DESIGN.md).  The CPU baseline is
the per-member oracle loop (the reference builds one Python object per member).

    python tools/prep_bench.py [--members 50000] [--wells 3]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--members", type=int, default=50000)
    ap.add_argument("--wells", type=int, default=3)
    ap.add_argument("--passes", type=int, default=8)
    ap.add_argument("--big", type=int, default=1 << 24, help="members for the bandwidth line")
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    import torch
    from noblegas_rtd_mcmc_amd import _lib
    from oracle import prep as oprep

    ctx = _lib.Context.get(0)
    ctx.set_stream(torch.cuda.current_stream().cuda_stream)
    p = lambda t: C.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731

    def inputs(n, seed):
        rng = np.random.default_rng(seed)
        h = dict(He4=rng.normal(6e-8, 2e-8, n), He3=rng.normal(1e-13, 3e-14, n), Ae=10 ** rng.uniform(-4, -1, n),
                 F=rng.uniform(0, 1, n), E=rng.uniform(2500, 3400, n), T=rng.uniform(0, 15, n),
                 Rterr=10 ** (rng.beta(2, 2, n) * 2 + np.log10(2e-8) - 1), x=rng.uniform(0.2, 3.0, (3, n)))
        return h, {k: torch.from_numpy(np.ascontiguousarray(v)).cuda() for k, v in h.items()}

    def he(dv, n, out):
        ctx.check(ctx.lib.ngrtd_he_comps(ctx.h, *[p(dv[k]) for k in ("He4", "He3", "Ae", "F", "E", "T", "Rterr")],
                                         0.0, n, p(out), _lib.MEM_DEVICE), "he_comps")

    ids = (C.c_int32 * 3)(0, 1, 2)

    def cfc(dv, n, out):
        ctx.check(ctx.lib.ngrtd_cfc_corr(ctx.h, 0, ids, 3, p(dv["E"]), p(dv["T"]), p(dv["Ae"]), p(dv["F"]), None,
                                         None, p(dv["x"]), n, p(out), _lib.MEM_DEVICE), "cfc_corr")

    def timed(fn, reps):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps

    # (1) the prep.py workload: members x wells x passes He_comps + members x wells CFC
    n = args.members * args.wells
    h, dv = inputs(n, 1)
    out_he = torch.empty(5, n, dtype=torch.float64, device="cuda")
    out_cfc = torch.empty(3, n, dtype=torch.float64, device="cuda")
    ms_prep = timed(lambda: [he(dv, n, out_he) for _ in range(args.passes)] + [cfc(dv, n, out_cfc)], 5)
    ref = oprep.he_comps(h["He4"], h["He3"], h["Ae"], h["F"], h["E"], h["T"], h["Rterr"])
    got = out_he.cpu().numpy()
    err = max(np.max(np.abs(got[0] - ref["He4_eq"]) / np.abs(ref["He4_eq"])),
              np.max(np.abs(got[1] - ref["He4_atm"]) / np.abs(ref["He4_atm"])))
    # CPU: per-member loop of the oracle (the reference's one-object-per-member loop)
    t0 = time.perf_counter()
    m = 0
    while time.perf_counter() - t0 < 5.0:
        i = m % n
        oprep.he_comps(h["He4"][i], h["He3"][i], h["Ae"][i], h["F"][i], h["E"][i], h["T"][i], h["Rterr"][i])
        m += 1
    cpu_per_s = m / (time.perf_counter() - t0)
    # (2) bandwidth line at a size that fills the chip
    nb = args.big
    _, db = inputs(nb, 2)
    ob = torch.empty(5, nb, dtype=torch.float64, device="cuda")
    oc = torch.empty(3, nb, dtype=torch.float64, device="cuda")
    ms_he = timed(lambda: he(db, nb, ob), args.reps)
    ms_cfc = timed(lambda: cfc(db, nb, oc), args.reps)
    he_bytes, cfc_bytes = 12 * 8.0, (4 + 3 + 3) * 8.0
    print(json.dumps({
        "workload": "prep.py He ensembles: %d members x %d wells x %d passes He_comps + CFC11/12/113 pptv"
                    % (args.members, args.wells, args.passes),
        "prep_ms": ms_prep, "he_comps_per_s": n * args.passes / (ms_prep * 1e-3),
        "cpu_baseline": {"value": cpu_per_s, "unit": "He_comps members/s", "cores": 1, "kind": "port",
                         "sample": "%d per-member oracle/prep.py he_comps calls, 5 s" % m},
        "max_rel_err_vs_oracle": float(err),
        "he_comps_big": {"members": nb, "ms": ms_he, "bytes_per_member": he_bytes,
                         "GBps": nb * he_bytes / (ms_he * 1e-3) / 1e9},
        "cfc_corr_big": {"members": nb, "ms": ms_cfc, "bytes_per_member": cfc_bytes,
                         "GBps": nb * cfc_bytes / (ms_cfc * 1e-3) / 1e9}}), flush=True)
    assert err <= 1e-12


if __name__ == "__main__":
    main()
