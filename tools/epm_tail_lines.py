"""Model of the exp_pist_flow block-tail table's L2 traffic at the c4 shape (CPU only).

Each unit of an exp_pist_flow plan reads ONE entry of the block-tail surrogate table
(ngrtd.hip epm_prepare; [block b - 1][piece p][kChebN][C] doubles): block b = m / S + 1 from
its first unmasked age m (tp_m >= tau (1 - 1/eta)), piece p from tau' = tau / eta.  The
dispatcher deals walker blocks to the 8 XCDs (logp_fused_kernel's XCD-aware numbering: XCD x
runs walkers [x W/8, (x+1) W/8)), and every XCD's L2 misses each 128-B line its units touch
once.  This script draws the bench's prior ensemble (seed 34568, as bench.py's model lines),
maps every unit to its entry and counts

  * the entries the ensemble reaches at all (the table holds blocks x pieces of the window),
  * the distinct 128-B lines per XCD: the compulsory L2 misses of one launch.

    python tools/epm_tail_lines.py [--walkers 2048] [--wells 64]
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

S, CHEB_N, EPM_OCT0, SUB = 16, 12, -4, 4     # kEpmBlock, kChebN, kEpmOct0, kChebSub (ngrtd_device.hpp)


def piece(tp):
    """epm_piece of tau' (binary octave, kChebSub pieces per octave), no tail piece needed here."""
    e = np.floor(np.log2(tp)).astype(np.int64)
    j = np.floor((tp / np.exp2(e) - 1.0) * SUB).astype(np.int64)
    return (e - EPM_OCT0) * SUB + j


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--walkers", type=int, default=2048)
    ap.add_argument("--wells", type=int, default=64)
    ap.add_argument("--ages", type=int, default=1200)
    args = ap.parse_args()
    from noblegas_rtd_mcmc_amd import workloads
    W, L, N, C = args.walkers, args.wells, args.ages, 5
    spec = workloads.c4_spec(L=L, N=N, mod_type1="exp_pist_flow",
                             par_names=workloads.model_par_names("exp_pist_flow", None, ""))
    th = workloads.sample_prior(spec, W, np.random.default_rng(34568))
    roles = list(spec.roles)
    tau, eta = th[roles.index("tau1")], th[roles.index("eta1")]          # [L][W]
    tpk = np.arange(N) + 0.5                                              # the yearly grid's ages
    m = np.minimum(np.searchsorted(tpk, tau * (1.0 - 1.0 / eta), side="left"), N - 1)
    b = m // S + 1
    has_tail = b * S < N
    p = piece(tau / eta)
    nb = (N - 1) // S
    p0, p1 = int(p[has_tail].min()), int(p[has_tail].max())
    npc = p1 - p0 + 1
    ent_bytes = CHEB_N * C * 8
    entry = (b - 1) * npc + (p - p0)
    blocks = W // (512 // L)                                              # walker blocks of 512 / L walkers
    xcd = (np.arange(W) // (512 // L)) // max(1, blocks // 8)
    per = []
    for x in range(8):
        e = np.unique(entry[has_tail & (xcd == x)[None, :]])
        lines = set()
        for v in e.tolist():
            o = v * ent_bytes
            lines.update(range(o // 128, (o + ent_bytes - 1) // 128 + 1))
        per.append(len(lines) * 128)
    reach = np.unique(entry[has_tail])
    out = {"units": int(tau.size), "units_with_tail": int(has_tail.sum()), "blocks": nb, "pieces": npc,
           "table_bytes": nb * npc * ent_bytes, "entry_bytes": ent_bytes, "entries_reached": int(reach.size),
           "reached_bytes": int(reach.size) * ent_bytes, "per_xcd_line_bytes": per,
           "l2_miss_bytes_per_launch": int(sum(per))}
    import json
    print(json.dumps(out))


if __name__ == "__main__":
    main()
