#!/usr/bin/env python3
"""Per-kernel register / spill / scratch / occupancy table of one HIP source, from the
compiler's kernel-resource-usage remarks (no GPU needed).
    python tools/resource_usage.py [SOURCE] [--filter SUBSTR] [-D NAME=VAL ...]"""
import argparse
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("source", nargs="?", default=os.path.join(REPO, "noblegas_rtd_mcmc_amd", "csrc", "ngrtd_dz.hip"))
    ap.add_argument("--filter", default="logp_fused_kernel")
    ap.add_argument("-D", action="append", default=[])
    args = ap.parse_args()
    import __graft_entry__ as g
    flags = g.HIPCC_FLAGS + g.EXTRA_FLAGS.get(os.path.basename(args.source), []) + ["-D" + d for d in args.D]
    out = subprocess.run(["hipcc"] + flags + ["-Rpass-analysis=kernel-resource-usage", "-c", "-o", "/dev/null",
                                              os.path.abspath(args.source)], capture_output=True, text=True, cwd="/tmp")
    rows, cur = [], None
    for line in out.stderr.splitlines():
        m = re.search(r"remark:\s+(Function Name|VGPRs|AGPRs|SGPRs|SGPRs Spill|VGPRs Spill|ScratchSize \[bytes/lane\]|"
                      r"Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\S+)", line)
        if not m:
            continue
        k, v = m.group(1), m.group(2)
        if k == "Function Name":
            cur = {"name": v}
            rows.append(cur)
        elif cur is not None:
            cur[k.split(" [")[0]] = v
    if out.returncode:
        sys.stderr.write(out.stderr[-3000:])
        raise SystemExit(out.returncode)
    for r in rows:
        if args.filter in r["name"]:
            m = re.search(r"ILi(\d+)ELb(\d)ELi(\d+)ELi(\d+)E", r["name"])
            nm = "logp_fused<%s,%s,%s,%s>" % m.groups() if m else r["name"][:60]
            print("%-28s VGPR %4s  SGPR %4s  SGPRspill %4s  VGPRspill %4s  scratch %4s  occ %s" % (
                nm, r.get("VGPRs"), r.get("SGPRs"), r.get("SGPRs Spill"), r.get("VGPRs Spill"), r.get("ScratchSize"),
                r.get("Occupancy")))


if __name__ == "__main__":
    main()
