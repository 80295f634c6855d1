#!/usr/bin/env python3
"""Per-kernel durations of the longest back-to-back run of one kernel in a rocprofv3
--kernel-trace CSV (bench.py's timed region: K launches with no gap above --gap us), next to
the all-launch average rocprofv3 --stats reports (which also counts the untimed probe,
warm-up and host-staged launches).
    python tools/trace_region.py TRACE.csv [--kernel SUBSTR] [--gap 20]"""
import argparse
import csv
import json
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--kernel", default="logp_fused_kernel<5, true, 2, 0>")
    ap.add_argument("--gap", type=float, default=20.0, help="max idle gap inside a run (us)")
    args = ap.parse_args()
    rows = sorted((r for r in csv.DictReader(open(args.trace)) if args.kernel in r["Kernel_Name"]),
                  key=lambda r: int(r["Start_Timestamp"]))
    st = [int(r["Start_Timestamp"]) for r in rows]
    en = [int(r["End_Timestamp"]) for r in rows]
    dur = [(b - a) / 1e3 for a, b in zip(st, en)]
    runs, cur = [], [0]
    for i in range(1, len(rows)):
        if st[i] - en[i - 1] < args.gap * 1e3:
            cur.append(i)
        else:
            runs.append(cur)
            cur = [i]
    runs.append(cur)
    out = {"kernel": args.kernel, "launches": len(rows), "mean_all_us": statistics.mean(dur),
           "runs": [{"launches": len(r), "mean_us": statistics.mean(dur[i] for i in r),
                     "median_us": statistics.median(dur[i] for i in r),
                     "span_per_launch_us": (en[r[-1]] - st[r[0]]) / 1e3 / len(r)} for r in runs if len(r) >= 10]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
