#!/usr/bin/env python3
"""Average each PMC counter per kernel over dispatches: python tools/pmc_summary.py DIR..."""
import collections
import csv
import glob
import os
import sys


def summarize(dirs):
    agg = collections.defaultdict(list)
    dur = collections.defaultdict(list)
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"]
                agg[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
                dur[(k, r["Counter_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
    out = collections.defaultdict(dict)
    for (k, c), v in agg.items():
        out[k][c] = sum(v) / len(v)
        out[k]["dur_us[" + c + "]"] = sum(dur[(k, c)]) / len(dur[(k, c)])
    return out


if __name__ == "__main__":
    res = summarize(sys.argv[1:])
    for k, d in res.items():
        if "ngrtd" not in k:
            continue
        print(k[:70])
        for c, v in sorted(d.items()):
            if not c.startswith("dur"):
                print("   %-24s %14.1f" % (c, v))
