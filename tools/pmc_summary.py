#!/usr/bin/env python3
"""Sum rocprofv3 --pmc counter_collection.csv values per kernel (name prefix match).

  python tools/pmc_summary.py DIR [kernel-substring]
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(d):
    out = defaultdict(lambda: defaultdict(float))
    calls = defaultdict(set)
    files = [d] if os.path.isfile(d) else glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    for f in files:
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            out[k][r["Counter_Name"]] += float(r["Counter_Value"])
            calls[k].add(r.get("Dispatch_Id") or r.get("Correlation_Id"))
    return out, calls


if __name__ == "__main__":
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    out, calls = load(sys.argv[1])
    for k, cs in out.items():
        if sub in k:
            n = max(len(calls[k]), 1)
            print(k[:90], "dispatches", n)
            for c, v in sorted(cs.items()):
                print(f"   {c:28s} {v / n:16.4g} per dispatch")
