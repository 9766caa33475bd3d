#!/usr/bin/env python3
"""Exact per-dispatch HBM-side bytes from the request-size counters (tools/gpu_pmc_exact.sh).

  python tools/pmc_exact_report.py gpurun_out/pmcx [--out profiles/r2/pmc_exact.json]

For every kernel: L2->fabric read bytes (32/64/128-B requests: RDREQ_32B, RDREQ - RDREQ_32B -
BUBBLE, BUBBLE), fabric write bytes (WRREQ_64B at 64 B, the rest at 32 B), and the DRAM-side
bytes (RDREQ_DRAM_32B, WRREQ_WRITE_DRAM_32B, 32-B units; Infinity-Cache hits excluded), as the
median over dispatches of the same kernel.  Per-instance counters are summed per dispatch.
"""
import argparse
import csv
import json
import os
from collections import defaultdict


def load(path):
    """kernel -> counter -> {dispatch: value}"""
    out = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))
    f = os.path.join(path, "run_counter_collection.csv")
    if not os.path.exists(f):
        return out
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
        out[k][r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    return out


def med(d):
    v = sorted(d.values())
    return v[len(v) // 2] if v else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("d")
    ap.add_argument("--out")
    a = ap.parse_args()
    res = {}
    for t in ("cal", "ppr", "bench", "logs", "logs_fused", "logs250k", "tmpl", "corr"):
        if not any(os.path.isdir(os.path.join(a.d, f"{t}_{p}")) for p in ("rd", "dram", "wr")):
            continue
        rd, dr, wr = (load(os.path.join(a.d, f"{t}_{p}")) for p in ("rd", "dram", "wr"))
        kern = {}
        for k in set(rd) | set(dr) | set(wr):
            c = {n: med(v) for n, v in {**rd[k], **dr[k], **wr[k]}.items()}
            rq, bub, r32 = c.get("TCC_EA0_RDREQ_sum"), c.get("TCC_BUBBLE_sum"), c.get("TCC_EA0_RDREQ_32B_sum")
            e = {"dispatches": len(next(iter(rd[k].values()), {})), "counters": c}
            if None not in (rq, bub, r32):
                e["read_bytes"] = 32 * r32 + 64 * (rq - r32 - bub) + 128 * bub
            w, w64 = c.get("TCC_EA0_WRREQ_sum"), c.get("TCC_EA0_WRREQ_64B_sum")
            if None not in (w, w64):
                e["write_bytes"] = 64 * w64 + 32 * (w - w64)
            if c.get("TCC_EA0_RDREQ_DRAM_32B") is not None:
                e["dram_read_bytes"] = 32 * c["TCC_EA0_RDREQ_DRAM_32B"]
            if c.get("TCC_EA0_WRREQ_WRITE_DRAM_32B") is not None:
                e["dram_write_bytes"] = 32 * c["TCC_EA0_WRREQ_WRITE_DRAM_32B"]
            kern[k] = e
        res[t] = kern
    txt = json.dumps(res, indent=1, sort_keys=True)
    if a.out:
        open(a.out, "w").write(txt + "\n")
    for t, ks in res.items():
        print(f"== {t}")
        for k, e in sorted(ks.items()):
            f = lambda x: "-" if x is None else f"{x / 1e6:10.2f}"  # noqa: E731
            print(f"  {k[:48]:48s} rd {f(e.get('read_bytes'))} MB  wr {f(e.get('write_bytes'))} MB  "
                  f"dram rd {f(e.get('dram_read_bytes'))} MB  dram wr {f(e.get('dram_write_bytes'))} MB")


if __name__ == "__main__":
    main()
