#!/usr/bin/env python3
"""MFMA utilisation of the correlation kernels from tools/gpu_pmc_mfma.sh's passes.

  python tools/pmc_mfma_report.py gpurun_out/<tag> [--out F]

Per kernel and pod count (median over the dispatches of the timed call; the warm-up call's are
the first half): duration (kernel trace), the held clock GRBM_GUI_ACTIVE / 8 XCDs / duration,
MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / 1024 SIMDs / (GRBM_GUI_ACTIVE / 8) (the fraction of the
SIMD cycles the matrix pipe was busy, at the clock the chip held), the same against the 2.4 GHz
nameplate clock, and DRAM-side bytes = 32 B x (TCC_EA0_RDREQ_DRAM_32B + TCC_EA0_WRREQ_WRITE_DRAM_32B).
"""
import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict


def short(k):
    return k.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]


def load(d):
    cnt = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))  # kernel -> counter -> dispatch -> v
    dur = defaultdict(dict)  # kernel -> dispatch -> ns
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            cnt[short(r["Kernel_Name"])][r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            dur[short(r["Kernel_Name"])][r["Dispatch_Id"]] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    return cnt, dur


def med(v):
    v = sorted(v)
    return v[len(v) // 2] if v else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("d")
    ap.add_argument("--out")
    a = ap.parse_args()
    res = {}
    pods_seen = sorted({int(m.group(1)) for p in os.listdir(a.d) for m in [re.match(r"p(\d+)_pass1$", p)] if m})
    for pods in pods_seen:
        c1, d1 = load(os.path.join(a.d, f"p{pods}_pass1"))
        c2, _ = load(os.path.join(a.d, f"p{pods}_pass2"))
        out = {}
        for k in c1:
            if not k.startswith("corr"):
                continue
            ds = sorted(c1[k].get("GRBM_GUI_ACTIVE", {}).keys(), key=int)
            ds = ds[len(ds) // 2:] if len(ds) > 1 else ds  # the timed call's dispatches
            if not ds:
                continue
            g = {n: med([c1[k][n][x] for x in ds if x in c1[k][n]]) for n in c1[k]}
            g.update({n: med(list(c2[k][n].values())[len(c2[k][n]) // 2:] or list(c2[k][n].values()))
                      for n in c2.get(k, {})})
            ns = med([d1[k][x] for x in ds if x in d1.get(k, {})])
            e = {"dispatches_per_call": len(ds), "ms": ns / 1e6 if ns else None, "counters": g}
            if ns and g.get("GRBM_GUI_ACTIVE"):
                cyc = g["GRBM_GUI_ACTIVE"] / 8.0
                e["clock_ghz"] = cyc / ns
                if g.get("SQ_VALU_MFMA_BUSY_CYCLES") is not None:
                    e["mfma_busy_at_held_clock"] = g["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024.0 / cyc
                    e["mfma_busy_vs_2p4ghz"] = g["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024.0 / (2.4 * ns)
            if g.get("TCC_EA0_RDREQ_DRAM_32B") is not None:
                e["dram_bytes"] = 32.0 * (g["TCC_EA0_RDREQ_DRAM_32B"] + g.get("TCC_EA0_WRREQ_WRITE_DRAM_32B", 0.0))
                rd, wr = c2[k]["TCC_EA0_RDREQ_DRAM_32B"], c2[k].get("TCC_EA0_WRREQ_WRITE_DRAM_32B", {})
                d2 = sorted(rd.keys(), key=int)
                d2 = d2[len(d2) // 2:] if len(d2) > 1 else d2  # the timed call's dispatches
                e["dram_bytes_call_total"] = 32.0 * sum(rd[x] + wr.get(x, 0.0) for x in d2)
            out[k] = e
        res[str(pods)] = out
    txt = json.dumps(res, indent=1, sort_keys=True)
    if a.out:
        open(a.out, "w").write(txt + "\n")
    for pods, ks in res.items():
        for k, e in sorted(ks.items(), key=lambda kv: -(kv[1].get("ms") or 0) * kv[1]["dispatches_per_call"]):
            print(f"{pods:>8} {k[:60]:60s} n={e['dispatches_per_call']:3d} ms={e.get('ms') or 0:8.3f} "
                  f"clk={e.get('clock_ghz', 0):.2f} mfma={e.get('mfma_busy_at_held_clock', 0):.3f} "
                  f"(vs 2.4GHz {e.get('mfma_busy_vs_2p4ghz', 0):.3f}) dram={e.get('dram_bytes', 0) / 1e9:.2f} GB")


if __name__ == "__main__":
    main()
