#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel-trace database (or CSV) into a per-kernel stats table."""
import csv
import json
import sqlite3
import sys
from collections import defaultdict


def load(path):
    rows = []
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        for name, dur, vgpr, sgpr, lds, scr, gx, wx in c.execute(
                "select name, duration, vgpr_count, sgpr_count, lds_size, scratch_size, grid_x, workgroup_x from kernels"):
            rows.append((name, dur, vgpr, sgpr, lds, scr, gx // max(wx, 1)))
    else:
        with open(path) as f:
            for r in csv.DictReader(f):
                rows.append((r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"]),
                             r.get("VGPR_Count"), r.get("SGPR_Count"), r.get("LDS_Block_Size"),
                             r.get("Scratch_Size"), None))
    return rows


def summarize(rows):
    agg = defaultdict(lambda: [0, 0, None, None, None, None, None])
    for name, dur, vgpr, sgpr, lds, scr, nwg in rows:
        a = agg[name]
        a[0] += 1
        a[1] += dur
        a[2:] = [vgpr, sgpr, lds, scr, nwg]
    tot = sum(a[1] for a in agg.values())
    out = []
    for name, (n, d, vgpr, sgpr, lds, scr, nwg) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        out.append(dict(kernel=name, calls=n, total_ms=d / 1e6, avg_us=d / n / 1e3, pct=100.0 * d / tot,
                        vgpr=vgpr, sgpr=sgpr, lds=lds, scratch=scr, workgroups=nwg))
    return out


if __name__ == "__main__":
    s = summarize(load(sys.argv[1]))
    if len(sys.argv) > 2:
        json.dump(s, open(sys.argv[2], "w"), indent=1)
    print(f"{'kernel':70s} {'calls':>6s} {'avg_us':>10s} {'total_ms':>10s} {'pct':>6s} vgpr lds")
    for r in s:
        print(f"{r['kernel'][:70]:70s} {r['calls']:6d} {r['avg_us']:10.2f} {r['total_ms']:10.3f} {r['pct']:6.1f} "
              f"{r['vgpr']} {r['lds']}")
