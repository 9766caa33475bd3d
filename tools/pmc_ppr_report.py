#!/usr/bin/env python3
"""PMC report for the PageRank step: FETCH_SIZE calibrated on tools/pmc_calib's known byte counts.

  python tools/pmc_ppr_report.py gpurun_out/pmc2 [--out profiles/r2/pmc_ppr.json]
"""
import argparse
import csv
import json
import os
from collections import defaultdict


def counters(path):
    """kernel short name -> counter -> list of per-dispatch values."""
    out = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(os.path.join(path, "run_counter_collection.csv"))):
        name = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
        out[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return out


def med(v):
    v = sorted(v)
    return v[len(v) // 2] if v else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("d")
    ap.add_argument("--out")
    a = ap.parse_args()
    res = {"calibration": {}, "ppr_step": {}}
    cf, cw, ce, ct = (counters(os.path.join(a.d, n)) for n in ("cal_fetch", "cal_write", "cal_ea", "cal_tcc"))
    gathers = 1 << 24
    # gather8 launches in order: big (16M distinct lines), l3 (8 MiB table), run (2M distinct lines)
    g = cf["gather8"]["FETCH_SIZE"]
    res["calibration"] = {
        "stream16_1GiB": {"FETCH_SIZE_KiB": med(cf["stream16"]["FETCH_SIZE"]), "known_KiB": (1 << 30) / 1024,
                          "bytes_per_KiB_counted": (1 << 30) / (med(cf["stream16"]["FETCH_SIZE"]) * 1024)},
        "gather8_big_16M_lines": {"FETCH_SIZE_KiB": g[0], "bytes_counted_per_gather": g[0] * 1024 / gathers,
                                  "note": "includes the 64 MiB index stream (4 B per gather, coalesced)"},
        "gather8_l3_8MiB_table": {"FETCH_SIZE_KiB": g[1], "bytes_counted_per_gather": g[1] * 1024 / gathers},
        "gather8_run8_2M_lines": {"FETCH_SIZE_KiB": g[2], "bytes_counted_per_gather": g[2] * 1024 / gathers},
        "TCC_EA0_RDREQ": ce["gather8"].get("TCC_EA0_RDREQ_sum"), "TCC_EA0_RDREQ_32B": ce["gather8"].get(
            "TCC_EA0_RDREQ_32B_sum"),
        "TCC_HIT": ct["gather8"].get("TCC_HIT_sum"), "TCC_MISS": ct["gather8"].get("TCC_MISS_sum"),
    }
    pf, pw, pe, pt, ps = (counters(os.path.join(a.d, n)) for n in ("ppr_fetch", "ppr_write", "ppr_ea", "ppr_tcc",
                                                                     "ppr_sq"))
    for k in pf:
        if not k.startswith("ppr_step"):
            continue
        f, w = med(pf[k]["FETCH_SIZE"]), med(pw[k]["WRITE_SIZE"])
        res["ppr_step"][k] = {
            "dispatches": len(pf[k]["FETCH_SIZE"]), "FETCH_SIZE_KiB_median": f, "WRITE_SIZE_KiB_median": w,
            "TCC_EA0_RDREQ_median": med(pe[k]["TCC_EA0_RDREQ_sum"]),
            "TCC_EA0_RDREQ_32B_median": med(pe[k]["TCC_EA0_RDREQ_32B_sum"]),
            "TCC_HIT_median": med(pt[k]["TCC_HIT_sum"]), "TCC_MISS_median": med(pt[k]["TCC_MISS_sum"]),
            "SQ": {c: med(v) for c, v in ps[k].items()},
        }
    txt = json.dumps(res, indent=1)
    if a.out:
        open(a.out, "w").write(txt + "\n")
    print(txt)


if __name__ == "__main__":
    main()
