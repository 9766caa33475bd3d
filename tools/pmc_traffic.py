#!/usr/bin/env python3
"""HBM traffic per launch from separate rocprofv3 FETCH_SIZE / WRITE_SIZE passes.

  python tools/pmc_traffic.py FETCH_DIR WRITE_DIR --pods N [--out profiles/pmc_latest.json]

Units and gfx950 corrections follow /opt/skills/guides/MI355X_MICROARCH.md (§HBM):
FETCH_SIZE and WRITE_SIZE are KiB; FETCH_SIZE reports exactly 1/2 of the bytes of a coalesced
streaming read on gfx950, so it is doubled; WRITE_SIZE is taken as is.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import load  # noqa: E402


def per_launch(d, counter):
    out, calls = load(d)
    res = {}
    for k, cs in out.items():
        if counter in cs:
            n = max(len(calls[k]), 1)
            res[k] = cs[counter] / n
    return res


def short(name):
    s = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return s.split("(")[0]


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--pods", type=int, required=True)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    f = per_launch(a.fetch_dir, "FETCH_SIZE")
    w = per_launch(a.write_dir, "WRITE_SIZE")
    kern = {}
    for k in sorted(set(f) | set(w)):
        if "at::native" in k or "rocclr" in k:
            continue
        fb = f.get(k, 0.0) * 1024 * 2
        wb = w.get(k, 0.0) * 1024
        kern[short(k)] = {"fetch_bytes_corrected": fb, "write_bytes": wb, "hbm_bytes": fb + wb,
                          "FETCH_SIZE_KiB_raw": f.get(k), "WRITE_SIZE_KiB_raw": w.get(k)}
    score = [v for k, v in kern.items() if k.startswith("rolling_score")]
    res = {"pods": a.pods, "source": {"fetch": a.fetch_dir, "write": a.write_dir},
           "correction": "FETCH_SIZE KiB x1024 x2 (gfx950 half-count), WRITE_SIZE KiB x1024",
           "krca_rolling_score_bytes_per_launch": score[0]["hbm_bytes"] if score else None,
           "kernels": kern}
    txt = json.dumps(res, indent=1)
    if a.out:
        open(a.out, "w").write(txt + "\n")
    print(txt)
