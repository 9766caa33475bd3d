#!/usr/bin/env python3
"""profiles/pmc_latest.json from an exact-counter report (tools/pmc_exact_report.py output).

  python tools/pmc_latest.py gpurun_out/pmcx/pmc_exact.json [more.json ...] --out profiles/pmc_latest.json

Per kernel: hbm_bytes = DRAM-side read + write bytes per dispatch (TCC_EA0_RDREQ_DRAM_32B and
TCC_EA0_WRREQ_WRITE_DRAM_32B, 32-B units: exact for a streamed 1 GiB read in tools/pmc_calib;
Infinity-Cache hits are included, so for a gathered table that stays on die this is L2-miss
traffic, not HBM traffic).  Later files override earlier ones per section.  bench.py reads
krca_rolling_score_bytes_per_launch into roofline.traffic.
"""
import argparse
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("reports", nargs="+")
    ap.add_argument("--out", required=True)
    ap.add_argument("--pods", type=int, default=1_000_000)
    a = ap.parse_args()
    kern, src = {}, {}
    for f in a.reports:
        rep = json.load(open(f))
        for sec in ("bench", "ppr", "logs", "logs_fused", "tmpl"):
            for k0, e in rep.get(sec, {}).items():
                k = ("fused/" if sec == "logs_fused" else "") + k0  # the KRCA_LOG_FUSED=2 scan's kernels
                if "dram_read_bytes" not in e or "dram_write_bytes" not in e:
                    continue
                if sec.startswith("logs") and e.get("dispatches", 2) < 2:  # (tmpl: one scan per call too)
                    continue  # the sizing call's first-scan kernels (log_lines ...), not the scan's
                if k0.startswith("at::") or k0.startswith("__amd") or k0.startswith("elementwise"):
                    continue  # torch / runtime setup kernels
                kern[k] = {"section": sec, "dram_read_bytes": e["dram_read_bytes"],
                           "dram_write_bytes": e["dram_write_bytes"],
                           "hbm_bytes": e["dram_read_bytes"] + e["dram_write_bytes"],
                           "fabric_read_request_bytes": e.get("read_bytes"), "fabric_write_bytes": e.get("write_bytes")}
                src[k] = f
    score = [v["hbm_bytes"] for k, v in kern.items() if k.startswith("rolling_score")]
    out = {"pods": a.pods, "source": src,
           "counters": "hbm_bytes = 32 * (TCC_EA0_RDREQ_DRAM_32B + TCC_EA0_WRREQ_WRITE_DRAM_32B) per dispatch (median)",
           "krca_rolling_score_bytes_per_launch": score[0] if score else None, "kernels": kern}
    open(a.out, "w").write(json.dumps(out, indent=1, sort_keys=True) + "\n")
    print(json.dumps({k: round(v["hbm_bytes"] / 1e6, 2) for k, v in kern.items()}, indent=1))


if __name__ == "__main__":
    main()
