#!/usr/bin/env python3
"""profiles/pmc_mfma_latest.json from tools/pmc_mfma_report.py output (the correlation's counters).

  python tools/pmc_mfma_latest.py gpurun_out/<tag>/pmcmfma/pmc_mfma.json --src <tag> --out profiles/pmc_mfma_latest.json

Per pod count: the DRAM-side bytes of one krca_corr_prepare + krca_corr_topk call (sum over its
kernels of dispatches x median bytes per dispatch; 32 B x (TCC_EA0_RDREQ_DRAM_32B +
TCC_EA0_WRREQ_WRITE_DRAM_32B), Infinity-Cache hits included) and the main pass's MFMA-busy fraction
at the clock the chip held (SQ_VALU_MFMA_BUSY_CYCLES / 1024 SIMDs / (GRBM_GUI_ACTIVE / 8)), that clock,
and the same busy cycles against the 2.4 GHz nameplate.  bench.py's corr leg reads it into
corr.roofline (traffic, mfma_busy)."""
import argparse
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("report")
    ap.add_argument("--src", required=True)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    rep = json.load(open(a.report))
    out = {"source": a.src, "counters": "tools/gpu_pmc_mfma.sh passes; tools/pmc_mfma_report.py", "pods": {}}
    for pods, ks in rep.items():
        tot = sum(e.get("dram_bytes_call_total", e.get("dram_bytes", 0.0) * e["dispatches_per_call"]) for e in ks.values())
        main_k = [k for k in ks if k.startswith("corr_tiles") and ", 0, " in k]
        m = ks[main_k[0]] if main_k else {}
        out["pods"][pods] = {
            "dram_bytes_per_call": tot,
            "main_pass": {"kernel": main_k[0] if main_k else None, "batches": m.get("dispatches_per_call"),
                          "ms_per_batch_serialised": m.get("ms"), "clock_ghz": m.get("clock_ghz"),
                          "mfma_busy_at_held_clock": m.get("mfma_busy_at_held_clock"),
                          "mfma_busy_vs_2p4ghz": m.get("mfma_busy_vs_2p4ghz"), "dram_bytes_per_batch": m.get("dram_bytes")},
            "kernels": {k: {"dispatches": e["dispatches_per_call"], "ms": e.get("ms"), "dram_bytes": e.get("dram_bytes"),
                            "mfma_busy_at_held_clock": e.get("mfma_busy_at_held_clock")} for k, e in ks.items()}}
    open(a.out, "w").write(json.dumps(out, indent=1, sort_keys=True) + "\n")
    print(json.dumps({p: (v["dram_bytes_per_call"] / 1e9, v["main_pass"]["mfma_busy_at_held_clock"])
                      for p, v in out["pods"].items()}))


if __name__ == "__main__":
    main()
