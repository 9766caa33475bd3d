#!/usr/bin/env python3
"""A/B of the krca_rolling_score kernel variants on one tensor (C4 shape by default).

Every variant must produce bit-identical outputs (same arithmetic); prints per-variant event
timings and the equality check against the first variant.
  python tools/score_ab.py [--pods 1000000] [--reps 5]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kubernetes-rca-system_amd"))

VARIANTS = [("ring_buf", {"KRCA_SCORE_IMPL": 2}), ("ring", {"KRCA_SCORE_IMPL": 1})] + [
    (f"pipe_c{c}", {"KRCA_SCORE_IMPL": 0, "KRCA_SCORE_CHUNK": c}) for c in (10, 12, 15, 20, 30)] + [
    ("pipe_c20_default_policy", {"KRCA_SCORE_IMPL": 0, "KRCA_SCORE_CHUNK": 20, "KRCA_SCORE_NT": 0}),
    ("lds", {"KRCA_SCORE_IMPL": 5}), ("lds_default_policy", {"KRCA_SCORE_IMPL": 5, "KRCA_SCORE_NT": 0})]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pods", type=int, default=1_000_000)
    ap.add_argument("--tsteps", type=int, default=1440)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--only", default="")
    ap.add_argument("--rounds", type=int, default=1, help="alternate the selected variants this many times")
    a = ap.parse_args()
    import torch
    from krca import native, synth
    eng = native.NativeEngine(0)
    x = synth.make_metrics(a.pods, 8, a.tsteps, device="cuda")
    nbytes = 4 * a.pods * 8 * a.tsteps + 4 * a.pods * 8 + 9 * a.pods
    ref = None
    res = []
    defaults = {"KRCA_SCORE_IMPL": 0, "KRCA_SCORE_CHUNK": 20, "KRCA_SCORE_NT": 1}
    for rnd in range(a.rounds):
        for name, knobs in VARIANTS:
            if a.only and name not in a.only.split(","):
                continue
            # knobs are read once at library load: set them through krca_tune_set
            with native.tune(eng.lib, **dict(defaults, **knobs)):
                variant = native.SCORE_VARIANTS[eng.lib.krca_rolling_score_variant(a.pods, 8, a.tsteps, 60)]
                o = eng.rolling_score_device(x)
                torch.cuda.synchronize()
                ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.reps)]
                for s, e in ev:
                    s.record()
                    eng.rolling_score_device(x, out=o)
                    e.record()
                torch.cuda.synchronize()
            ms = [s.elapsed_time(e) for s, e in ev]
            out = {k: v.clone() for k, v in o.items()}
            same = None
            if ref is None:
                ref = out
            else:
                same = all(torch.equal(ref[k], out[k]) for k in ref)
            r = dict(variant=name, kernel=variant, round=rnd, ms=[round(m, 4) for m in ms], ms_avg=sum(ms) / len(ms),
                     ms_min=min(ms), tbs_avg=nbytes / (sum(ms) / len(ms) * 1e-3) / 1e12, identical_to_first=same)
            res.append(r)
            print(json.dumps(r), flush=True)
            del out


if __name__ == "__main__":
    main()
