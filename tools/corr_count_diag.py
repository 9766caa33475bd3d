"""Diagnose exact-count mismatches of krca_corr_topk on one configuration: the number of pods whose
|r| > tau count falls outside the float64 band, under several A/B knobs (GPU; tools only)."""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kubernetes-rca-system_amd"))
from krca import native, synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--pods", type=int, default=30000)
ap.add_argument("--T", type=int, default=1437)
ap.add_argument("--k", type=int, default=16)
ap.add_argument("--tau", type=float, default=0.6)
a = ap.parse_args()
eng = native.NativeEngine()
lib = eng.lib
x = synth.make_metrics(a.pods, 1, a.T, seed=a.T, group_size=20, device="cuda")
# the device's standardised rows (bit-identical to the C twin's: test_corr_prepare_matches_twin)
z = eng.corr_prepare_device(x)["z32"].double()
BAND = 1e-12


def bad_counts(res):
    cnt_all = torch.from_numpy(res["count"]).cuda()
    bad = []
    for r0 in range(0, a.pods, 2048):
        rr = torch.arange(r0, min(a.pods, r0 + 2048), device="cuda")
        R = z[rr] @ z.T
        R[torch.arange(len(rr), device="cuda"), rr] = 0.0
        A = R.abs()
        lo, hi = (A > a.tau + BAND).sum(1), (A > a.tau - BAND).sum(1)
        c = cnt_all[rr]
        m = (c < lo) | (c > hi)
        for i in torch.nonzero(m).flatten().tolist():
            bad.append((r0 + i, int(c[i]), int(lo[i]), int(hi[i])))
    return bad


for knobs in ({}, {"KRCA_CORR_PROJ": 0}, {"KRCA_CORR_RS_Q16": 0}, {"KRCA_CORR_RS_GROUP": 0},
              {"KRCA_CORR_AMB_TILE": 0}, {"KRCA_CORR_BATCH": 3}):
    with native.tune(lib, **knobs):
        res = eng.corr_topk(x, k=a.k, tau=a.tau)
    b = bad_counts(res)
    print(knobs, "bad", len(b), b[:4], flush=True)

# the pairs of the bad pods whose exact |r| clears tau but whose fp16 screening value does not clear
# tau + eps (so they were decided by the band logic or missed)
z2 = eng.corr_prepare_device(x)
zh = z2["zh"][:a.pods, :].view(torch.float16).double()[:, :a.T]
res = eng.corr_topk(x, k=a.k, tau=a.tau)
b = bad_counts(res)
T = a.T
eps = 2.0 ** -10 * 1.001 + T * 2.0 ** -24 + (T ** 0.5) * 2.0 ** -23
dn = (z.float().double() - zh).norm(dim=1)
for p, c, lo, hi in b[:6]:
    r = z[p] @ z.T
    s = zh[p] @ zh.T
    r[p] = 0
    s[p] = 0
    m = (r.abs() > a.tau) & (s.abs() <= a.tau + eps)
    idx = torch.nonzero(m).flatten().tolist()
    print("pod", p, "count", c, "want", lo, "near pairs", len(idx), flush=True)
    for q in idx[:8]:
        print("   q", q, "r %.9f S %.9f S-r %.3e dn_p %.3e dn_q %.3e" % (float(r[q]), float(s[q]), float(s[q] - r[q]),
                                                                  float(dn[p]), float(dn[q])), flush=True)
