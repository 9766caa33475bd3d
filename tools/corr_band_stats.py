#!/usr/bin/env python3
"""Pairs with |r| within eps of tau per 256x256 tile at C3 (float64 on the device, torch): how
the ambiguous pairs of krca_corr_topk's exact count are spread.  python tools/corr_band_stats.py"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kubernetes-rca-system_amd"))
from krca import synth  # noqa: E402

P, T, tau, eps = 100_000, 1440, 0.5, 1.07e-3
x = synth.make_metrics(P, 1, T, seed=1, group_size=20, device="cuda")[:, :, 0].double().T
x = x - x.mean(1, keepdim=True)
z = x / (x.norm(dim=1, keepdim=True) + 1e-300)
del x
nb = (P + 255) // 256
per = np.zeros((nb, nb), np.int64)
for r0 in range(0, P, 2048):
    r1 = min(P, r0 + 2048)
    R = (z[r0:r1] @ z.T).abs()
    band = (R > tau - eps) & (R <= tau + eps)
    rows = torch.arange(r0, r1, device="cuda")
    band[rows - r0, rows] = False
    cnt = band.view(r1 - r0, -1)
    pad = nb * 256 - P
    cnt = torch.nn.functional.pad(cnt.float(), (0, pad))
    blk = cnt.view(r1 - r0, nb, 256).sum(2)  # [rows, col blocks]
    for i0 in range(r0, r1, 256):
        per[i0 // 256] += blk[i0 - r0:i0 - r0 + 256].sum(0).long().cpu().numpy()
up = np.triu(per)
v = up[up > 0]
print(json.dumps(dict(band_pairs_upper=int(up.sum()), tiles=int((np.triu(np.ones_like(per)) > 0).sum()),
                      tiles_with_pairs=int((up > 0).sum()), mean=float(v.mean()), p50=float(np.median(v)),
                      p99=float(np.percentile(v, 99)), max=int(v.max()), diag_mean=float(np.diag(per).mean()))))
