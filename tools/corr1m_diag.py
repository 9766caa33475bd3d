"""Diagnostic: C4 correlation at 1M pods (seed 2, tau 0.5, k 10) twice; for the 4096 sampled rows of
tests/test_gpu_corr.py::test_corr_c4_1m_pods print every row whose top-k set differs from a float64
device reference (gap > 1e-12) with the device and reference partners, and whether the two device
runs agree."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "kubernetes-rca-system_amd"), os.path.join(ROOT, "oracle")]
import oracle  # noqa: E402
from krca import native, synth  # noqa: E402

P, T, k, TAU = 1_000_000, 1440, 10, 0.5
eng = native.NativeEngine()
x = synth.make_metrics(P, 1, T, seed=2, group_size=20, device="cuda")
eng.corr_topk(x[:, :4096], k=k, tau=TAU)
r1 = eng.corr_topk(x, k=k, tau=TAU)
r2 = eng.corr_topk(x, k=k, tau=TAU)
for key in r1:
    print("runs identical", key, bool(np.array_equal(r1[key], r2[key])), flush=True)
z32 = oracle.c_corr_z32(x.cpu().numpy(), 0)[0]
del x
torch.cuda.empty_cache()
z = torch.from_numpy(z32).cuda().double()
rows = np.sort(np.random.default_rng(7).choice(P, 4096, replace=False))
nbad = 0
for i in range(0, len(rows), 512):
    rr = torch.as_tensor(rows[i:i + 512], device=z.device).long()
    R = z[rr] @ z.T
    R[torch.arange(len(rr)), rr] = 0.0
    a = R.abs()
    a[torch.arange(len(rr)), rr] = -1.0
    top = torch.topk(a, k + 3, dim=1)
    for res, tag in ((r1, "run1"), (r2, "run2")):
        gi = torch.from_numpy(res["idx"][rows[i:i + 512]]).to(z.device).long()
        want = torch.sort(top.indices[:, :k], dim=1).values
        got = torch.sort(gi, dim=1).values
        gap = top.values[:, k - 1] - top.values[:, k]
        bad = ((want != got).any(1) & (gap > 1e-12)).nonzero().flatten().tolist()
        for b in bad:
            nbad += 1
            p = int(rows[i + b])
            print(tag, "pod", p, "cert", float(res["cert"][p]), "count", int(res["count"][p]))
            print("  device", res["idx"][p].tolist(), [round(float(v), 6) for v in res["val"][p]])
            print("  ref   ", top.indices[b].tolist(), [round(float(v), 6) for v in top.values[b]])
            ex = R[b, torch.from_numpy(res["idx"][p]).to(z.device).long()]
            print("  exact of device partners", [round(float(v), 6) for v in ex])
print("bad rows", nbad)
