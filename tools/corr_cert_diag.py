"""Rows whose reported top-k set differs from the float64 reference (outside ties), with their
certificates, for the overflow-refill mesh of tests/test_gpu_corr.py under the current knobs (GPU;
tools only).  A wrong set must never carry cert > 0."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kubernetes-rca-system_amd"))
from krca import native, synth  # noqa: E402

eng = native.NativeEngine()
P, T, k, tau = 1800, 256, 10, 0.5
base = synth.make_metrics(P, 1, T, seed=11, group_size=0)
x = base.clone()
for g0 in (0, 600):
    x[:, g0:g0 + 600, 0] = base[:, g0:g0 + 1, 0]
x = x.cuda()
res = eng.corr_topk(x, k=k, tau=tau)
z = eng.corr_prepare_device(x)["z32"].double()
R = z @ z.T
R.fill_diagonal_(0.0)
A = R.abs()
A.fill_diagonal_(-1.0)
top = torch.topk(A, k + 1, dim=1)
gap = (top.values[:, k - 1] - top.values[:, k]).cpu().numpy()
want = np.sort(top.indices[:, :k].cpu().numpy(), 1)
got = np.sort(res["idx"], 1)
wrong = np.nonzero((want != got).any(1) & (gap > 1e-12))[0]
print("knobs", {kk: v for kk, v in os.environ.items() if kk.startswith("KRCA_")})
print("wrong sets", len(wrong), "of which certified", int((res["cert"][wrong] > 0).sum()),
      "uncertified rows", int((res["cert"] <= 0).sum()), flush=True)
for p in wrong[:5]:
    print("  row", p, "cert", float(res["cert"][p]), "gap", float(gap[p]), "got", res["idx"][p].tolist(),
          "want", top.indices[p, :k].tolist())
