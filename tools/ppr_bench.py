#!/usr/bin/env python3
"""PageRank step microbench at C4 (1M pods / 20M edges): the bench's 30-iteration propagate on
one device, seeded with fixed synthetic anomaly scores; per-iteration time from HIP events.

  python tools/ppr_bench.py [--pods 1000000] [--edges 20000000] [--dict 1] [--reps 10] [--check]
--dict 0 packs every block direct (one gather per edge): the A/B of DESIGN.md §3.2.
--check compares the fixed point with the C oracle (bit-identical).  Prints one JSON line.
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kubernetes-rca-system_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pods", type=int, default=1_000_000)
    ap.add_argument("--edges", type=int, default=20_000_000)
    ap.add_argument("--dict", type=int, default=1)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--check", action="store_true")
    a = ap.parse_args()
    import torch
    from krca import native, synth
    from krca.rca import RANKING, Comm, DeviceShard, RcaStep
    eng = native.NativeEngine(0)
    m = synth.make_graph(a.pods, n_edges=a.edges, seed=0)
    rng = np.random.default_rng(0)
    s = (np.abs(rng.standard_normal(a.pods)) * 1.5).astype(np.float32)
    s[m.roots] = 12.0
    for h in synth.caller_hops(m, m.roots):
        s[h] = np.maximum(s[h], 7.0)
    cfg = RANKING
    with native.tune(eng.lib, KRCA_PPR_DICT=a.dict):
        sh = DeviceShard(eng, None, m.row_ptr, m.col, m.outdeg, a.pods, a.pods, 1, cfg)
    sh.score_out = {"score": torch.from_numpy(s).cuda()}
    step = RcaStep(sh, Comm(), cfg, 0)
    step.propagate()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.reps)]
    for e0, e1 in ev:
        e0.record()
        step.propagate()
        e1.record()
    torch.cuda.synchronize()
    ms = [e0.elapsed_time(e1) for e0, e1 in ev]
    N, E = a.pods, m.n_edges
    plan = sh.plan.cpu().numpy().reshape(-1, 4)
    nu = plan[:, 0] >> 32
    ne = plan[:, 3] - plan[:, 2]
    d = nu > 0
    edge_bytes = int(4 * nu[d].sum() + 2 * ne[d].sum() + 4 * ne[~d].sum())
    # algorithmic bytes per iteration: plan + lane info (a 2-byte word per lane and
    # a 2-byte sum slot per row) + packed columns + q and the alpha/outdeg coefficients read + weight
    # codes written + codes gathered once (compulsory); r is written on the last iteration.
    # fabric_bytes_per_iter prices the gathered table once per XCD instead (8 XCDs, each with its
    # own L2: the least an L2-miss counter can show for a table that every XCD's rows gather from
    # at random).
    base = 32 * len(plan) + 4 * 256 * len(plan) + edge_bytes + 8 * N + 8 * N + 4 * N
    per_iter = base + 4 * N
    fabric_per_iter = base + 8 * 4 * N
    out = dict(kernel="ppr propagate (init + 30 x (step + reduce))", dict=a.dict, pods=N, edges=E,
               dict_blocks=int(d.sum()), blocks=len(plan), gathers=int(nu[d].sum() + ne[~d].sum()),
               ms=ms, ms_median=float(np.median(ms)), us_per_iter=float(np.median(ms)) * 1e3 / cfg.iters,
               bytes_per_iter=per_iter, fabric_bytes_per_iter=fabric_per_iter)
    if a.check:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        _, r, _, q = oracle.c_ppr(m.row_ptr, m.col, m.outdeg, s, cfg.alpha, cfg.iters, 0.0, cfg.floor(len(s), 8),
                                  return_q=True)
        out["bit_identical"] = bool(np.array_equal(sh.r[:N].cpu().numpy(), r))
        idx, _ = step.merge(*sh.local_topk(cfg.k))
        out["top10_identical"] = [int(i) for i in idx] == oracle.topk_ref(oracle.c_rca_key(r, q), cfg.k)[0].tolist()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
