#!/usr/bin/env python3
"""PageRank step microbench at C4 (1M pods / 20M edges): the bench's 30-iteration propagate on
one device, seeded with fixed synthetic anomaly scores; per-iteration time from HIP events.

  python tools/ppr_bench.py [--pods 1000000] [--edges 20000000] [--dict 1] [--reps 10] [--check]
                            [--order none|random|rcm] [--xcd 0|1]
--dict 0 packs every block direct (one gather per edge): the A/B of DESIGN.md §3.2.
--order relabels the pods before packing (random: a seeded permutation; rcm: reverse Cuthill-McKee
of the symmetrised mesh) -- the locality experiment of DESIGN.md §3.2; --xcd sets KRCA_PPR_XCD.
--check compares the fixed point with the C oracle on the original labels (bit-identical: the
int64 sums are order-free).  Prints one JSON line.
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kubernetes-rca-system_amd"))


def order(m, how):
    """perm[new] = old pod id."""
    N = m.n_pods
    if how == "none":
        return np.arange(N, dtype=np.int64)
    if how == "random":
        return np.random.default_rng(7).permutation(N).astype(np.int64)
    import scipy.sparse as sp
    from scipy.sparse.csgraph import reverse_cuthill_mckee
    A = sp.csr_matrix((np.ones(len(m.col), np.int8), m.col, m.row_ptr), shape=(N, N))
    return np.asarray(reverse_cuthill_mckee((A + A.T).tocsr(), symmetric_mode=True), np.int64)


def relabel(m, perm):
    """The mesh with pod perm[i] renamed i (rows re-sorted, callers ascending)."""
    N = len(perm)
    inv = np.empty_like(perm)
    inv[perm] = np.arange(N)
    deg = np.diff(m.row_ptr)[perm]
    rp = np.zeros(N + 1, np.int64)
    np.cumsum(deg, out=rp[1:])
    idx = np.repeat(m.row_ptr[perm] - rp[:-1], deg) + np.arange(rp[-1])
    key = np.sort(np.repeat(np.arange(N, dtype=np.int64), deg) * N + inv[m.col[idx]])
    return rp, (key % N).astype(np.int32), np.asarray(m.outdeg)[perm].astype(np.int32)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pods", type=int, default=1_000_000)
    ap.add_argument("--edges", type=int, default=20_000_000)
    ap.add_argument("--dict", type=int, default=1)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--order", default="none", choices=["none", "random", "rcm"])
    ap.add_argument("--xcd", type=int, default=0)
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
    perm = order(m, a.order)
    rp, col, od = relabel(m, perm)
    inv = np.empty_like(perm)
    inv[perm] = np.arange(len(perm))
    with native.tune(eng.lib, KRCA_PPR_DICT=a.dict):
        sh = DeviceShard(eng, None, rp, col, od, a.pods, a.pods, 1, cfg)
    eng.lib.krca_tune_set(b"KRCA_PPR_XCD", a.xcd)
    sh.score_out = {"score": torch.from_numpy(s[perm]).cuda()}
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
    iters_run, _ = sh.ctl_read()  # the stop rule's count: the launches past it return at once
    N, E = a.pods, m.n_edges
    plan = sh.plan.cpu().numpy().reshape(-1, 4)
    nu = plan[:, 0] >> 32
    ne = plan[:, 3] - plan[:, 2]
    d = nu > 0
    edge_bytes = int(4 * nu[d].sum() + 2 * ne[d].sum() + 4 * ne[~d].sum())
    # algorithmic bytes per iteration: plan + lane info (two 2-byte words per
    # ppr_step lane, krca_ppr_lane_size) + packed columns + q and the alpha/outdeg coefficients read + weight
    # codes written + codes gathered once (compulsory); r is written on the last iteration.
    # fabric_bytes_per_iter prices the gathered table once per XCD instead (8 XCDs, each with its
    # own L2: the least an L2-miss counter can show for a table that every XCD's rows gather from
    # at random).
    lane_bytes = 2 * int(eng.lib.krca_ppr_lane_size(4 * len(plan)))
    base = 32 * len(plan) + lane_bytes + edge_bytes + 8 * N + 8 * N + 4 * N
    per_iter = base + 4 * N
    fabric_per_iter = base + 8 * 4 * N
    out = dict(kernel="ppr propagate (init + 30 x (step + reduce))", dict=a.dict, order=a.order, xcd=a.xcd, pods=N, edges=E,
               dict_blocks=int(d.sum()), blocks=len(plan), gathers=int(nu[d].sum() + ne[~d].sum()),
               ms=ms, ms_median=float(np.median(ms)), us_per_iter=float(np.median(ms)) * 1e3 / cfg.iters,
               iters_run=iters_run,
               # the whole propagate per iteration that did work (an upper bound: it includes the
               # launches past the stop rule, ~5 us each); per-dispatch times are in the kernel trace
               us_per_working_iter=float(np.median(ms)) * 1e3 / max(iters_run, 1),
               bytes_per_iter=per_iter, fabric_bytes_per_iter=fabric_per_iter)
    if a.check:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        _, r, _, q = oracle.c_ppr(m.row_ptr, m.col, m.outdeg, s, cfg.alpha, cfg.iters, 0.0, cfg.floor(sh.N, sh.M),
                                  return_q=True)
        out["bit_identical"] = bool(np.array_equal(sh.r[:N].cpu().numpy()[inv], r))
        idx, _ = step.merge(*sh.local_topk(cfg.k))
        idx = perm[np.asarray(idx, np.int64)]
        out["top10_identical"] = [int(i) for i in idx] == oracle.topk_ref(oracle.c_rca_key(r, q), cfg.k)[0].tolist()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
