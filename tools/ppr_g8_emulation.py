#!/usr/bin/env python3
"""One rank of a G-rank PageRank solve, emulated on one GPU: what an iteration
costs at G = 8 on the host and on the device, against the ~1 ms scoring step it overlaps.

Rank 0 of G = 8 on the C4 mesh (1M pods / 20M edges): its 125k-row shard of the pull-CSR with the
8-slice exchange layout (w_all = G slices of krca_ppr_slice_words(n_max)), and a device copy of its
send slice into slice 0 standing in for the all-gather (the other slices keep the codes of a first
real solve, so the gathers read realistic values; the partial-sum slots are those of that solve).
Folded iterations as RcaStep runs them: init, exchange, iters x (krca_ppr_shard_step_folded,
exchange), finish.  Measured:

  gpu_us_per_iter   the same 30 iterations captured in a HIP graph and replayed: device time only
  eager_us_per_iter the eager launch sequence, wall clock from the first call to the synchronisation
  host_us_per_iter  host time to enqueue one iteration (ctypes call + copy), no synchronisation
  kernel_us         HIP events around one step kernel

A real all-gather adds RCCL's own latency (not emulated here).  Prints one JSON line.
  python tools/ppr_g8_emulation.py [--pods 1000000] [--edges 20000000] [--world 8] [--iters 30] [--reps 20]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kubernetes-rca-system_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pods", type=int, default=1_000_000)
    ap.add_argument("--edges", type=int, default=20_000_000)
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import torch
    from krca import native, synth
    from krca.rca import RANKING, DeviceShard, shard_graph, shard_range, slice_words, step_flags
    eng = native.NativeEngine(0)
    m = synth.make_graph(a.pods, n_edges=a.edges, seed=0)
    rng = np.random.default_rng(0)
    s = (np.abs(rng.standard_normal(a.pods)) * 1.5).astype(np.float32)
    s[m.roots] = 12.0
    cfg = RANKING.replace(iters=a.iters)
    G = a.world
    lo, hi, n_max = shard_range(a.pods, G, 0)
    rp, col, od = shard_graph(m.row_ptr, m.col, m.outdeg, lo, hi)
    sh = DeviceShard(eng, None, rp, col, od, a.pods, n_max, G, cfg)
    sh.score_out = {"score": torch.from_numpy(s[lo:hi]).cuda()}
    sw = slice_words(n_max)
    # the other ranks' slices: the codes of a real init on the whole mesh's first n_max * G pods
    full = []
    for g in range(G):
        glo, ghi, _ = shard_range(a.pods, G, g)
        o = DeviceShard(eng, None, *shard_graph(m.row_ptr, m.col, m.outdeg, glo, ghi), a.pods, n_max, G, cfg)
        o.score_out = {"score": torch.from_numpy(s[glo:ghi].copy() if ghi > glo else np.zeros(1, np.float32)).cuda()}
        o.init(cfg.alpha, cfg.floor(a.pods, 8))
        full.append(o.send.clone())
        del o
    base = torch.cat(full)
    st = torch.cuda.current_stream()

    def exchange():  # stand-in for the all-gather: this rank's slice lands in slot 0
        sh.w_all[:sw].copy_(sh.send)

    def propagate():
        sh.init(cfg.alpha, cfg.floor(a.pods, 8))
        exchange()
        for it in range(1, cfg.iters + 1):
            sh.step_folded(cfg.alpha, cfg.tol, it, step_flags(cfg.tol, it == cfg.iters))
            exchange()
        sh.finish(cfg.alpha, cfg.tol, cfg.iters)

    sh.w_all.copy_(base)
    for _ in range(3):
        propagate()
    torch.cuda.synchronize()
    # eager wall clock and host enqueue time
    eager, host = [], []
    for _ in range(a.reps):
        sh.w_all.copy_(base)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        propagate()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        host.append((t1 - t0) / (a.iters + 1) * 1e6)
        eager.append((t2 - t0) / (a.iters + 1) * 1e6)
    # one step kernel alone (HIP events on the launch stream)
    ks = []
    for it in range(1, 11):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        sh.step_folded(cfg.alpha, cfg.tol, it, 0)
        e1.record(st)
        torch.cuda.synchronize()
        ks.append(e0.elapsed_time(e1) * 1e3)
    # device time only: the iterations captured in a HIP graph
    g = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    side.wait_stream(st)
    with torch.cuda.graph(g, stream=side):
        propagate()
    st.wait_stream(side)
    gpu = []
    for _ in range(a.reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        g.replay()
        e1.record(st)
        torch.cuda.synchronize()
        gpu.append(e0.elapsed_time(e1) * 1e3 / (a.iters + 1))
    out = dict(what=f"rank 0 of G={G} emulated on one GPU (device copy for the all-gather)", pods=a.pods,
               edges=m.n_edges, shard_rows=hi - lo, shard_edges=int(rp[-1]), blocks=int(sh.plan_len // 4),
               iters=a.iters, slice_bytes=8 * sw,
               gpu_us_per_iter=float(np.median(gpu)), eager_us_per_iter=float(np.median(eager)),
               host_us_per_iter=float(np.median(host)), kernel_us=float(np.median(ks)),
               solve_eager_ms=float(np.median(eager)) * (a.iters + 1) / 1e3,
               solve_graph_ms=float(np.median(gpu)) * (a.iters + 1) / 1e3)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
