#!/usr/bin/env python3
"""The ranks of a G-rank PageRank solve, emulated on one GPU: what an iteration
costs at G = 8 on the host and on the device, against the ~1 ms scoring step it overlaps.

The C4 mesh (1M pods / 20M edges) cut into G = 8 shards of the pull-CSR with the G-slice exchange
layout, once with uniform pod ranges and once with krca.rca.Partition.balanced's ranges.  Every
rank's step kernel is timed on its own (the w_all of all ranks' init codes, so the gathers read
realistic values); the SLOWEST rank -- every iteration's all-gather waits for it -- then runs the
folded iterations as RcaStep does (init, exchange, iters x (krca_ppr_shard_step_folded, exchange),
finish) with a device copy of its send slice standing in for the all-gather.  Measured:

  gpu_us_per_iter   the same 30 iterations captured in a HIP graph and replayed: device time only
  eager_us_per_iter the eager launch sequence, wall clock from the first call to the synchronisation
  host_us_per_iter  host time to enqueue one iteration (ctypes call + copy), no synchronisation
  rank_kernel_us    HIP events around one step kernel of every rank

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
    from krca.rca import RANKING, DeviceShard, Partition, shard_graph, slice_words, step_flags
    eng = native.NativeEngine(0)
    m = synth.make_graph(a.pods, n_edges=a.edges, seed=0)
    rng = np.random.default_rng(0)
    s = (np.abs(rng.standard_normal(a.pods)) * 1.5).astype(np.float32)
    s[m.roots] = 12.0
    cfg = RANKING.replace(iters=a.iters)
    G = a.world
    fl = cfg.floor(a.pods, 8)
    st = torch.cuda.current_stream()
    out = dict(what=f"ranks of G={G} emulated on one GPU (device copy for the all-gather)", pods=a.pods,
               edges=m.n_edges, iters=a.iters)
    for pname, part in (("uniform", Partition.uniform(a.pods, G)), ("balanced", Partition.balanced(m.row_ptr, G))):
        sw = slice_words(part.n_slot)
        shards = []
        for g in range(G):
            lo, hi, n_slot = part.range(g)
            sh = DeviceShard(eng, None, *shard_graph(m.row_ptr, m.col, m.outdeg, lo, hi, part), a.pods, n_slot, G, cfg)
            sh.score_out = {"score": torch.from_numpy(s[lo:hi].copy() if hi > lo else np.zeros(1, np.float32)).cuda()}
            sh.init(cfg.alpha, fl)
            shards.append(sh)
        base = torch.cat([sh.send for sh in shards])  # every rank's init codes: realistic gathers
        kern = []
        for sh in shards:  # one step kernel per rank, HIP events on the launch stream
            sh.w_all.copy_(base)
            ks = []
            for it in range(1, 11):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                sh.step_folded(cfg.alpha, cfg.tol, it, 0)
                e1.record(st)
                torch.cuda.synchronize()
                ks.append(e0.elapsed_time(e1) * 1e3)
            kern.append(float(np.median(ks)))
        slow = int(np.argmax(kern))
        sh = shards[slow]

        def exchange():  # stand-in for the all-gather: this rank's slice lands in its slot
            sh.w_all[slow * sw:(slow + 1) * sw].copy_(sh.send)

        def propagate():
            sh.init(cfg.alpha, fl)
            exchange()
            for it in range(1, cfg.iters + 1):
                sh.step_folded(cfg.alpha, cfg.tol, it, step_flags(cfg.tol, it == cfg.iters))
                exchange()
            sh.finish(cfg.alpha, cfg.tol, cfg.iters)

        sh.w_all.copy_(base)
        for _ in range(3):
            propagate()
        torch.cuda.synchronize()
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
        g = torch.cuda.CUDAGraph()  # device time only: the solve captured in a HIP graph
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
        out[pname] = dict(bounds=[int(b) for b in part.bounds], rank_rows=[int(v) for v in np.diff(part.bounds)],
                          rank_edges=[int(v) for v in np.diff(m.row_ptr[part.bounds])],
                          rank_kernel_us=kern, slowest_rank=slow, slice_bytes=8 * sw,
                          gpu_us_per_iter=float(np.median(gpu)), eager_us_per_iter=float(np.median(eager)),
                          host_us_per_iter=float(np.median(host)),
                          solve_eager_ms=float(np.median(eager)) * (a.iters + 1) / 1e3,
                          solve_graph_ms=float(np.median(gpu)) * (a.iters + 1) / 1e3)
        del shards, sh, g
        torch.cuda.empty_cache()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
