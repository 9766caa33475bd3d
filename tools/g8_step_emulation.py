#!/usr/bin/env python3
"""One rank's pipelined RCA step at G = 8, emulated on one GPU: which pod partition keeps the
PageRank solve from bounding the step (krca.rca.Partition).

bench.py's step on rank g of G: the scoring of its pods (krca_rolling_score) on one HIP stream
while the previous step's PageRank (init, 30 folded steps, each followed by the exchange, finish,
key, top-k) runs on the other; every PageRank iteration waits for the all-gather, i.e. for the rank
with the most edges.  Here the rank with the most PageRank work under each partition runs exactly
that two-stream pipeline on its own shard (its metric rows generated as bench.py generates them),
with a device copy of its send slice standing in for the all-gather (RCCL's own latency is not
included: it adds the same per-iteration time under either partition).  Reports ms per step for
the uniform ranges (ceil(N / G) pods) and for Partition.balanced, plus each one's scoring and
PageRank parts run alone.  Prints one JSON line.

The replicated alternative: every rank scores its own pods, the scores are all-gathered once per
step, and each rank runs the whole mesh's solve alone (no collective inside the solve).

  python tools/g8_step_emulation.py [--pods 1000000] [--edges 20000000] [--world 8] [--steps 20]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kubernetes-rca-system_amd"))


class CopyComm:
    """Comm stand-in: the exchange lands this rank's send slice in its own slot of w_all."""

    def __init__(self, world, rank, sw):
        self.world, self.rank, self.sw = world, rank, sw

    def exchange(self, shard):
        shard.w_all[self.rank * self.sw:(self.rank + 1) * self.sw].copy_(shard.send)


def run_rank(a, m, hops, cfg, part, g, M, T):
    """bench.py's two-stream pipeline on rank g's shard: ms per step, and its two parts alone."""
    import torch
    from krca import native, synth
    from krca.rca import DeviceShard, RcaStep, shard_graph, slice_words
    G = part.world
    lo, hi, n_slot = part.range(g)
    rp, col, od = shard_graph(m.row_ptr, m.col, m.outdeg, lo, hi, part)
    x = synth.make_metrics_range(lo, hi, M, T, seed=0, roots=m.roots, hop_sets=hops, device="cuda")
    engs = [native.NativeEngine(0) for _ in range(2)]
    shards = [DeviceShard(e, x, rp, col, od, a.pods, n_slot, G, cfg) for e in engs]
    comm = CopyComm(G, g, slice_words(n_slot))
    steps = [RcaStep(sh, comm, cfg, lo) for sh in shards]
    streams = [torch.cuda.Stream() for _ in range(2)]
    done = [None]

    def enqueue(i):
        j = i % 2
        with torch.cuda.stream(streams[j]):
            if done[0] is not None:
                streams[j].wait_event(done[0])
            shards[j].score()
            done[0] = torch.cuda.Event()
            done[0].record()
            steps[j].propagate()
            shards[j].local_topk(cfg.k)

    for i in range(4):
        enqueue(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        enqueue(i)
    torch.cuda.synchronize()
    pipe_ms = (time.perf_counter() - t0) / a.steps * 1e3
    parts = {}
    for name, fn in (("scoring", shards[0].score), ("pagerank", steps[0].propagate)):
        ev = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            ev.append(e0.elapsed_time(e1))
        parts[name] = float(np.median(ev))
    res = dict(pods=hi - lo, edges=int(m.row_ptr[hi] - m.row_ptr[lo]), pipelined_ms_per_step=pipe_ms,
               scoring_ms_alone=parts["scoring"], pagerank_ms_alone=parts["pagerank"])
    del x, shards, steps, engs
    torch.cuda.empty_cache()
    return res


def run_replicated(a, m, hops, cfg, part, g, M, T):
    """The replicated-PageRank step on rank g: scoring of its pods, the all-gather of the scores
    (4 B per pod; a device copy into the full vector stands in for it), then the whole mesh's
    30-iteration solve on this rank alone (no per-iteration collective), pipelined as bench.py's
    two streams.  ms per step, and the parts alone."""
    import torch
    from krca import native, synth
    from krca.rca import Comm, DeviceShard, RcaStep, shard_graph
    lo, hi, n_slot = part.range(g)
    rp, col, od = shard_graph(m.row_ptr, m.col, m.outdeg, lo, hi, part)
    x = synth.make_metrics_range(lo, hi, M, T, seed=0, roots=m.roots, hop_sets=hops, device="cuda")
    engs = [native.NativeEngine(0) for _ in range(2)]
    scor = [DeviceShard(e, x, rp, col, od, a.pods, n_slot, part.world, cfg) for e in engs]
    full = [DeviceShard(e, None, m.row_ptr, m.col, m.outdeg, a.pods, a.pods, 1, cfg) for e in engs]
    sfull = [torch.zeros(a.pods, dtype=torch.float32, device="cuda") for _ in range(2)]
    for sh, sv in zip(full, sfull):
        sh.score_out = {"score": sv}
    steps = [RcaStep(sh, Comm(), cfg, 0) for sh in full]
    streams = [torch.cuda.Stream() for _ in range(2)]
    done = [None]

    def gather(j):  # the all-gather of the scores: this rank's slice into the full vector
        sfull[j][lo:hi].copy_(scor[j].score_out["score"][:hi - lo])

    def enqueue(i):
        j = i % 2
        with torch.cuda.stream(streams[j]):
            if done[0] is not None:
                streams[j].wait_event(done[0])
            scor[j].score()
            done[0] = torch.cuda.Event()
            done[0].record()
            gather(j)
            steps[j].propagate()
            full[j].local_topk(cfg.k)

    for i in range(4):
        enqueue(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        enqueue(i)
    torch.cuda.synchronize()
    pipe_ms = (time.perf_counter() - t0) / a.steps * 1e3
    parts = {}
    for name, fn in (("scoring", scor[0].score), ("pagerank_full_mesh", steps[0].propagate)):
        ev = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            ev.append(e0.elapsed_time(e1))
        parts[name] = float(np.median(ev))
    res = dict(pods=hi - lo, edges=int(m.row_ptr[-1]), pipelined_ms_per_step=pipe_ms,
               scoring_ms_alone=parts["scoring"], pagerank_ms_alone=parts["pagerank_full_mesh"])
    del x, scor, full, steps, engs
    torch.cuda.empty_cache()
    return res


def run_decoupled(a, m, hops, cfg, spart, ppart, gs, gp, M, T):
    """Scoring and PageRank on different partitions: rank gs's scoring shard (spart's range), then
    the score exchange (one all-gather of 4 B per pod; a device copy of this rank's slice into the
    full vector stands in for it), then the PageRank solve of rank gp's rows under ppart (every
    iteration's exchange a device copy, as run_rank), pipelined as bench.py's two streams.  The
    job's step is the slowest rank's: gs and gp are the binding ranks of the two partitions."""
    import torch
    from krca import native, synth
    from krca.rca import DeviceShard, RcaStep, shard_graph, slice_words
    G = ppart.world
    slo, shi, s_slot = spart.range(gs)
    plo, phi, p_slot = ppart.range(gp)
    rp, col, od = shard_graph(m.row_ptr, m.col, m.outdeg, plo, phi, ppart)
    x = synth.make_metrics_range(slo, shi, M, T, seed=0, roots=m.roots, hop_sets=hops, device="cuda")
    engs = [native.NativeEngine(0) for _ in range(2)]
    scor = [DeviceShard(e, x, np.zeros(1, np.int64), np.zeros(0, np.int32), np.zeros(0, np.int32), a.pods, s_slot,
                        G, cfg) for e in engs]
    ppr = [DeviceShard(e, None, rp, col, od, a.pods, p_slot, G, cfg) for e in engs]
    sfull = [torch.zeros(a.pods + p_slot, dtype=torch.float32, device="cuda") for _ in range(2)]
    for sh, sv in zip(ppr, sfull):
        sh.score_out = {"score": sv[plo:plo + max(phi - plo, 1)]}
    comm = CopyComm(G, gp, slice_words(p_slot))
    steps = [RcaStep(sh, comm, cfg, plo) for sh in ppr]
    streams = [torch.cuda.Stream() for _ in range(2)]
    done = [None]

    def enqueue(i):
        j = i % 2
        with torch.cuda.stream(streams[j]):
            if done[0] is not None:
                streams[j].wait_event(done[0])
            scor[j].score()
            done[0] = torch.cuda.Event()
            done[0].record()
            sfull[j][slo:shi].copy_(scor[j].score_out["score"][:shi - slo])
            steps[j].propagate()
            ppr[j].local_topk(cfg.k)

    for i in range(4):
        enqueue(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        enqueue(i)
    torch.cuda.synchronize()
    pipe_ms = (time.perf_counter() - t0) / a.steps * 1e3
    parts = {}
    for name, fn in (("scoring", scor[0].score), ("pagerank", steps[0].propagate)):
        ev = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            ev.append(e0.elapsed_time(e1))
        parts[name] = float(np.median(ev))
    res = dict(scoring_rank=gs, scoring_pods=shi - slo, pagerank_rank=gp, pagerank_pods=phi - plo,
               pagerank_edges=int(m.row_ptr[phi] - m.row_ptr[plo]), pipelined_ms_per_step=pipe_ms,
               scoring_ms_alone=parts["scoring"], pagerank_ms_alone=parts["pagerank"])
    del x, scor, ppr, steps, engs
    torch.cuda.empty_cache()
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pods", type=int, default=1_000_000)
    ap.add_argument("--edges", type=int, default=20_000_000)
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--ppr-grids", default="", help="comma list of KRCA_PPR_GRID values: the uniform "
                    "partition's binding rank re-run with the PageRank step's grid capped (leaving CUs to "
                    "the scoring that overlaps it); e.g. 256,512")
    ap.add_argument("--only-grids", action="store_true", help="skip the partition / replicated runs")
    ap.add_argument("--decoupled", default="", help="comma list of edge slacks: scoring on the uniform ranges, "
                    "PageRank on Partition.balanced(edge_slack=...) ranges (scores exchanged once per step); "
                    "runs only these")
    a = ap.parse_args()
    from krca import synth
    from krca.rca import RANKING, Partition
    M, T = 8, 1440
    m = synth.make_graph(a.pods, n_edges=a.edges, seed=0)
    hops = synth.caller_hops(m, m.roots)
    cfg = RANKING.replace(seed_floor=RANKING.floor(a.pods, M))
    G = a.world
    out = dict(what=f"one rank's pipelined step at G={G} on one GPU (device copy for the all-gather)",
               pods=a.pods, edges=m.n_edges, steps=a.steps)
    if a.ppr_grids:
        from krca import native
        part = Partition.uniform(a.pods, G)
        g = int(np.argmax(np.diff(m.row_ptr[part.bounds])))
        lib = native.load_library()
        out["uniform_ppr_grid"] = {}
        for grid in [int(v) for v in a.ppr_grids.split(",")]:
            assert lib.krca_tune_set(b"KRCA_PPR_GRID", grid) == 0
            out["uniform_ppr_grid"][str(grid)] = run_rank(a, m, hops, cfg, part, g, M, T)
        lib.krca_tune_set(b"KRCA_PPR_GRID", 0)
        if a.only_grids:
            print(json.dumps(out), flush=True)
            return
    if a.decoupled:
        spart = Partition.uniform(a.pods, G)
        gs = int(np.argmax(np.diff(spart.bounds)))
        out["decoupled"] = {}
        part = Partition.uniform(a.pods, G)
        g = int(np.argmax(np.diff(m.row_ptr[part.bounds])))
        out["uniform_coupled"] = dict(rank=g, **run_rank(a, m, hops, cfg, part, g, M, T))
        for slack in [float(v) for v in a.decoupled.split(",")]:
            ppart = Partition.balanced(m.row_ptr, G, edge_slack=slack)
            edges = np.diff(m.row_ptr[ppart.bounds])
            pods = np.diff(ppart.bounds)
            res = {f"ppr_rank{gp}": run_decoupled(a, m, hops, cfg, spart, ppart, gs, gp, M, T)
                   for gp in sorted({int(np.argmax(edges)), int(np.argmax(pods))})}
            out["decoupled"][str(slack)] = dict(bounds=[int(b) for b in ppart.bounds], ranks=res,
                                                step_ms_bound=max(r["pipelined_ms_per_step"] for r in res.values()))
        print(json.dumps(out), flush=True)
        return
    for pname, part in (("uniform", Partition.uniform(a.pods, G)), ("balanced", Partition.balanced(m.row_ptr, G))):
        edges = np.diff(m.row_ptr[part.bounds])
        pods = np.diff(part.bounds)
        res = {}
        # the rank with the most edges (every PageRank iteration waits for it) and the one with the
        # most pods (the longest scoring): the job's step is at least the slower of the two
        for g in sorted({int(np.argmax(edges)), int(np.argmax(pods))}):
            res[f"rank{g}"] = run_rank(a, m, hops, cfg, part, g, M, T)
        out[pname] = dict(bounds=[int(b) for b in part.bounds], ranks=res,
                          step_ms_bound=max(r["pipelined_ms_per_step"] for r in res.values()))
    part = Partition.uniform(a.pods, G)
    pods = np.diff(part.bounds)
    g = int(np.argmax(pods))
    out["replicated"] = dict(ranks={f"rank{g}": run_replicated(a, m, hops, cfg, part, g, M, T)})
    out["replicated"]["step_ms_bound"] = out["replicated"]["ranks"][f"rank{g}"]["pipelined_ms_per_step"]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
