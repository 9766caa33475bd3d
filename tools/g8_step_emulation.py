#!/usr/bin/env python3
"""One rank's pipelined RCA step at G = 8, emulated on one GPU: which pod partition keeps the
PageRank solve from bounding the step (krca.rca.Partition).

bench.py's step on rank g of G: the scoring of its pods (krca_rolling_score) on one HIP stream
while the previous step's PageRank (init, --iters folded steps, each followed by the exchange, finish,
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

Every pipe's two streams live in this one process: with the box's default 4 hardware queues per
process some pipes get both of theirs on one queue and run serialised; pass
--hw-queues 8 (GPU_MAX_HW_QUEUES, set before HIP starts) when comparing several pipes.
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
    solve on this rank alone (no per-iteration collective), pipelined as bench.py's
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


class Pipe:
    """bench.py's two-stream pipelined step of one rank, built once and timed repeatedly: the scoring
    of x (rows [slo, shi) of the uniform ranges), then the PageRank solve of rank gp's rows of
    `part` -- on the same shard (coupled: part's range is the scoring range) or, with split, on a
    PageRank-only shard seeded from a full score vector into which a device copy lands this rank's
    scores (standing in for SplitShard's score all-gather)."""

    def __init__(self, a, m, cfg, x, slo, shi, s_slot, part, gp, split, roles=False):
        import torch
        from krca import native
        from krca.rca import Comm, DeviceShard, RcaStep, shard_graph, slice_words
        self.torch, self.cfg, self.split, self.slo, self.shi = torch, cfg, split, slo, shi
        G = part.world
        plo, phi, p_slot = part.range(gp)
        rp, col, od = shard_graph(m.row_ptr, m.col, m.outdeg, plo, phi, part)
        engs = [native.NativeEngine(0) for _ in range(2)]
        if split:
            nograph = (np.zeros(1, np.int64), np.zeros(0, np.int32), np.zeros(0, np.int32))
            self.scor = [DeviceShard(e, x, *nograph, a.pods, s_slot, G, cfg) for e in engs]
            self.ppr = [DeviceShard(e, None, rp, col, od, a.pods, p_slot, G, cfg) for e in engs]
            self.sfull = [torch.zeros(a.pods + p_slot, dtype=torch.float32, device="cuda") for _ in range(2)]
            for sh, sv in zip(self.ppr, self.sfull):
                sh.score_out = {"score": sv[plo:plo + max(phi - plo, 1)]}
        else:
            self.scor = self.ppr = [DeviceShard(e, x, rp, col, od, a.pods, p_slot, G, cfg) for e in engs]
            # the default key needs every pod's scores: a device copy of this rank's into a full
            # vector stands in for the score all-gather RcaStep makes at G > 1
            self.sfull = [torch.zeros(a.pods + p_slot, dtype=torch.float32, device="cuda") for _ in range(2)]
        from krca.rca import Explain
        self.ex = Explain(m.row_ptr, m.col) if cfg.key == "explained" else None
        self.N, self.plo, self.floor = a.pods, plo, cfg.floor(a.pods, 8)
        # a one-range partition is the replicated solve: one rank's exchange is the buffer swap
        comm = Comm(1, 0) if G == 1 else CopyComm(G, gp, slice_words(p_slot))
        self.steps = [RcaStep(sh, comm, cfg, plo) for sh in self.ppr]
        self.streams = [torch.cuda.Stream() for _ in range(2)]
        self.done = None
        # roles: the scoring always on one stream, the solve on a second, high-priority one (events
        # order them: solve i after scoring i, scoring i + 2 after solve i, whose state it reuses)
        self.roles = roles
        if roles:
            self.s_stream = torch.cuda.Stream()
            self.p_stream = torch.cuda.Stream(priority=-1)
            self.ev_s = [None, None]
            self.ev_p = [None, None]
        self.info = dict(pagerank_rank=gp, pagerank_pods=phi - plo, pagerank_edges=int(m.row_ptr[phi] - m.row_ptr[plo]),
                         scoring_pods=shi - slo)

    def cand(self, j):
        """The step's candidates (bench.py: RcaStep.local_candidates)."""
        if self.ex is None:
            return self.ppr[j].local_topk(self.cfg.k)
        if not self.split:
            self.sfull[j][self.slo:self.shi].copy_(self.scor[j].score_out["score"][:self.shi - self.slo])
        return self.ppr[j].local_topk_explained(self.cfg.k, self.sfull[j][:self.N], self.floor, self.ex, self.plo)

    def enqueue(self, i):
        torch, j = self.torch, i % 2
        if self.roles:
            with torch.cuda.stream(self.s_stream):
                if self.ev_p[j] is not None:
                    self.s_stream.wait_event(self.ev_p[j])
                self.scor[j].score()
                self.ev_s[j] = torch.cuda.Event()
                self.ev_s[j].record()
            with torch.cuda.stream(self.p_stream):
                self.p_stream.wait_event(self.ev_s[j])
                if self.split:
                    self.sfull[j][self.slo:self.shi].copy_(self.scor[j].score_out["score"][:self.shi - self.slo])
                self.steps[j].propagate()
                self.cand(j)
                self.ev_p[j] = torch.cuda.Event()
                self.ev_p[j].record()
            return
        with torch.cuda.stream(self.streams[j]):
            if self.done is not None:
                self.streams[j].wait_event(self.done)
            self.scor[j].score()
            self.done = torch.cuda.Event()
            self.done.record()
            if self.split:
                self.sfull[j][self.slo:self.shi].copy_(self.scor[j].score_out["score"][:self.shi - self.slo])
            self.steps[j].propagate()
            self.cand(j)

    def timed(self, n):
        torch = self.torch
        for i in range(4):
            self.enqueue(i)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(n):
            self.enqueue(i)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n * 1e3

    def alone(self):
        torch, parts = self.torch, {}
        for name, fn in (("scoring", self.scor[0].score), ("pagerank", self.steps[0].propagate)):
            ev = []
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                fn()
                e1.record()
                torch.cuda.synchronize()
                ev.append(e0.elapsed_time(e1))
            parts[name + "_ms_alone"] = float(np.median(ev))
        return parts


def ab_decoupled(a, m, hops, cfg, slacks, reps, M, T):
    """The coupled uniform step of the rank with the most edges against SplitShard's step (scoring
    on uniform rank 0's pods, PageRank on each binding rank of Partition.balanced(edge_slack)),
    built once and timed in alternation `reps` times (the box's clock drifts between separate runs
    by more than the difference measured)."""
    import torch
    from krca import synth
    from krca.rca import Partition
    G = a.world
    spart = Partition.uniform(a.pods, G)
    g = int(np.argmax(np.diff(m.row_ptr[spart.bounds])))
    slo, shi, s_slot = spart.range(g)
    x = synth.make_metrics_range(slo, shi, M, T, seed=0, roots=m.roots, hop_sets=hops, device="cuda")
    pipes = {f"coupled_rank{g}": Pipe(a, m, cfg, x, slo, shi, s_slot, spart, g, False)}
    if a.roles:
        pipes[f"coupled_rank{g}_roles"] = Pipe(a, m, cfg, x, slo, shi, s_slot, spart, g, False, roles=True)
    bounds = {}
    for slack in slacks:
        ppart = Partition.balanced(m.row_ptr, G, edge_slack=slack)
        bounds[str(slack)] = [int(b) for b in ppart.bounds]
        for gp in sorted({int(np.argmax(np.diff(m.row_ptr[ppart.bounds]))), int(np.argmax(np.diff(ppart.bounds)))}):
            pipes[f"split{slack}_rank{gp}"] = Pipe(a, m, cfg, x, slo, shi, s_slot, ppart, gp, True)
            if a.roles:
                pipes[f"split{slack}_rank{gp}_roles"] = Pipe(a, m, cfg, x, slo, shi, s_slot, ppart, gp, True, roles=True)
    if a.with_replicated:  # every rank solves the whole mesh on the gathered scores
        pipes["replicated"] = Pipe(a, m, cfg, x, slo, shi, s_slot, Partition([0, a.pods]), 0, True)
    times = {k: [] for k in pipes}
    for _ in range(reps):
        for k, p in pipes.items():
            times[k].append(p.timed(a.steps))
    out = {k: dict(p.info, pipelined_ms_per_step=float(np.median(times[k])), runs=times[k], **p.alone())
           for k, p in pipes.items()}
    del pipes, x
    torch.cuda.empty_cache()
    return dict(scoring_rank=g, ppr_bounds=bounds, pipes=out)


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
                    "runs only these, timed in alternation with the coupled uniform step")
    ap.add_argument("--reps", type=int, default=5, help="--decoupled: alternating timed runs per pipeline")
    ap.add_argument("--with-replicated", action="store_true", help="--decoupled: add the replicated solve")
    ap.add_argument("--roles", action="store_true", help="--decoupled: add role-stream pipes (scoring stream + "
                    "high-priority solve stream)")
    ap.add_argument("--grid", type=int, default=0, help="KRCA_PPR_GRID for every pipe (0: the occupancy grid)")
    ap.add_argument("--hw-queues", type=int, default=0, help="GPU_MAX_HW_QUEUES for this process (0: the environment's)")
    ap.add_argument("--iters", type=int, default=12,
                    help="PageRank steps per solve, run as a fixed-iteration solve: the emulated exchange leaves the "
                         "other ranks' slots empty, so the stop rule cannot decide here.  Default 12 = the rule's "
                         "11 iterations at C4 (bench.py ppr_iters_run) + the step that finds the convergence "
                         "(a full step here, an early exit in the real solve: conservative); 30 = rounds 2-4")
    a = ap.parse_args()
    if a.hw_queues:  # before anything starts HIP
        os.environ["GPU_MAX_HW_QUEUES"] = str(a.hw_queues)
    from krca import synth
    from krca.rca import RANKING, Partition
    M, T = 8, 1440
    m = synth.make_graph(a.pods, n_edges=a.edges, seed=0)
    hops = synth.caller_hops(m, m.roots)
    cfg = RANKING.replace(seed_floor=RANKING.floor(a.pods, M), tol=0.0, iters=a.iters)
    G = a.world
    out = dict(what=f"one rank's pipelined step at G={G} on one GPU (device copy for the all-gather)",
               pods=a.pods, edges=m.n_edges, steps=a.steps, ppr_steps_per_solve=a.iters)
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
    if a.grid:
        from krca import native
        assert native.load_library().krca_tune_set(b"KRCA_PPR_GRID", a.grid) == 0
        out["ppr_grid"] = a.grid
    if a.decoupled:
        out["decoupled_ab"] = ab_decoupled(a, m, hops, cfg, [float(v) for v in a.decoupled.split(",")], a.reps, M, T)
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
