#!/usr/bin/env python3
"""Probe: does giving the PageRank half of the pipelined C4 step its own few CUs (a CU-masked HIP
stream, hipExtStreamCreateWithCUMask) keep it from slowing the HBM-bound scoring it runs beside?

bench.py overlaps step i+1's scoring (krca_rolling_score, HBM-bound) with step i's PageRank
(latency-bound persistent kernels on every CU).  Here, on the C4 mesh: the scoring alone and the
PageRank solve alone on masked streams of several CU counts, then bench.py's two-stream pipeline
with the scoring on mask A and the PageRank on mask B.  Prints one JSON line.

  python tools/cu_mask_probe.py [--pods 1000000] [--steps 12]
"""
import argparse
import ctypes
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
    ap.add_argument("--steps", type=int, default=12)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--prio-only", action="store_true", help="only the stream-priority pipelines")
    a = ap.parse_args()
    import torch
    from krca import native, synth
    from krca.rca import RANKING, Comm, DeviceShard, RcaStep, shard_graph

    N, M, T = a.pods, 8, 1440
    cfg = RANKING.replace(seed_floor=RANKING.floor(N, M))
    m = synth.make_graph(N, n_edges=a.edges, seed=0)
    x = synth.make_metrics_range(0, N, M, T, seed=0, roots=m.roots, hop_sets=synth.caller_hops(m, m.roots),
                                 device=torch.device("cuda", 0))
    rp, col, od = shard_graph(m.row_ptr, m.col, m.outdeg, 0, N)
    engs = [native.NativeEngine(0) for _ in range(2)]
    shards = [DeviceShard(e, x, rp, col, od, N, N, 1, cfg) for e in engs]
    steps = [RcaStep(s, Comm(), cfg, 0) for s in shards]
    lib = engs[0].lib
    n_cu = torch.cuda.get_device_properties(0).multi_processor_count
    create = lib.hipExtStreamCreateWithCUMask  # resolved through libkrca's HIP runtime
    create.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32)]
    create.restype = ctypes.c_int

    def masked(cus):
        words = (n_cu + 31) // 32
        arr = (ctypes.c_uint32 * words)()
        for c in cus:
            arr[c // 32] |= 1 << (c % 32)
        h = ctypes.c_void_p()
        rc = create(ctypes.byref(h), words, arr)
        if rc != 0:
            raise RuntimeError(f"hipExtStreamCreateWithCUMask: {rc}")
        return torch.cuda.ExternalStream(h.value, device=torch.device("cuda", 0))

    def timed(stream, fn, reps):
        out = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(stream):
                e0.record()
                fn()
                e1.record()
            torch.cuda.synchronize()
            out.append(e0.elapsed_time(e1))
        return float(np.median(out))

    def ppr_solve(st):
        st.propagate()
        st.local_candidates()

    res = {"n_cu": n_cu, "pods": N, "ppr_iters": None, "scoring_alone_ms": {}, "pagerank_alone_ms": {},
           "pipeline_ms_per_step": {}}
    with torch.cuda.stream(torch.cuda.current_stream()):
        steps[0].run()  # warm: plan, workspaces, the stop rule's count
        steps[1].run()
    res["ppr_iters"] = steps[0].last_iters
    layouts = {}
    layouts["low32"] = (list(range(32, n_cu)), list(range(32)))
    for mb in (16, 32, 64):
        stride = n_cu // mb
        b = [c for c in range(n_cu) if c % stride == 0][:mb]
        layouts[f"strided{mb}"] = ([c for c in range(n_cu) if c not in set(b)], b)
    full = torch.cuda.Stream()
    res["scoring_alone_ms"]["all"] = timed(full, shards[0].score, a.reps)
    res["pagerank_alone_ms"]["all"] = timed(full, lambda: ppr_solve(steps[0]), a.reps)
    streams = {}
    for name, (ca, cb) in ([] if a.prio_only else layouts.items()):
        sa, sb = masked(ca), masked(cb)
        streams[name] = (sa, sb)
        res["scoring_alone_ms"][name + "_A"] = timed(sa, shards[0].score, a.reps)
        lib.krca_tune_set(b"KRCA_PPR_GRID", 5 * len(cb))
        res["pagerank_alone_ms"][name + "_B"] = timed(sb, lambda: ppr_solve(steps[0]), a.reps)
        lib.krca_tune_set(b"KRCA_PPR_GRID", 0)
        print(name, res["scoring_alone_ms"][name + "_A"], res["pagerank_alone_ms"][name + "_B"], flush=True)

    def pipeline(sa, sb, grid):
        lib.krca_tune_set(b"KRCA_PPR_GRID", grid)
        done = [None]
        pend = None
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(a.steps):
            j = i % 2
            with torch.cuda.stream(sa):
                if done[0] is not None:
                    sa.wait_event(done[0])
                shards[j].score()
                ev = torch.cuda.Event()
                ev.record()
                done[0] = ev
            with torch.cuda.stream(sb):
                sb.wait_event(ev)
                steps[j].propagate()
                cur = (j, *steps[j].local_candidates())
            if pend is not None:
                with torch.cuda.stream(sb):
                    steps[pend[0]].merge(*steps[pend[0]].settle(pend[1], pend[2]))
            pend = cur
        with torch.cuda.stream(sb):
            steps[pend[0]].merge(*steps[pend[0]].settle(pend[1], pend[2]))
        torch.cuda.synchronize()
        lib.krca_tune_set(b"KRCA_PPR_GRID", 0)
        return (time.perf_counter() - t0) / a.steps * 1e3

    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    lo_p, hi_p = torch.cuda.Stream.priority_range()  # (lowest, highest): a lower number is a higher priority
    ph, pl = torch.cuda.Stream(priority=hi_p), torch.cuda.Stream(priority=lo_p)
    res["priority_range"] = [lo_p, hi_p]
    for rep in range(3):
        res["pipeline_ms_per_step"].setdefault("all_all", []).append(pipeline(s1, s2, 0))
        res["pipeline_ms_per_step"].setdefault("prio_scoring_high", []).append(pipeline(ph, pl, 0))
        res["pipeline_ms_per_step"].setdefault("prio_pagerank_high", []).append(pipeline(pl, ph, 0))
        print("prio", res["pipeline_ms_per_step"]["all_all"][-1], res["pipeline_ms_per_step"]["prio_scoring_high"][-1],
              res["pipeline_ms_per_step"]["prio_pagerank_high"][-1], flush=True)
        if a.prio_only:
            continue
        for name, (sa, sb) in streams.items():
            nb = len(layouts[name][1])
            res["pipeline_ms_per_step"].setdefault(name, []).append(pipeline(sa, sb, 5 * nb))
            print(name, res["pipeline_ms_per_step"][name][-1], flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
