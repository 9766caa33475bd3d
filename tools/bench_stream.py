#!/usr/bin/env python3
"""C5 streaming replay bench (BASELINE configs[4]): per-window latency of incremental rescoring +
13-pattern log histograms + error-template histograms + warm-started re-ranking, pod-sharded.

  python tools/bench_stream.py [--pods 1000000] [--windows 8] [--lines-per-window 2500000]
  python -m torch.distributed.run --nproc-per-node G --master-addr 127.0.0.1 tools/bench_stream.py

History: T = 1440 steps are streamed in first (one krca_stream_score call per rank, timed
separately).  Each window then brings delta = 1 new metric step per pod (one sample per 15 s), the
window's log text (10M lines/min over 15 s windows = 2.5M lines, one container per pod, the rank's
pods only) and a warm-started PageRank to the networkx stop rule (tol 1e-9) with one all-gather per
iteration.  The window's log text is uploaded host -> device every window (pinned staging buffer)
and timed on its own line (h2d_ms); window_ms is the device work with the text resident.
Synthetic data (krca/synth.py); the log corpus is generated once and re-sent every window.  Rank 0
prints one JSON line; times are the max over ranks.
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
    ap.add_argument("--metrics", type=int, default=8)
    ap.add_argument("--tsteps", type=int, default=1440)
    ap.add_argument("--windows", type=int, default=8)
    ap.add_argument("--no-prime", action="store_true", help="skip StreamingRCA.prime (the first window then "
                    "pays the log pass's kernel loads and workspace sizing)")
    ap.add_argument("--delta", type=int, default=1)
    ap.add_argument("--lines-per-window", type=int, default=2_500_000)
    ap.add_argument("--no-templates", action="store_true")
    ap.add_argument("--phases", action="store_true",
                    help="run the window's three parts one after another with events between them (per-part "
                         "times) instead of StreamingRCA.window (log pass beside the re-ranking)")
    a = ap.parse_args()
    import torch
    import torch.distributed as dist
    from krca import native, synth
    from krca.agents.logs import pack_documents
    from krca.rca import Comm, Config, shard_range
    from krca.stream import StreamingRCA, window_bytes
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = os.environ.get("KRCA_BENCH_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    eng = native.NativeEngine(local)
    P, M, T = a.pods, a.metrics, a.tsteps
    mesh = synth.make_graph(P, n_edges=a.edges, seed=0)
    hops = synth.caller_hops(mesh, mesh.roots)
    lo, hi, _ = shard_range(P, world, rank)
    x = synth.make_metrics_range(lo, hi, M, T + a.windows * a.delta, seed=0, roots=mesh.roots, hop_sets=hops,
                                 device=torch.device("cuda", local))
    cfg = Config()
    s = StreamingRCA(eng, mesh.row_ptr, mesh.col, mesh.outdeg, M, cfg, horizon=T, tol=1e-9, max_iter=100,
                     comm=Comm(world, rank))
    docs = synth.make_log_corpus(hi - lo, lines_per_doc=a.lines_per_window / P, seed=1 + rank, hazard_rate=0.001)
    blob, off = pack_documents(docs)
    native.check_doc_off(off, len(blob))
    eng.check_log_unicode(blob)
    n_lines = sum(d.count("\n") + (1 if d and not d.endswith("\n") else 0) for d in docs)
    if not a.no_prime:  # the log pass's kernel loads and workspace sizing, before the first window
        s.prime(len(blob), len(docs), lines_per_doc=n_lines / max(len(docs), 1), templates=not a.no_templates)
    host = torch.empty(max(len(blob), 1), dtype=torch.uint8).pin_memory()
    host[:len(blob)] = torch.frombuffer(bytearray(blob), dtype=torch.uint8)
    text = torch.empty(max(len(blob), 1), dtype=torch.uint8, device=eng.device)
    offd = torch.from_numpy(off).to(eng.device)
    torch.cuda.synchronize()

    def ev():
        return torch.cuda.Event(enable_timing=True)

    def max_over_ranks(v):
        if world == 1:
            return v
        t = torch.tensor([v], dtype=torch.float64, device=eng.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    e0, e1 = ev(), ev()
    e0.record()
    s.push_metrics(x[:T])
    e1.record()
    torch.cuda.synchronize()
    prefill_ms = max_over_ranks(e0.elapsed_time(e1))
    s.rerank()  # cold solve on the history
    torch.cuda.synchronize()
    rows = []
    t = T
    for w in range(a.windows):
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        es = [ev() for _ in range(5)]
        es[0].record()
        text[:len(blob)].copy_(host[:len(blob)], non_blocking=True)  # the window's log text, PCIe
        es[1].record()
        torch.cuda.synchronize()
        w0 = time.perf_counter()
        es[2].record()
        if a.phases:
            s.push_metrics(x[t:t + a.delta])
            es[3].record()
            s.push_logs(text[:len(blob)], offd, templates=not a.no_templates, validate=False)
            es4 = ev()
            es4.record()
            s.rerank()
        else:
            s.window(x[t:t + a.delta], text[:len(blob)], offd, validate=False, templates=not a.no_templates)
        es[4].record()
        torch.cuda.synchronize()
        wall = (time.perf_counter() - w0) * 1e3
        t += a.delta
        row = dict(h2d_ms=max_over_ranks(es[0].elapsed_time(es[1])), iters=s.last_iters,
                   device_ms=max_over_ranks(es[2].elapsed_time(es[4])), window_ms=max_over_ranks(wall))
        if a.phases:
            row.update(score_ms=max_over_ranks(es[2].elapsed_time(es[3])),
                       logs_ms=max_over_ranks(es[3].elapsed_time(es4)),
                       rerank_ms=max_over_ranks(es4.elapsed_time(es[4])))
        rows.append(row)
    med = {k: float(np.median([r[k] for r in rows])) for k in rows[0]}
    p95 = {k: float(np.percentile([r[k] for r in rows], 95)) for k in rows[0]}
    wb = window_bytes(hi - lo, M, a.delta)
    if rank == 0:
        res = {
            "metric": "C5 streaming window latency (ms): rescoring + log histograms + templates + warm re-ranking",
            "value": med["window_ms"], "unit": "ms/window", "higher_is_better": False, "n_gpus": world,
            "config": {"workload": "C5: 1M pods x 8 metrics, 1 new step per 15 s window, 2.5M log lines per window "
                                   "(10M/min), warm-started PPR to tol 1e-9, pod-sharded", "pods": P,
                       "edges": mesh.n_edges, "metrics": M, "history": T, "delta": a.delta,
                       "log_lines_per_window_rank0": n_lines, "log_bytes_per_window_rank0": len(blob),
                       "windows": a.windows, "templates": not a.no_templates, "ranks": world, "primed": not a.no_prime},
            "median": med, "p95": p95, "windows": rows, "prefill_ms": prefill_ms,
            "prefill_gbs_rank0": (4 * (hi - lo) * M * T) / (prefill_ms * 1e-3) / 1e9,
            "mode": "phases (sequential, per-part events)" if a.phases else "StreamingRCA.window (log pass on a side stream)",
            "stream_score_bytes_rank0": wb,
            "stream_score_gbs_rank0": wb / (med["score_ms"] * 1e-3) / 1e9 if a.phases else None,
            "logs_gbs_rank0": len(blob) / (med["logs_ms"] * 1e-3) / 1e9 if a.phases else None,
            "h2d_gbs_rank0": len(blob) / (med["h2d_ms"] * 1e-3) / 1e9,
            "window_incl_h2d_ms": med["window_ms"] + med["h2d_ms"],
            "data": "synthetic (krca/synth.py; one log window re-sent every window)",
        }
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
