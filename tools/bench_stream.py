#!/usr/bin/env python3
"""C5 streaming replay bench (BASELINE configs[4]) on one device: per-window latency of
incremental rescoring + 13-pattern log histograms + warm-started re-ranking.

  python tools/bench_stream.py [--pods 1000000] [--windows 8] [--lines-per-window 2500000]

History: T = 1440 steps are streamed in first (one krca_stream_score call over the 46 GB tensor,
timed separately).  Each window then brings delta = 1 new metric step per pod (one sample per
15 s), 2.5M log lines (10M lines/min over 15 s windows) and a warm-started PageRank to the
networkx stop rule (tol 1e-9).  Synthetic data: the mesh generator of krca/synth.py; the window's
log corpus is generated once and re-scanned every window.  Prints one JSON line.
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
    ap.add_argument("--metrics", type=int, default=8)
    ap.add_argument("--tsteps", type=int, default=1440)
    ap.add_argument("--windows", type=int, default=8)
    ap.add_argument("--delta", type=int, default=1)
    ap.add_argument("--lines-per-window", type=int, default=2_500_000)
    a = ap.parse_args()
    import torch
    from krca import native, synth
    from krca.agents.logs import pack_documents
    from krca.rca import Config
    from krca.stream import StreamingRCA, window_bytes
    eng = native.NativeEngine(0)
    P, M, T = a.pods, a.metrics, a.tsteps
    mesh = synth.make_graph(P, avg_degree=20, seed=0)
    hops = synth.caller_hops(mesh, mesh.roots)
    x = synth.make_metrics(P, M, T + a.windows * a.delta, seed=0, roots=mesh.roots, hop_sets=hops, device="cuda")
    cfg = Config()
    s = StreamingRCA(eng, mesh.row_ptr, mesh.col, mesh.outdeg, M, cfg, horizon=T, tol=1e-9, max_iter=100)
    docs = synth.make_log_corpus(P, lines_per_doc=a.lines_per_window / P, seed=1, hazard_rate=0.001)
    blob, off = pack_documents(docs)
    text = eng.upload_blob(blob)
    offd = torch.from_numpy(off).cuda()
    n_lines = sum(d.count("\n") + (1 if d and not d.endswith("\n") else 0) for d in docs)
    torch.cuda.synchronize()

    def ev():
        return torch.cuda.Event(enable_timing=True)

    e0, e1 = ev(), ev()
    e0.record()
    s.push_metrics(x[:T])
    e1.record()
    torch.cuda.synchronize()
    prefill_ms = e0.elapsed_time(e1)
    s.rerank()  # cold solve on the history
    torch.cuda.synchronize()
    rows = []
    t = T
    for w in range(a.windows):
        es = [ev() for _ in range(4)]
        w0 = time.perf_counter()
        es[0].record()
        s.push_metrics(x[t:t + a.delta])
        es[1].record()
        s.push_logs(text, offd)
        es[2].record()
        top, _ = s.rerank()
        es[3].record()
        torch.cuda.synchronize()
        wall = (time.perf_counter() - w0) * 1e3
        t += a.delta
        rows.append(dict(score_ms=es[0].elapsed_time(es[1]), logs_ms=es[1].elapsed_time(es[2]),
                         rerank_ms=es[2].elapsed_time(es[3]), iters=s.last_iters, wall_ms=wall))
    med = {k: float(np.median([r[k] for r in rows])) for k in rows[0]}
    wb = window_bytes(P, M, a.delta)
    res = {
        "metric": "C5 streaming window latency (ms): rescoring + log histograms + warm re-ranking",
        "value": med["wall_ms"], "unit": "ms/window", "higher_is_better": False, "n_gpus": 1,
        "config": {"workload": "C5: 1M pods x 8 metrics, 1 new step per 15 s window, 2.5M log lines per window "
                               "(10M/min), warm-started PPR to tol 1e-9",
                   "pods": P, "edges": mesh.n_edges, "metrics": M, "history": T, "delta": a.delta,
                   "log_lines_per_window": n_lines, "log_bytes_per_window": len(blob), "windows": a.windows},
        "median": med, "windows": rows, "prefill_ms": prefill_ms,
        "prefill_gbs": (4 * P * M * T) / (prefill_ms * 1e-3) / 1e9,
        "stream_score_bytes": wb, "stream_score_gbs": wb / (med["score_ms"] * 1e-3) / 1e9,
        "logs_gbs": len(blob) / (med["logs_ms"] * 1e-3) / 1e9,
        "data": "synthetic (krca/synth.py; one log window reused)",
    }
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
