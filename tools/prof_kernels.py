#!/usr/bin/env python3
"""Short driver for rocprofv3 runs (kernel trace / PMC passes) of single krca kernels.

  python tools/prof_kernels.py score  [--pods 1000000] [--reps 3]
  python tools/prof_kernels.py ppr    [--pods 1000000] [--reps 3]
  python tools/prof_kernels.py logs   [--docs 1000000] [--reps 3]
  python tools/prof_kernels.py corr   [--pods 100000] [--reps 3]
  python tools/prof_kernels.py tmpl   [--docs 1000000] [--reps 3]   (a13 template hashing + histograms)
  python tools/prof_kernels.py f2     [--pods 1000000] [--reps 3]   (selector bit matrix + env DNS matches)
  python tools/prof_kernels.py bc     [--pods 20000]  [--reps 1]    (f3 betweenness)
Prints per-kernel event-timed averages and the algorithmic bytes.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kubernetes-rca-system_amd"))


def timed(torch, fn, reps):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return [a.elapsed_time(b) for a, b in ev]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("what", choices=["score", "ppr", "logs", "corr", "pods", "bc", "events", "tmpl", "f2"])
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--pods", type=int, default=1_000_000)
    ap.add_argument("--docs", type=int, default=1_000_000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--tsteps", type=int, default=1440)
    ap.add_argument("--tau", type=float, default=0.5)
    a = ap.parse_args()
    import torch
    from krca import native, synth
    eng = native.NativeEngine(0)
    out = {}
    if a.what == "score":
        x = synth.make_metrics(a.pods, 8, a.tsteps, device="cuda")
        o = eng.rolling_score_device(x)
        ms = timed(torch, lambda: eng.rolling_score_device(x, out=o), a.reps)
        nbytes = 4 * a.pods * 8 * a.tsteps + 4 * a.pods * 8 + 9 * a.pods
        out = dict(kernel="krca_rolling_score", ms=ms, bytes=nbytes, gbs=nbytes / (min(ms) * 1e-3) / 1e9)
    elif a.what == "ppr":
        from krca.rca import Comm, Config, DeviceShard, RcaStep, shard_graph, shard_range
        m = synth.make_graph(a.pods, avg_degree=20, seed=0)
        x = synth.make_metrics(a.pods, 8, 64, device="cuda", roots=m.roots)
        cfg = Config(iters=30, window=30)
        rp, col, od = shard_graph(m.row_ptr, m.col, m.outdeg, 0, a.pods)
        sh = DeviceShard(eng, x, rp, col, od, a.pods, a.pods, 1, cfg)
        step = RcaStep(sh, Comm(), cfg, 0)
        step.run()
        ms = timed(torch, lambda: step.run(to_host=False), a.reps)
        N, E = a.pods, m.n_edges
        per_iter = 8 * (N + 1) + 4 * E + 8 * N + 8 * N + 8 * N  # row_ptr, col, w(compulsory), acc, w out
        out = dict(kernel="ppr step (30 it)", ms=ms, edges=E, bytes_per_iter=per_iter)
    elif a.what == "corr":
        x = synth.make_metrics(a.pods, 1, a.tsteps, device="cuda", group_size=20)
        z = eng.corr_prepare_device(x)
        r = eng.corr_topk_device(z, 10, a.tau)
        ms_prep = timed(torch, lambda: eng.corr_prepare_device(x), a.reps)
        ms = timed(torch, lambda: eng.corr_topk_device(z, 10, a.tau, out=r), a.reps)
        P, T = a.pods, a.tsteps
        flops = P * (P + 1) * T  # upper triangle incl. diagonal, 2 flops per MAC
        ws = eng._ws["corr_cand"].view(torch.int32)
        cap = eng.lib.krca_corr_cand_cap()
        cnt = ws[2 * P * cap: 2 * P * cap + P].float()  # candidates per pod (appends, not clipped at cap)
        out = dict(kernel="corr top-k", ms=ms, ms_prepare=ms_prep, flops=flops,
                   tflops=flops / (min(ms) * 1e-3) / 1e12, certified=float((r["cert"] > 0).float().mean()),
                   cand_over=int((cnt > cap).sum()),
                   cand_mean=float(cnt.mean()), cand_max=float(cnt.max()), cand_p99=float(cnt.quantile(0.99)))
    elif a.what == "bc":
        # f3: betweenness over a strongly connected service graph (each node links to 2 random
        # earlier nodes, both directions: the worst case, every source reaches every node)
        N = a.pods
        rng = np.random.default_rng(0)
        v = np.repeat(np.arange(1, N, dtype=np.int64), 2)
        u = (rng.random(len(v)) * v).astype(np.int64)
        key = np.unique(np.concatenate([u * N + v, v * N + u]))
        src, dst = key // N, key % N
        rp = np.zeros(N + 1, np.int64)
        np.cumsum(np.bincount(src, minlength=N), out=rp[1:])
        col = dst.astype(np.int32)
        eng.betweenness(rp, col, batch=a.batch)
        t0 = time.perf_counter()
        for _ in range(a.reps):
            bc = eng.betweenness(rp, col, batch=a.batch)
        s = (time.perf_counter() - t0) / a.reps
        E = len(col)
        # per source: the forward BFS and the dependency pull each read every reached edge once
        out = dict(kernel="krca_betweenness", nodes=N, edges=E, s=s, teps=2 * N * E / s, bc_sum=float(bc.sum()))
    elif a.what == "events":
        from krca import eventcols
        E = a.pods * 10  # default 10M events
        t0 = time.time()
        cols = eventcols.make_events(E, seed=0, n_hosts=1024)
        slot, key, layout = eventcols.group_records(cols)
        t_host = time.time() - t0
        S = layout[-1][0] + layout[-1][1]
        ds, dk = torch.from_numpy(slot).cuda(), torch.from_numpy(key).cuda()
        eng.group_reduce_device(ds, dk, S, 3, n_ranked=E)
        ms = timed(torch, lambda: eng.group_reduce_device(ds, dk, S, 3, n_ranked=E), a.reps)
        # algorithmic: one read of the records (12 B), the object records again for ranks 2-3
        # (2 x 12 B + an 8-B top gather), one 64-B slot record written
        nbytes = 12 * len(slot) + 2 * 20 * E + 64 * S
        out = dict(kernel="krca_group_reduce", events=E, records=len(slot), slots=S, ms=ms, bytes=nbytes,
                   gbs=nbytes / (min(ms) * 1e-3) / 1e9, host_records_s=t_host)
    elif a.what == "pods":
        from krca import podstate
        P = a.pods * 10
        pc, off, cc = podstate.make_pod_states(P, seed=0)
        d = [torch.from_numpy(pc).cuda(), torch.from_numpy(off).cuda(), torch.from_numpy(cc.view(np.int16)).cuda()]
        eng.pod_classify_device(*d)
        ms = timed(torch, lambda: eng.pod_classify_device(*d), a.reps)
        nbytes = P * (1 + 8 + 2) + 8 + 2 * len(cc)
        out = dict(kernel="krca_pod_classify", pods=P, containers=len(cc), ms=ms, bytes=nbytes,
                   gbs=nbytes / (min(ms) * 1e-3) / 1e9)
    elif a.what == "tmpl":
        from krca.agents.logs import pack_documents
        docs = synth.make_log_corpus(a.docs, lines_per_doc=2.5, seed=0, hazard_rate=0.001)
        blob, off = pack_documents(docs)
        scan = eng.log_scan_device(eng.upload_blob(blob), torch.from_numpy(off).cuda())
        eng.template_hist_device(scan)
        ms = timed(torch, lambda: eng.template_hist_device(scan), a.reps)
        L = scan["n_lines_total"]
        # text once, line offsets (16 B) read, hashes (8 B) written, histogram pass (8 B in, 12 B out)
        nbytes = len(blob) + 16 * L + 8 * L + 20 * L
        out = dict(kernel="template hash + histograms", ms=ms, lines=L, docs=a.docs, bytes=nbytes,
                   gbs=nbytes / (min(ms) * 1e-3) / 1e9)
    elif a.what == "f2":
        # selector test: D objects with 6 label items each (interned ids from 4096), S = 256 selectors
        # of 1-3 items; env DNS inference: V env values (~48 B) against the 4 DNS keys of 2,000 services
        rng = np.random.default_rng(0)
        D, S = a.pods, 256
        lab = np.sort(rng.integers(0, 4096, (D, 6)), axis=1).astype(np.int32).ravel()
        lab_off = np.arange(0, 6 * D + 1, 6, dtype=np.int64)
        sl = rng.integers(1, 4, S)
        sel = np.concatenate([np.sort(rng.choice(4096, k, replace=False)) for k in sl]).astype(np.int32)
        sel_off = np.concatenate([[0], np.cumsum(sl)]).astype(np.int64)
        eng.selector_match(lab, lab_off, sel, sel_off)
        t0 = time.perf_counter()
        for _ in range(a.reps):
            bits = eng.selector_match(lab, lab_off, sel, sel_off)
        sel_s = (time.perf_counter() - t0) / a.reps
        names = [f"svc-{i:04d}" for i in range(2000)]
        keys = [f"{n}{suf}" for n in names for suf in ("", ".default", ".default.svc", ".default.svc.cluster.local")]
        V = a.pods // 10
        vals = [f"http://{names[rng.integers(2000)]}.default.svc:8080/api/v{i % 7}" if i % 3 else f"value-{i}"
                for i in range(V)]
        from krca import topograph
        eng.substr_match(*topograph.pack_strings(vals), *topograph.pack_strings(keys))
        t0 = time.perf_counter()
        for _ in range(a.reps):
            pairs = eng.substr_match(*topograph.pack_strings(vals), *topograph.pack_strings(keys))
        sub_s = (time.perf_counter() - t0) / a.reps
        out = dict(kernel="f2 selector + substring", objects=D, selectors=S, selector_s=sel_s,
                   hits=int(np.unpackbits(bits.view(np.uint8)).sum()), env_values=V, keys=len(keys), substr_s=sub_s,
                   pairs=len(pairs))
    else:
        from krca.agents.logs import pack_documents
        docs = synth.make_log_corpus(a.docs, lines_per_doc=2.5, seed=0, hazard_rate=0.001)
        blob, off = pack_documents(docs)
        text = eng.upload_blob(blob)
        offd = torch.from_numpy(off).cuda()
        eng.log_scan_device(text, offd)
        ms = timed(torch, lambda: eng.log_scan_device(text, offd), a.reps)
        L = sum(d.count("\n") + (1 if d and not d.endswith("\n") else 0) for d in docs[:1000]) / 1000 * a.docs
        out = dict(kernel="log scan", ms=ms, bytes=len(blob), lines=L, docs=a.docs,
                   gbs=len(blob) / (min(ms) * 1e-3) / 1e9)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
