#!/usr/bin/env python3
"""Root-cause ranking definitions compared on planted faults — TEST INFRASTRUCTURE (CPU, the C
oracle; DESIGN.md §3.2 "Ranking").  For seeded C2-shaped meshes (10k pods / 200k edges, 8 metrics
x 1440 steps) with 10 planted root pods and their callers perturbed hop by hop (krca/synth.py),
reports the recall@10 of the planted roots for PageRank damping alpha, seed floor and ranking key
(r = propagated mass alone, r*q = mass times own anomaly, psq = mass received from callers x
sqrt(own anomaly), explained = mass received from callers x the anomaly no explaining dependency
accounts for (krca.rca.Config's default key), u = that unexplained anomaly alone (no PageRank),
recv = the mass received from callers alone (no anomaly of its own), q = anomaly alone).  Failure
models (--model): default (the root carries the largest anomaly), spread (the callers carry the
symptoms, synth.spread_hops; --spread is its old spelling) and chain (held out: two faults in one
call chain, synth.chain_roots; nothing was tuned on it).

  python tests/ranking_ablation.py [--seeds 3] [--model default|spread|chain] [--out F]
"""
import argparse
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [os.path.join(ROOT, "kubernetes-rca-system_amd"), os.path.join(ROOT, "oracle")]
import oracle  # noqa: E402
from krca import synth  # noqa: E402


def psq_key(r, q, alpha):
    """The mass a pod received from its callers (r minus its own teleport share (1 - alpha) p_i)
    times the square root of its own anomaly: an alternative key evaluated beside r and r*q."""
    rr, qq = r.astype(np.float64), q.astype(np.float64)
    p = qq / qq.sum() * 2.0 ** 60 if qq.sum() > 0 else np.zeros_like(qq)
    return (rr - (1.0 - alpha) * p) * np.sqrt(qq)


def model_mesh(model, pods, edges, seed):
    """-> (mesh with .roots = the planted roots, metrics [T, P, 8] float32 numpy) of one failure model."""
    m = synth.make_graph(pods, n_edges=edges, seed=seed)
    if model == "chain":
        m.roots = synth.chain_roots(m, seed=seed)
    hops = synth.spread_hops(m, m.roots, seed=seed) if model == "spread" else synth.caller_hops(m, m.roots)
    kw = synth.SPREAD_SIGMAS if model == "spread" else {}
    x = synth.make_metrics(pods, 8, 1440, seed=seed, roots=m.roots, hop_sets=hops, **kw).numpy()
    return m, x


def ablation_key(key, o, alpha):
    """One ranking key of a finished c_ppr_ex solve o (r, q, recv, d, key = the explained key)."""
    if key == "explained":
        return o["key"]
    if key == "rq":
        return oracle.c_rca_key(o["r"], o["q"])
    if key == "psq":
        return psq_key(o["r"], o["q"], alpha)
    if key == "u":  # the unexplained anomaly alone: the explanation pass without PageRank
        return np.maximum(o["q"] - o["d"], 0).astype(np.float64)
    if key == "recv":  # the mass received from callers alone
        return o["recv"].astype(np.float64)
    return o["r"].astype(np.float64)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, default=3)
    ap.add_argument("--pods", type=int, default=10_000)
    ap.add_argument("--edges", type=int, default=200_000)
    ap.add_argument("--out")
    ap.add_argument("--model", choices=("default", "spread", "chain"), default="default")
    ap.add_argument("--spread", action="store_true",
                    help="the anomaly spreads to the callers (synth.spread_hops: 20 sampled callers per root and "
                         "hop, 2 hops; root 8 sigma, hop h 9 * 0.9^(h-1) sigma): the callers look as anomalous "
                         "as the root, the reference's premise that symptoms show up upstream of the cause")
    a = ap.parse_args()
    if a.spread:
        a.model = "spread"
    from scipy.special import ndtri
    auto = round(float(ndtri(1.0 - 1.0 / (2.0 * a.pods * 8))), 3)  # expected max |z| of P*M null series
    defs = [(al, fl, key) for al in (0.85, 0.5) for fl in (0.0, 4.0, auto, 5.0)
            for key in ("r", "rq", "psq", "explained", "u", "recv")] + [(None, None, "q")]
    hits = {d: [] for d in defs}
    for seed in range(a.seeds):
        m, x = model_mesh(a.model, a.pods, a.edges, seed)
        s = oracle.c_rolling_score(x, 60)["score"]
        roots = set(m.roots.tolist())
        solves = {}
        for al, fl, key in defs:
            if key == "q":
                kv = s.astype(np.float64)
            else:
                if (al, fl) not in solves:
                    o = oracle.c_ppr_ex(m.row_ptr, m.col, m.outdeg, s, al, 30, 0.0, fl)
                    o["key"] = oracle.rca_keys_from(o, s, fl, m.row_ptr, m.col, "explained")  # sets o["d"]
                    solves[(al, fl)] = o
                o = solves[(al, fl)]
                kv = ablation_key(key, o, al)
            idx, _ = oracle.topk_ref(kv, 10)
            hits[(al, fl, key)].append(len(roots & set(int(i) for i in idx)) / len(roots))
    rows = [dict(alpha=al, seed_floor=fl, key=key, recall_at_10=float(np.mean(v)), per_seed=v)
            for (al, fl, key), v in hits.items()]
    txt = json.dumps(dict(config=vars(a), rows=rows), indent=1)
    if a.out:
        open(a.out, "w").write(txt + "\n")
    for r in rows:
        print(f"alpha={r['alpha']} floor={r['seed_floor']} key={r['key']:3s} recall@10={r['recall_at_10']:.2f} {r['per_seed']}")


if __name__ == "__main__":
    main()
