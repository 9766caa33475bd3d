#!/usr/bin/env python3
"""Root-cause ranking definitions on the C4 mesh (1M pods / 20M edges, 8 metrics x 1440 steps) on
the GPU, through the bench's own pieces (krca.rca.DeviceShard / RcaStep: the device scoring and
the bit-exact fixed-point PageRank).  Recall@10 of the 10 planted roots for damping alpha, seed
floor and ranking key (r = propagated mass, rq = mass x own anomaly (rounds 2-4), psq = mass received
x sqrt(own anomaly), explained = mass received x the anomaly no explaining dependency accounts for
(krca.rca.Config's key; its top-10 at the Config's alpha and floor also checked against the C
oracle), u = the unexplained anomaly alone (the explanation pass without PageRank), recv = the mass
received from callers alone (PageRank without the pod's own anomaly), q = own anomaly alone), plus
the diagnostics that explain them: each root's score s (max |z| at the last step) and its rank
among all pods, and how many pods pass each floor.  The "auto" floor is the expected maximum |z|
of P*M null series, Phi^-1(1 - 1/(2 P M)).  u and recv come from the device solve's own arrays
(q, d = krca_rca_explain's output, r, and the teleport scale the last step recorded: the
expressions of krca_rca_key_explained).  --model: default, spread or chain (the held-out model of
synth.chain_roots).

  python tools/ranking_ablation_c4.py [--pods 1000000] [--edges 20000000] [--seeds 2] [--model M] --out F
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kubernetes-rca-system_amd"))


def auto_floor(n_series):
    from scipy.special import ndtri
    return float(ndtri(1.0 - 1.0 / (2.0 * n_series)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pods", type=int, default=1_000_000)
    ap.add_argument("--edges", type=int, default=20_000_000)
    ap.add_argument("--seeds", type=int, default=2)
    ap.add_argument("--out")
    ap.add_argument("--model", choices=("default", "spread", "chain"), default="default")
    ap.add_argument("--spread", action="store_true",
                    help="the anomaly spreads to the callers (synth.spread_hops: 20 sampled callers per root and "
                         "hop, 2 hops; root 8 sigma, hop h 9 * 0.9^(h-1) sigma): the callers look as anomalous "
                         "as the root, the reference's premise that symptoms show up upstream of the cause")
    a = ap.parse_args()
    if a.spread:
        a.model = "spread"
    import torch
    from krca import native, synth
    from krca.rca import RANKING, Comm, DeviceShard, Explain, RcaStep, shard_graph
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    eng = native.NativeEngine(0)
    M, T = 8, 1440
    af = auto_floor(a.pods * M)
    floors = [0.0, 4.0, 5.0, round(af, 3), 6.0]
    defs = [(al, fl, key) for al in (0.85, 0.5) for fl in floors for key in ("r", "rq", "psq", "explained")] + \
        [(RANKING.alpha, round(af, 3), "u"), (RANKING.alpha, round(af, 3), "recv"), (None, None, "q")]
    checks = []
    hits = {d: [] for d in defs}
    diag = []
    for seed in range(a.seeds):
        t0 = time.time()
        m = synth.make_graph(a.pods, n_edges=a.edges, seed=seed)
        if a.model == "chain":
            m.roots = synth.chain_roots(m, seed=seed)
        hops = synth.spread_hops(m, m.roots, seed=seed) if a.model == "spread" else synth.caller_hops(m, m.roots)
        kw = synth.SPREAD_SIGMAS if a.model == "spread" else {}
        x = synth.make_metrics_range(0, a.pods, M, T, seed=seed, roots=m.roots, hop_sets=hops, device="cuda", **kw)
        rp, col, od = shard_graph(m.row_ptr, m.col, m.outdeg, 0, a.pods)
        sh = DeviceShard(eng, x, rp, col, od, a.pods, a.pods, 1, RANKING)
        ex = Explain(m.row_ptr, m.col)
        sh.score()
        s = sh.score_out["score"].cpu().numpy()
        roots = set(m.roots.tolist())
        order = np.argsort(-s, kind="stable")
        rank_of = np.empty(a.pods, np.int64)
        rank_of[order] = np.arange(a.pods)
        noise = np.ones(a.pods, bool)
        noise[m.roots] = False
        for h in hops:
            noise[h] = False
        diag.append(dict(seed=seed, root_scores=[float(s[r]) for r in m.roots], root_rank_by_s=[int(rank_of[r]) for r in m.roots],
                         noise_max_s=float(s[noise].max()), pods_above={str(f): int((s > f).sum()) for f in floors},
                         noise_above={str(f): int((s[noise] > f).sum()) for f in floors}))
        for al, fl, key in defs:
            if key == "q":
                idx = order[:10]
            elif key in ("u", "recv"):  # from the device arrays of the explained solve at this alpha and floor
                cfg = RANKING.replace(alpha=al, seed_floor=fl, key="explained")
                sh.cfg = cfg
                st = RcaStep(sh, Comm(), cfg, 0, explain=ex)
                st.propagate()
                st.merge(*st.settle(*st.local_candidates()))
                q, d, r = sh.q[:a.pods], sh.d[:a.pods], sh.r[:a.pods]
                hdr = sh.ctl[:40].cpu().numpy()
                q_total, tele_used = int(hdr[8:16].view(np.int64)[0]), float(hdr[32:40].view(np.float64)[0])
                if key == "u":
                    kv = torch.clamp(q - d, min=0).double()
                else:
                    t = torch.floor(q.double() * (tele_used / q_total)) if q_total > 0 else \
                        torch.full_like(q, int(tele_used / a.pods), dtype=torch.float64)
                    kv = r.double() - t
                idx = torch.topk(kv, 10).indices.cpu().numpy()  # (float keys: exact ties are rare; order not checked)
            else:
                cfg = RANKING.replace(alpha=al, seed_floor=fl, key="rq" if key != "explained" else key)
                sh.cfg = cfg
                st = RcaStep(sh, Comm(), cfg, 0, explain=ex)
                st.propagate()
                if key in ("rq", "explained"):
                    idx, _ = st.merge(*st.settle(*st.local_candidates()))
                    if key == "explained" and al == RANKING.alpha and fl == round(af, 3):
                        ref, _, _ = oracle.rca_rank(m.row_ptr, m.col, m.outdeg, s, al, cfg.iters, fl, 10, tol=cfg.tol)
                        checks.append(dict(seed=seed, top10_identical=[int(i) for i in idx] == ref.tolist()))
                elif key == "psq":  # mass received from callers x sqrt(own anomaly) (tests/ranking_ablation.py)
                    rr, qq = sh.r[:a.pods].double(), sh.q[:a.pods].double()
                    p = qq / qq.sum() * 2.0 ** 60 if float(qq.sum()) > 0 else torch.zeros_like(qq)
                    idx = torch.topk((rr - (1.0 - al) * p) * qq.sqrt(), 10).indices.cpu().numpy()
                else:
                    idx = torch.topk(sh.r[:a.pods], 10).indices.cpu().numpy()
            hits[(al, fl, key)].append(len(roots & set(int(i) for i in idx)) / len(roots))
        print(f"seed {seed}: {time.time() - t0:.0f}s; roots s={np.round(diag[-1]['root_scores'], 2).tolist()} "
              f"rank_by_s={diag[-1]['root_rank_by_s']} noise_max_s={diag[-1]['noise_max_s']:.2f}", flush=True)
        del x, sh
        torch.cuda.empty_cache()
    rows = [dict(alpha=al, seed_floor=fl, key=key, recall_at_10=float(np.mean(v)), per_seed=v)
            for (al, fl, key), v in hits.items()]
    out = dict(config=dict(vars(a), metrics=M, tsteps=T, window=RANKING.window, auto_floor=af), rows=rows,
               diagnostics=diag, oracle_checks=checks)
    txt = json.dumps(out, indent=1)
    if a.out:
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        open(a.out, "w").write(txt + "\n")
    for r in rows:
        print(f"alpha={r['alpha']} floor={r['seed_floor']} key={r['key']:3s} recall@10={r['recall_at_10']:.2f} "
              f"{r['per_seed']}", flush=True)
    print("oracle checks:", checks, flush=True)


if __name__ == "__main__":
    main()
