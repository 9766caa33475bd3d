#!/usr/bin/env python3
"""Scale goldens: networkx PageRank on synthetic meshes and the C2-mini fixture.

Test infrastructure, run by hand in the build container (`python tests/golden/capture_scale.py`);
nothing on the GPU box runs it.  It writes data only (inputs + expected outputs):

  ppr_nx_meshes.npz  two seeded meshes (2,000 nodes / 40,000 edges and 20,000 / 400,000, edges
                     stored) with anomaly seeds; networkx 3.4.2 nx.pagerank, converged (tol 1e-15)
                     under the ranking definition of krca.rca.Config (alpha 0.5, personalization
                     max(s - 4, 0) quantised to 2^-32 as the device does) and at nx's default
                     alpha 0.85 with the raw seeds; the top-10 by r_i * p_i.
  c2mini.npz         C2-mini (tests/golden/c2mini.py inputs, sha256 recorded):
                       a5  rolling z-scores: C twin (oracle/krca_oracle.c) + float64 restatement
                       a9  per-pod top-10 |Pearson r| (float64, tau = 0.5 counts)
                       a10 nx.pagerank + top-10 key under the ranking definition
                       a12 13-bin line histograms from the REFERENCE's own error_patterns
                           (ref:agents/logs_agent.py:20-34, imported read-only) and re.search
                       a13 template histograms (oracle.template_hist; new primitive, unpinned)
"""
import os
import re
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "kubernetes-rca-system_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, HERE)

SEED_FLOOR, ALPHA = 4.0, 0.5  # krca.rca.Config defaults (the ranking definition)


def quantised_personalization(seed, floor):
    """max(s - floor, 0) quantised like the device (floor((s - floor) * 2^32) / 2^32, float64)."""
    v = np.asarray(seed, np.float32).astype(np.float64) - np.float64(np.float32(floor))
    return np.where(v > 0, np.floor(v * 2.0 ** 32), 0.0) / 2.0 ** 32


def nx_rank(edges, n, pers, alpha):
    import networkx as nx
    g = nx.DiGraph()
    g.add_nodes_from(range(n))
    g.add_edges_from(map(tuple, edges.tolist()))
    pd = {i: float(pers[i]) for i in range(n)} if pers is not None else None
    r = nx.pagerank(g, alpha=alpha, personalization=pd, max_iter=10000, tol=1e-15)
    return np.array([r[i] for i in range(n)])


def topk_key(r, p, k=10):
    key = r * p
    order = np.lexsort((np.arange(len(key)), -key))
    return order[:k].astype(np.int32)


def csr(edges, n):
    """pull-CSR (row i = callers j of i, ascending) from caller -> callee edges."""
    src, dst = edges[:, 0], edges[:, 1]
    o = np.lexsort((src, dst))
    rp = np.zeros(n + 1, np.int64)
    np.cumsum(np.bincount(dst, minlength=n), out=rp[1:])
    return rp, src[o].astype(np.int32), np.bincount(src, minlength=n).astype(np.int32)


def meshes():
    from krca import synth
    out = {}
    for name, n, e, seed in (("m2k", 2000, 40_000, 11), ("m20k", 20_000, 400_000, 12)):
        m = synth.make_graph(n, n_edges=e, seed=seed)
        rows = np.repeat(np.arange(n), np.diff(m.row_ptr))
        edges = np.stack([m.col.astype(np.int64), rows], 1)  # caller -> callee
        rng = np.random.default_rng(seed)
        s = np.abs(rng.standard_normal(n)) * 1.3
        roots = rng.choice(n, 10, replace=False)
        s[roots] = rng.uniform(8, 14, 10)
        callers = np.unique(edges[np.isin(edges[:, 1], roots), 0])
        s[callers] = np.maximum(s[callers], rng.uniform(4.5, 9, len(callers)))
        s = s.astype(np.float32)
        p = quantised_personalization(s, SEED_FLOOR)
        r = nx_rank(edges, n, p, ALPHA)
        r85 = nx_rank(edges, n, s.astype(np.float64), 0.85)
        out.update({f"{name}_edges": edges.astype(np.int32), f"{name}_seed": s, f"{name}_rank": r,
                    f"{name}_top10": topk_key(r, p / p.sum()), f"{name}_rank_a085": r85,
                    f"{name}_roots": np.sort(roots)})
        print(name, "top10", out[f"{name}_top10"].tolist(), "roots", np.sort(roots).tolist())
    np.savez_compressed(os.path.join(HERE, "ppr_nx_meshes.npz"), **out)


def reference_patterns():
    """The 13 patterns as the reference's LogsAgent holds them (imported read-only)."""
    import tempfile
    from capture_reference import REF, install_stubs
    sys.dont_write_bytecode = True
    install_stubs()
    sys.path.insert(0, REF)
    cwd = os.getcwd()
    os.chdir(tempfile.mkdtemp(prefix="krca_ref_"))  # the reference writes logs into the CWD
    try:
        from agents.logs_agent import LogsAgent
        return list(LogsAgent(None).error_patterns.items())
    finally:
        os.chdir(cwd)


def c2mini():
    import c2mini as C
    import oracle
    e, x, blob, off = C.inputs()
    P = C.P
    sc = oracle.c_rolling_score(x, C.W)
    z64, s64, n64 = oracle.rolling_score_f64(x, C.W)
    z = oracle.corr_standardize(x, 0)
    cidx, cr, ccount, cgap = oracle.corr_rows(z, np.arange(P), 10, 0.5)
    seed = sc["score"]
    p = quantised_personalization(seed, SEED_FLOOR)
    r = nx_rank(e, P, p, ALPHA)
    pats = reference_patterns()
    hist = np.zeros((P, 13), np.int32)
    nl = np.zeros(P, np.int32)
    th, tc, td = [], [], []
    for d in range(P):
        text = blob[off[d]:off[d + 1]].decode("utf-8", "surrogatepass")
        lines = text.splitlines()
        nl[d] = len(lines)
        for ln in lines:
            for b, (_, pat) in enumerate(pats):
                if re.search(pat, ln, re.IGNORECASE):
                    hist[d, b] += 1
        for h, c in oracle.template_hist(text):
            th.append(h)
            tc.append(c)
            td.append(d)
    np.savez_compressed(
        os.path.join(HERE, "c2mini.npz"), sha=np.array(C.sha(e, x, off)), edges=e.astype(np.int32),
        z_last=sc["z_last"], score=sc["score"], n_exceed=sc["n_exceed"], flags=sc["flags"], z_last_f64=z64,
        n_exceed_f64=n64, corr_idx=cidx, corr_r=cr, corr_count=ccount, corr_gap=cgap, ppr_rank=r,
        ppr_top10=topk_key(r, p / p.sum()), log_lines=nl, log_hist=hist,
        tmpl_doc=np.array(td, np.int32), tmpl_hash=np.array(th, np.uint64), tmpl_count=np.array(tc, np.int32))
    print("c2mini top10", topk_key(r, p / p.sum()).tolist(), "roots", C.ROOTS, "log lines", int(nl.sum()))


def c2mini_templates():
    """Rewrite only the a13 fields of c2mini.npz from oracle.template_hist (round 5: a masked word
    became the one byte 0xFF instead of "<*>"); every other field is kept as captured."""
    import c2mini as C
    import oracle
    path = os.path.join(HERE, "c2mini.npz")
    g = dict(np.load(path))
    e, x, blob, off = C.inputs()
    assert C.sha(e, x, off) == str(g["sha"])
    th, tc, td = [], [], []
    for d in range(C.P):
        for h, c in oracle.template_hist(blob[off[d]:off[d + 1]].decode("utf-8", "surrogatepass")):
            th.append(h)
            tc.append(c)
            td.append(d)
    g.update(tmpl_doc=np.array(td, np.int32), tmpl_hash=np.array(th, np.uint64), tmpl_count=np.array(tc, np.int32))
    np.savez_compressed(path, **g)
    print("c2mini templates", len(th))


if __name__ == "__main__":
    if sys.argv[1:] == ["--templates"]:
        c2mini_templates()
    else:
        meshes()
        c2mini()
