"""CPU stand-in for krca.native.NativeEngine, built from oracle/ — TESTS ONLY.

It lets the CPU test suite exercise the agents' host logic (findings formatting, ordering,
error contracts) against the reference goldens without a GPU.  The product path never uses
it: krca.native.default_engine() has no CPU fallback.
"""
import numpy as np

import oracle


class OracleLogScan:
    def __init__(self, docs):
        self.n_lines, self.hist, self._ex = [], [], []
        for text in docs:
            n, h, ex = oracle.log_hist(text)
            self.n_lines.append(n)
            self.hist.append(h)
            self._ex.append(ex)
        self.n_lines = np.asarray(self.n_lines, np.int32)
        self.hist = np.asarray(self.hist, np.int32).reshape(-1, 13)

    def examples(self, d, c):
        return self._ex[d][c]


class OracleEngine:
    def usage_flags(self, usage):
        return oracle.c_usage_flags(usage)

    def rolling_score(self, x, window=60, z_threshold=3.0):
        x = np.asarray(x.cpu() if hasattr(x, "cpu") else x, np.float32)
        r = oracle.c_rolling_score(x, window, z_threshold)
        r["n_exceed_host"] = r["n_exceed"]
        r["_x"] = x
        return r

    def gather_last(self, x, idx):
        x = np.asarray(x.cpu() if hasattr(x, "cpu") else x, np.float32)
        return x[-1][np.asarray(idx, np.int64)]

    def topk(self, v, k):
        v = np.asarray(v.cpu() if hasattr(v, "cpu") else v)
        return oracle.topk_ref(v, k)

    def log_scan(self, blob, doc_off):
        docs = [blob[doc_off[i]:doc_off[i + 1]].decode("utf-8", "surrogatepass") for i in range(len(doc_off) - 1)]
        return OracleLogScan(docs)

    def rank_root_causes(self, seed, row_ptr, col, outdeg, cfg=None, k=None, n_metrics=1):
        from krca.rca import RANKING
        cfg = cfg or RANKING
        seed = np.asarray(seed.cpu() if hasattr(seed, "cpu") else seed, np.float32)
        k = min(int(k or cfg.k), len(outdeg))
        key, o = oracle.rca_keys(row_ptr, col, outdeg, seed, cfg.alpha, cfg.iters, cfg.floor(len(outdeg), n_metrics),
                                 key=cfg.key, tol=cfg.tol)
        idx, _ = oracle.topk_ref(key, k)
        rr = o["r"].astype(np.float64) / 2.0 ** 60
        qt = float(o["q"].sum())
        val = key[idx].view(np.float64) / (2.0 ** 60 * qt) if qt > 0 else np.zeros(len(idx))
        return idx, val, rr

    def pod_classify(self, pod_code, cont_off, cont_code):
        return oracle.pod_classify_ref(pod_code, cont_off, cont_code)

    def betweenness(self, row_ptr, col, normalized=True, directed=True, batch=1024):
        import networkx as nx
        N = len(row_ptr) - 1
        g = nx.DiGraph() if directed else nx.Graph()
        g.add_nodes_from(range(N))
        for u in range(N):
            for e in range(row_ptr[u], row_ptr[u + 1]):
                g.add_edge(u, int(col[e]))
        bc = nx.betweenness_centrality(g, normalized=normalized)
        return np.array([bc[i] for i in range(N)])

    def selector_match(self, lab, lab_off, sel, sel_off):
        return oracle.selector_match_ref(lab, lab_off, sel, sel_off)

    def substr_match(self, text, val_off, pat, pat_off):
        return oracle.substr_match_ref(text, val_off, pat, pat_off)

    def group_reduce(self, slot, key, S, R=1, n_ranked=None):
        return oracle.group_reduce_ref(slot, key, S, R, n_ranked)
