"""Streaming replay (BASELINE configs[4]): per-window incremental rescoring,
log histograms + error templates and warm-started re-ranking, pod-sharded over G ranks.

Every window (15 s of cluster time in the C5 config) brings `delta` new metric steps per pod and
the log lines written since the previous window.  Rank g of G owns pods [g*n_max, ...) (the
partition of krca/rca.py): their metric stream, their containers' logs and their rows of the
pull-CSR.

1. krca_stream_score carries the rank's rolling z-score state forward by the new steps only
   (float64 window sums, the last W samples and the exceedance bits of the last H evaluated steps
   stay in HBM), so a window costs O(n_local*M*delta) instead of re-reading the history; its
   outputs equal krca_rolling_score over the whole series so far, bit for bit.  No communication.
2. The window's log text of the rank's containers goes through krca_log_index / krca_log_match
   (13-pattern histograms per container, the reference's LogsAgent semantics,
   ref:agents/logs_agent.py:147-151) and krca_template_hash / krca_template_hist (error-template
   histograms per container).  No communication.
3. PageRank is re-seeded with the new scores and warm-started from the previous window's ranks
   (krca_ppr_shard_init_warm), iterating to the networkx L1 stop rule with ONE all-gather per
   iteration (Comm.exchange; G = 1: a buffer swap); the root-cause top-k merges G x k candidates.
   Integer fixed point: each window's ranks are bit-identical to oracle/krca_oracle.c run on the
   same chain, for any G.

The per-rank numeric work sits behind the shard interface of krca/rca.py (DeviceShard; the CPU
tests drive the same orchestration with tests/numpy_shard.py over gloo).
"""
from .rca import Comm, Config, DeviceShard, RcaStep, shard_graph, shard_range


class StreamingRCA:
    def __init__(self, engine, row_ptr, col, outdeg, n_metrics, cfg=None, horizon=1440, tol=1e-9, max_iter=100,
                 check_every=4, comm=None, shard=None):
        """row_ptr / col / outdeg: the whole mesh's pull-CSR (host arrays); this rank keeps its rows.
        comm: krca.rca.Comm (world, rank) — default one rank.  shard: a prepared per-rank backend
        (tests); default DeviceShard on `engine`."""
        self.eng = engine
        self.cfg = cfg or Config()
        self.comm = comm or Comm()
        self.N = int(len(outdeg))
        self.M = int(n_metrics)
        self.H = int(horizon)
        self.tol, self.max_iter, self.check_every = float(tol), int(max_iter), int(check_every)
        self.lo, self.hi, self.n_max = shard_range(self.N, self.comm.world, self.comm.rank)
        if shard is None:
            rp, c, od = shard_graph(row_ptr, col, outdeg, self.lo, self.hi)
            shard = DeviceShard(engine, None, rp, c, od, self.N, self.n_max, self.comm.world, self.cfg)
        self.shard = shard
        self.rca = RcaStep(self.shard, self.comm, self.cfg, self.lo)
        self.t = 0          # metric steps consumed so far
        self.solved = False  # a previous solve exists (warm start)
        self.last_iters = 0

    # -- 1. metrics ------------------------------------------------------------------------------
    def push_metrics(self, x_new):
        """x_new float32 [delta, n_local, M] (time-major, this rank's pods [lo, hi))."""
        d, P, M = x_new.shape
        if P != self.hi - self.lo or M != self.M:
            raise ValueError(f"stream window shape {tuple(x_new.shape)}: rank owns {self.hi - self.lo} pods x {self.M}")
        o = self.shard.stream_score(x_new, self.t, self.H)
        self.t += int(d)
        return o

    # -- 2. logs ---------------------------------------------------------------------------------
    def push_logs(self, text, doc_off, templates=True, validate=True):
        """Window log text of this rank's containers (uint8 device tensor, 16-byte aligned) and its
        container offsets (int64 device tensor): 13-bin histograms (+ template histograms)."""
        scan = self.eng.log_scan_device(text, doc_off, validate=validate)
        if templates:
            scan["templates"] = self.eng.template_hist_device(scan)
        return scan

    # -- 3. re-ranking ---------------------------------------------------------------------------
    def rerank(self):
        s, cfg = self.shard, self.cfg
        if self.solved:
            s.init_warm(cfg.alpha, cfg.floor(s.N, s.M))
        else:
            s.init(cfg.alpha, cfg.floor(s.N, s.M))
        self.comm.exchange(s)
        s.reduce(cfg.alpha, self.tol, 1)
        for it in range(self.max_iter):
            s.step(cfg.alpha, 3)  # tol > 0: residual + ranks every iteration
            self.comm.exchange(s)
            s.reduce(cfg.alpha, self.tol, 0)
            if (it + 1) % self.check_every == 0 and it + 1 < self.max_iter and s.ctl_read()[1]:
                break
        iters, conv = s.ctl_read()
        self.last_iters = iters if conv else -iters
        self.solved = True
        return self.rca.merge(*s.local_topk(cfg.k))

    def window(self, x_new, log_text=None, doc_off=None):
        """One streaming window: rescoring, log histograms (+ templates), re-ranking."""
        out = {"scores": self.push_metrics(x_new)}
        if log_text is not None:
            out["logs"] = self.push_logs(log_text, doc_off)
        out["top"] = self.rerank()
        out["iters"] = self.last_iters
        return out


def window_bytes(P, M, delta):
    """Algorithmic HBM bytes of one krca_stream_score call: state 20 B per series
    read + written; per step 4 B new, 4 B old and 4 B ring write per series, 8 B exceedance word
    read + written; outputs 4*M + 9 B per pod."""
    S = P * M
    return S * (40 + 20 * delta) + P * (4 * M + 9)
