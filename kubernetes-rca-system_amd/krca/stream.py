"""Streaming replay (BASELINE configs[4]): per-window incremental rescoring,
log histograms and warm-started re-ranking on one device.

Every window (15 s of cluster time in the C5 config) brings `delta` new metric steps per pod and
the log lines written since the previous window:

1. krca_stream_score carries the rolling z-score state forward by the new steps only (float64
   window sums, the last W samples and the exceedance bits of the last H evaluated steps stay in
   HBM), so a window costs O(P*M*delta) instead of re-reading the whole history; its outputs equal
   krca_rolling_score over the whole series so far, bit for bit.
2. The window's log text goes through krca_log_index / krca_log_match (13-pattern histograms per
   container, the reference's LogsAgent semantics applied to the window).
3. PageRank is re-seeded with the new scores and warm-started from the previous window's ranks
   (krca_ppr_shard_init_warm), iterating to the networkx L1 stop rule; the root-cause top-k
   follows as in the batch step.  Everything is integer fixed point, so each window's ranks are
   bit-identical to oracle/krca_oracle.c run on the same chain.
"""
import ctypes

from .rca import Comm, Config, DeviceShard, RcaStep


class StreamingRCA:
    def __init__(self, engine, row_ptr, col, outdeg, n_metrics, cfg=None, horizon=1440, tol=1e-9, max_iter=100,
                 check_every=4):
        import torch
        self.torch, self.eng, self.lib = torch, engine, engine.lib
        self.cfg = cfg or Config()
        self.N = int(len(outdeg))
        self.M = int(n_metrics)
        self.H = int(horizon)
        self.tol, self.max_iter, self.check_every = float(tol), int(max_iter), int(check_every)
        self.shard = DeviceShard(engine, None, row_ptr, col, outdeg, self.N, self.N, 1, self.cfg)
        self.rca = RcaStep(self.shard, Comm(), self.cfg, 0)
        dev = engine.device
        nbytes = self.lib.krca_stream_state_size(self.N, self.M, self.cfg.window, self.H)
        self.state = torch.empty(int(nbytes), dtype=torch.uint8, device=dev)
        self.out = dict(z_last=torch.empty((self.N, self.M), dtype=torch.float32, device=dev),
                        score=torch.empty(self.N, dtype=torch.float32, device=dev),
                        n_exceed=torch.empty(self.N, dtype=torch.int32, device=dev),
                        flags=torch.empty(self.N, dtype=torch.uint8, device=dev))
        self.t = 0          # metric steps consumed so far
        self.solved = False  # a previous solve exists (warm start)
        self.last_iters = 0

    def _chk(self, rc, what):
        from .native import _check
        _check(rc, what)

    # -- 1. metrics ------------------------------------------------------------------------------
    def push_metrics(self, x_new):
        """x_new float32 [delta, P, M] on the device (time-major, like the batch tensor)."""
        d, P, M = x_new.shape
        assert P == self.N and M == self.M, "stream shape mismatch"
        p = self.eng.ptr
        o = self.out
        self._chk(self.lib.krca_stream_score(p(x_new), P, M, int(d), self.t, self.cfg.window, self.H,
                                             float(self.cfg.z_threshold), p(self.state), p(o["z_last"]),
                                             p(o["score"]), p(o["n_exceed"]), p(o["flags"]), self.eng._stream()),
                  "krca_stream_score")
        self.t += int(d)
        self.shard.score_out = o
        return o

    # -- 2. logs ---------------------------------------------------------------------------------
    def push_logs(self, text, doc_off):
        """Window log text (uint8 device tensor, 16-byte aligned) and per-container offsets."""
        return self.eng.log_scan_device(text, doc_off)

    # -- 3. re-ranking ---------------------------------------------------------------------------
    def rerank(self):
        s, cfg, e, p = self.shard, self.cfg, self.eng, self.eng.ptr
        if self.solved:
            self._chk(self.lib.krca_ppr_shard_init_warm(p(s.score_out["score"]), float(cfg.seed_floor), p(s.outdeg),
                                                        s.n, s.n_max, s.N, float(cfg.alpha), p(s.ctl), p(s.q),
                                                        p(s.r), p(s.send), e._stream()), "krca_ppr_shard_init_warm")
        else:
            s.init(cfg.alpha, cfg.seed_floor)
        self.rca.comm.exchange(s)
        s.reduce(cfg.alpha, self.tol, 1)
        it_host, conv = ctypes.c_int32(0), ctypes.c_int32(0)
        for it in range(self.max_iter):
            s.step(cfg.alpha, 3)  # tol > 0: residual + ranks every iteration
            self.rca.comm.exchange(s)
            s.reduce(cfg.alpha, self.tol, 0)
            if (it + 1) % self.check_every == 0 and it + 1 < self.max_iter:
                self._chk(self.lib.krca_ppr_ctl_read(p(s.ctl), ctypes.byref(it_host), ctypes.byref(conv),
                                                     e._stream()), "krca_ppr_ctl_read")
                if conv.value:
                    break
        self._chk(self.lib.krca_ppr_ctl_read(p(s.ctl), ctypes.byref(it_host), ctypes.byref(conv), e._stream()),
                  "krca_ppr_ctl_read")
        self.last_iters = int(it_host.value) if conv.value else -int(it_host.value)
        self.solved = True
        return self.rca.merge(*s.local_topk(cfg.k))

    def window(self, x_new, log_text=None, doc_off=None):
        """One streaming window: rescoring, log histograms, re-ranking."""
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
