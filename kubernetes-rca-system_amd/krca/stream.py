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

4. Between windows a rank can snapshot its stream (rolling state, warm-start ranks, step count)
   to a file and a new process restore it: the stream then continues bit for bit.

The per-rank numeric work sits behind the shard interface of krca/rca.py (DeviceShard; the CPU
tests drive the same orchestration with tests/numpy_shard.py over gloo).
"""
import json

import numpy as np

from .rca import Comm, Config, DeviceShard, Explain, Partition, RcaStep, shard_graph

SNAPSHOT_VERSION = 1


class StreamingRCA:
    def __init__(self, engine, row_ptr, col, outdeg, n_metrics, cfg=None, horizon=1440, tol=1e-9, max_iter=100,
                 check_every=4, comm=None, shard=None, partition=None):
        """row_ptr / col / outdeg: the whole mesh's pull-CSR (host arrays); this rank keeps its rows.
        comm: krca.rca.Comm (world, rank) — default one rank.  shard: a prepared per-rank backend
        (tests); default DeviceShard on `engine`.  partition: a krca.rca.Partition, or "balanced"
        (pods + in-edges balanced ranges); default uniform ranges of ceil(N / G) pods."""
        self.eng = engine
        self.cfg = cfg or Config()
        self.comm = comm or Comm()
        self.N = int(len(outdeg))
        self.M = int(n_metrics)
        self.H = int(horizon)
        self.tol, self.max_iter, self.check_every = float(tol), int(max_iter), int(check_every)
        if partition == "balanced":
            partition = Partition.balanced(row_ptr, self.comm.world)
        self.part = partition or Partition.uniform(self.N, self.comm.world)
        self.lo, self.hi, self.n_max = self.part.range(self.comm.rank)
        if shard is None:
            rp, c, od = shard_graph(row_ptr, col, outdeg, self.lo, self.hi, self.part)
            shard = DeviceShard(engine, None, rp, c, od, self.N, self.n_max, self.comm.world, self.cfg,
                                pingpong=not self.comm.collective)
        self.shard = shard
        self.rca = RcaStep(self.shard, self.comm, self.cfg, self.lo, part=self.part,
                           explain=Explain(row_ptr, col) if self.cfg.key == "explained" else None)
        self.t = 0          # metric steps consumed so far
        self.solved = False  # a previous solve exists (warm start)
        self.last_iters = 0
        # the side stream of window()'s log pass, created here rather than in the first window (its
        # creation cost 7.5 ms of the first window's 8x-steady-state time in round 3)
        self._side = None
        if isinstance(self.shard, DeviceShard):
            self._side = engine.torch.cuda.Stream(device=engine.device)

    def prime(self, log_bytes, n_docs, lines_per_doc=2.5, templates=True):
        """Pay the log pass's one-time costs before the first window instead of in it: a synthetic
        text of `log_bytes` bytes in `n_docs` containers (`lines_per_doc` lines each) is scanned (and
        template-hashed) on the side stream.  That loads the log kernels' code and sizes the
        engine's line arrays and workspaces for windows of that size (a first window paid 7-8x the
        steady-state time for them).  No stream state changes: ranks, metric history, the
        iteration count stay as they were."""
        import numpy as np
        torch = self.eng.torch
        n_docs = max(int(n_docs), 1)
        n_lines = max(int(n_docs * lines_per_doc), n_docs)
        L = max(int(log_bytes) // n_lines, 2)
        line = np.full(L, ord("x"), np.uint8)
        line[-1] = ord("\n")
        blob = np.tile(line, n_lines)
        per = n_lines // n_docs
        off = np.minimum(np.arange(n_docs + 1, dtype=np.int64) * per * L, len(blob))
        off[-1] = len(blob)
        text = self.eng.upload_blob(blob.tobytes())
        offd = torch.from_numpy(off).to(self.eng.device)
        side = self._side or torch.cuda.current_stream(self.eng.device)
        side.wait_stream(torch.cuda.current_stream(self.eng.device))
        with torch.cuda.stream(side):
            logs = self.push_logs(text, offd, templates=templates, validate=False, _defer=True)
            if templates:
                self.eng.template_hist_finish(logs.get("templates", {}))
        side.synchronize()

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
    def push_logs(self, text, doc_off, templates=True, validate=True, _defer=False):
        """Window log text of this rank's containers (uint8 device tensor, 16-byte aligned) and its
        container offsets (int64 device tensor): 13-bin histograms (+ template histograms)."""
        scan = self.eng.log_scan_device(text, doc_off, validate=validate)
        if templates:
            scan["templates"] = self.eng.template_hist_device(scan, defer_huge=_defer)
        return scan

    # -- 3. re-ranking ---------------------------------------------------------------------------
    def rerank(self):
        return self._rerank_end(self._rerank_begin())

    def _rerank_begin(self):
        """Enqueue the re-rank's first part without synchronising: init (warm from the previous
        window's ranks), and for a warm stream the speculative first batch -- the previous window's
        iteration count + 1 folded steps (the last one tests the count), the last step's reduction,
        the key and the local top-k."""
        s, cfg = self.shard, self.cfg
        warm = self.solved
        if warm:
            s.init_warm(cfg.alpha, cfg.floor(s.N, s.M))
        else:
            s.init(cfg.alpha, cfg.floor(s.N, s.M))
        self.comm.exchange(s)
        st = dict(it=0, spec=None)
        if warm and self.last_iters > 0:
            # windows change little, so this usually converges: no step is launched past
            # convergence and the GPU never waits on a host poll.  Otherwise the candidates are
            # dropped (the finish and the key only read the state) and _rerank_end continues in
            # polled batches from step `it`.
            it = 0
            for _ in range(min(self.last_iters + 1, self.max_iter)):
                it += 1
                s.step_folded(cfg.alpha, self.tol, it, 3)
                self.comm.exchange(s)
            s.finish(cfg.alpha, self.tol, it)
            h = s.ctl_async()
            st.update(it=it, spec=(h, self.rca.local_candidates()))
        return st

    def _rerank_end(self, st):
        s, cfg = self.shard, self.cfg
        it = st["it"]
        if st["spec"] is not None:
            h, cand = st["spec"]
            top = self.rca.merge(*cand)
            iters, conv = s.ctl_wait(h)
            if conv or it >= self.max_iter:
                self.last_iters = iters if conv else -iters
                return top
        # folded iterations (each step reduces the previous one: one kernel + one exchange) in
        # batches of check_every; the convergence flag of batch b is read while batch b + 1 runs (a
        # pinned copy + event): the GPU never idles on the poll, and iterations enqueued past
        # convergence do nothing (the kernels exit on the device-held flag), so the ranks and the
        # iteration count are the same as with a synchronous check after every batch
        pending = None
        while it < self.max_iter:
            for _ in range(min(self.check_every, self.max_iter - it)):
                it += 1
                s.step_folded(cfg.alpha, self.tol, it, 3)  # tol > 0: residual + ranks every iteration
                self.comm.exchange(s)
            if pending is not None and s.ctl_wait(pending)[1]:
                break
            pending = s.ctl_async() if it < self.max_iter else None
        s.finish(cfg.alpha, self.tol, it)
        # the final counts ride behind the key / top-k launches: one synchronisation (the merge's
        # copy of the candidates) instead of a read-back before them
        h = s.ctl_async()
        top = self.rca.merge(*self.rca.local_candidates())
        iters, conv = s.ctl_wait(h)
        self.last_iters = iters if conv else -iters
        self.solved = True
        return top

    def window(self, x_new, log_text=None, doc_off=None, validate=True, templates=True):
        """One streaming window: rescoring, log histograms (+ templates), re-ranking.

        With log text, the log pass runs on a second HIP stream beside the re-ranking: the
        re-rank's first part is enqueued first (it needs the new scores only), then the log scan
        and the template pass go out on the side stream while those PageRank steps run (the scan's
        one synchronisation waits for the side stream only), and the templates' read-back of the
        oversized-container count comes after the re-rank's merge.  Outputs as without overlap."""
        if log_text is None:
            out = {"scores": self.push_metrics(x_new)}
            out["top"] = self.rerank()
            out["iters"] = self.last_iters
            return out
        torch = self.eng.torch
        main = torch.cuda.current_stream(self.eng.device)
        if self._side is None:
            self._side = torch.cuda.Stream(device=self.eng.device)
        side = self._side
        ready = main.record_event()  # the window's log text and offsets are on main
        out = {"scores": self.push_metrics(x_new)}
        st = self._rerank_begin()
        try:
            with torch.cuda.stream(side):
                side.wait_event(ready)
                logs = self.push_logs(log_text, doc_off, templates=templates, validate=validate, _defer=True)
        finally:
            # a log pass that raises (e.g. bad offsets) still leaves the re-rank completed, so the
            # next window warm-starts from this window's solve as the oracle chain does
            out["top"] = self._rerank_end(st)
            out["iters"] = self.last_iters
            main.wait_stream(side)
        tm = logs.get("templates", {})
        for v in list(logs.values()) + list(tm.values()):
            if isinstance(v, torch.Tensor):
                v.record_stream(main)  # allocated on side, read on main from here on
        if templates:
            self.eng.template_hist_finish(tm)  # synchronises main (after side)
        else:
            main.synchronize()
        out["logs"] = logs
        return out

    # -- 4. snapshots ----------------------------------------------------------------------------
    def _meta(self):
        return dict(version=SNAPSHOT_VERSION, shard=type(self.shard).__name__, N=self.N, M=self.M, H=self.H,
                    lo=self.lo, hi=self.hi, n_max=self.n_max, world=self.comm.world, rank=self.comm.rank,
                    cfg=self.cfg.as_dict(), tol=self.tol)

    def snapshot(self, path):
        """Write this rank's stream state to `path` (.npz; each rank its own file, e.g. a path with
        the rank in it): the rolling state of its pods, the ranks the next window warm-starts from,
        the step count and the configuration it was built with.  Taken between windows; restoring it
        into a StreamingRCA of the same mesh, partition and configuration continues the stream bit
        for bit (tests/test_stream_dist_cpu.py, tests/test_gpu_stream.py).  The reference persists
        investigations only (ref:utils/db_handler.py:13); this is the stream's own checkpoint."""
        meta = dict(self._meta(), t=self.t, solved=self.solved, last_iters=self.last_iters)
        arrays = self.shard.state_dict(self.M, self.H)
        blob = np.frombuffer(json.dumps(meta, sort_keys=True).encode(), np.uint8)
        with open(path, "wb") as f:
            np.savez(f, meta=blob, **arrays)

    def restore(self, path):
        """Load a snapshot written by :meth:`snapshot` (no pickles: allow_pickle=False).  Raises
        ValueError when it was taken on another mesh size, partition, horizon or configuration."""
        with np.load(path, allow_pickle=False) as z:
            meta = json.loads(bytes(z["meta"]).decode())
            arrays = {k: z[k] for k in z.files if k != "meta"}
        want = json.loads(json.dumps(self._meta(), sort_keys=True))
        diff = sorted(k for k in want if meta.get(k) != want[k])
        if diff:
            raise ValueError(f"snapshot {path} does not match this stream: {', '.join(diff)} differ")
        self.shard.load_state_dict(arrays, self.M, self.H)
        self.t, self.solved, self.last_iters = int(meta["t"]), bool(meta["solved"]), int(meta["last_iters"])


def window_bytes(P, M, delta):
    """Algorithmic HBM bytes of one krca_stream_score call: state 20 B per series
    read + written; per step 4 B new, 4 B old and 4 B ring write per series, 8 B exceedance word
    read + written; outputs 4*M + 9 B per pod."""
    S = P * M
    return S * (40 + 20 * delta) + P * (4 * M + 9)
