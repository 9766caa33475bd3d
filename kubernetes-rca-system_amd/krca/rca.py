"""The RCA hot path as one step: rolling z-scores -> seeded PageRank -> root-cause top-k.

This is the north-star path (BASELINE.json): for a pod mesh of N pods with M metrics x T steps
and a caller -> dependency graph, one step scores every pod (krca_rolling_score), seeds a
personalized PageRank with the anomalous pods (p_i ∝ max(score_i - seed_floor, 0)), propagates
for a fixed number of iterations (krca_ppr_shard_step: pull SpMV fused with the rank update),
and ranks pods by the mass they received from their callers times the part of their own anomaly
that no anomalous dependency explains (krca_rca_explain + krca_rca_key_explained +
krca_topk_i64; Config.key).

Multi-GPU: one process per GPU; rank g owns pods [g*n_max, (g+1)*n_max): its
slice of the metric tensor and its rows of the pull-CSR.  Scoring needs no communication.  Each
PageRank iteration ends with ONE all-gather over RCCL/xGMI of every rank's
[weight codes | partial-sum slots] slice (slice_words(n_max) int64: the n_max 32-bit weight codes,
then NSET sets of residual, dangling mass and seed total, NSPREAD slots each); the partial sums ride in the same payload and every rank reduces them
identically, so no extra collective or broadcast is needed.  Iterations are folded
(krca_ppr_shard_step_folded): each step first reduces the previous step's slot set itself, so an
iteration is one kernel and one exchange.  With one rank the exchange is a swap
of two buffers (the step kernel reads one and writes the other).  Arithmetic is integer fixed
point: the result is bit-identical for any G and to oracle/krca_oracle.c.  The final top-k merges G x k candidates.

A rank's PageRank rows need not be the pods it scores: :class:`SplitShard` (the bench's default at
G >= 4) scores a uniform range, all-gathers the scores once per step, and solves on an edge-balanced
:class:`Partition` range.

The per-rank numeric work is behind a small backend interface so the same orchestration runs
on the device (:class:`DeviceShard`, libkrca) and, in the CPU test-suite, on a NumPy restatement
with the gloo backend (tests/test_rca_dist_cpu.py).
"""
import ctypes
import math

import numpy as np

NSPREAD = 32
SET_WORDS = 3 * NSPREAD  # one slot set: residual | dangling | seed total, NSPREAD slots each
NSET = 3  # folded iterations rotate over 3 sets (read the previous step's, write, zero the next)
NSLOT = NSET * SET_WORDS  # == krca_ppr_nslot()


def wslots(n_max):
    """int64 offset of the partial-sum slots in a rank's exchange slice (after n_max uint32 codes)."""
    return (n_max + 1) // 2


def slice_words(n_max):
    """int64 words of one rank's exchange slice (== krca_ppr_slice_words)."""
    return wslots(n_max) + NSLOT


def remap_cols(col, n_max):
    """uint32 index of node j's weight code in w_all[G][slice] (csrc/ppr.hip remap_col)."""
    col = np.asarray(col, np.int64)
    return col + (col // n_max) * (2 * slice_words(n_max) - n_max)


def shard_range(N, world, rank):
    n_max = max(1, math.ceil(N / world))
    lo = min(N, rank * n_max)
    hi = min(N, lo + n_max)
    return lo, hi, n_max


# Partition.balanced: a rank may hold up to EDGE_SLACK x the mean in-edges per rank before its
# edges, not its pods, bound it.  1.5 is the measured best of a sweep of the G = 8 split step
# (1.25 / 1.5 / 2.0 / 3.0: DESIGN.md §5); bench.py's --ppr-edge-slack and StreamingRCA's
# partition="balanced" use this one value
EDGE_SLACK = 1.5


class Partition:
    """Contiguous pod ranges of G ranks: rank g owns pods [bounds[g], bounds[g+1]) -- their metric
    series, their rows of the pull-CSR -- and its exchange slice holds n_slot = max range weight
    codes.  A column j owned by rank g is addressed by its VIRTUAL id g * n_slot + (j - bounds[g]),
    so the device's remap (j + (j / n_max) * (2 * slice - n_max), csrc/ppr_layout.h) with n_max =
    n_slot lands every code in its owner's slice; for uniform ranges of n_slot pods the virtual id
    is the pod id itself.

    uniform(N, G): ranges of ceil(N / G) pods (shard_range).  balanced(row_ptr, G): ranges of at most
    t x N / G pods and t x EDGE_SLACK x E / G in-edges, t as small as covers the mesh.  The
    synthetic mesh wires services by preferential
    attachment, so the heavily called services sit at low pod ids: with uniform ranges rank 0 of 8
    holds 10.6M of the C4 mesh's 20M edges and its PageRank step takes 25 us against ~4 for the
    others (tools/ppr_g8_emulation.py, profiles/r4/ppr_g8_emulation.json), and every iteration's
    all-gather waits for it."""

    def __init__(self, bounds):
        b = np.asarray(bounds, np.int64)
        if b.ndim != 1 or len(b) < 2 or b[0] != 0 or np.any(np.diff(b) < 0):
            raise ValueError(f"partition bounds must rise from 0: {b[:8]}")
        self.bounds, self.world, self.N = b, len(b) - 1, int(b[-1])
        self.n_slot = max(1, int(np.max(np.diff(b))))

    @classmethod
    def uniform(cls, N, world):
        n_max = max(1, math.ceil(N / world))
        return cls([min(N, g * n_max) for g in range(world)] + [N])

    @classmethod
    def balanced(cls, row_ptr, world, edge_slack=EDGE_SLACK):
        """The smallest t for which G contiguous ranges of <= t * N / G pods and <= t * edge_slack *
        E / G in-edges each cover the mesh (bisection on t, greedy longest ranges), and those ranges."""
        rp = np.asarray(row_ptr, np.int64)
        N, E = len(rp) - 1, int(rp[-1])
        if world == 1 or N == 0:
            return cls([0] + [N] * world)
        pods_cap, edges_cap = N / world, edge_slack * max(E, 1) / world

        def cover(t):
            b, pos = [0], 0
            for _ in range(world):
                hi = min(N, pos + max(1, int(t * pods_cap)))
                # the longest range from pos whose in-edges stay within the cap (at least one pod)
                hi = max(pos + 1, min(hi, int(np.searchsorted(rp, rp[pos] + t * edges_cap, side="right")) - 1))
                pos = min(N, hi)
                b.append(pos)
            return b
        lo_t, hi_t = 1.0, float(world)
        for _ in range(50):
            mid = 0.5 * (lo_t + hi_t)
            if cover(mid)[-1] >= N:
                hi_t = mid
            else:
                lo_t = mid
        b = cover(hi_t)
        b[-1] = N
        return cls(b)

    def range(self, rank):
        """(lo, hi, n_slot) of `rank` (shard_range's triple)."""
        return int(self.bounds[rank]), int(self.bounds[rank + 1]), self.n_slot

    def owner(self, j):
        return np.clip(np.searchsorted(self.bounds, np.asarray(j, np.int64), side="right") - 1, 0, self.world - 1)

    def virtual(self, col):
        """Global pod ids -> the exchange layout's virtual ids (int32 when they fit)."""
        c = np.asarray(col, np.int64)
        g = self.owner(c)
        v = g * self.n_slot + (c - self.bounds[g])
        return v.astype(np.int32) if self.world * self.n_slot < 2 ** 31 else v

    def unpad(self, flat):
        """world * n_slot per-rank padded rows (gather order) -> the N rows in pod order."""
        a = np.asarray(flat)
        return np.concatenate([a[g * self.n_slot:g * self.n_slot + int(self.bounds[g + 1] - self.bounds[g])]
                               for g in range(self.world)])


def shard_graph(row_ptr, col, outdeg, lo, hi, part=None):
    """Rows [lo, hi) of a pull-CSR.  Column ids stay global, or become `part`'s virtual ids (the
    exchange layout of a Partition whose ranges are not all n_slot long)."""
    rp = np.asarray(row_ptr[lo:hi + 1], np.int64) - int(row_ptr[lo])
    c = np.asarray(col[int(row_ptr[lo]):int(row_ptr[hi])], np.int32)
    if part is not None:
        c = part.virtual(c)
    return rp, c, np.asarray(outdeg[lo:hi], np.int32)


def null_floor(n_series, minimum=4.0):
    """The seed floor of a mesh with n_series scored series: the expected maximum |z| of that many
    null (Gaussian) series, Phi^-1(1 - 1/(2 n)), at least `minimum`, rounded to 1e-3 so that every
    rank, the bench and the oracle chain get the same float (stdlib NormalDist: no scipy)."""
    from statistics import NormalDist
    if n_series <= 1:
        return float(minimum)
    return max(float(minimum), round(NormalDist().inv_cdf(1.0 - 1.0 / (2.0 * n_series)), 3))


class Config:
    """The one root-cause ranking definition ("Ranking"), shared by bench.py,
    :class:`RcaStep`, the streaming replay and ``Coordinator.ranked_root_causes``:

    * rolling z-scores over a trailing window of `window` steps, exceedance at |z| > z_threshold;
    * personalized PageRank (networkx 3.4.2 semantics) with damping `alpha` = 0.5 and
      personalization p_i ∝ max(s_i - floor, 0), s_i = the pod's max |z| at the last step.  The
      floor (|z| units) is `seed_floor` when given, else scale-aware: the expected maximum |z| of
      the mesh's P·M null series, at least `min_floor` = 4 (:func:`null_floor`; 4.0 up to ~16k
      series, 5.286 at the C4 mesh's 8M): a fixed floor lets the noise maxima of a large mesh
      (|z| ≈ 6 over 8M series) seed the walk (measured: DESIGN.md §3.2);
    * networkx's L1 stop rule: iterate until sum |r - r_prev| < N * `tol` (tol = 1e-10), at most
      `iters` = 30 iterations (a mesh too small for the weight codes to reach the tolerance -- N
      below ~100 -- runs all 30, which at alpha = 0.5 is within 1e-9 of the converged vector).  At
      C4 the rule stops after 11 iterations, 1.6e-5 of the mass from the 30-iteration vector, top-10
      identical on both failure models; tol = 0 runs exactly `iters` (the rounds
      2-4 definition, pinned to networkx 3.4.2 at 2k / 20k nodes: tests/golden/ppr_nx_meshes.npz).
      :class:`RcaStep` issues the previous solve's count + 1 steps without a host poll and checks
      the count when the step's candidates are settled;
    * pods ranked by `key`, top `k`, ties -> lower index:
      "explained" (default): (recv_i + t_i / 32) * u_i -- recv_i the mass pod i received from its
      callers in the last iteration, t_i its own teleport share (r_i = recv_i + t_i), u_i =
      max(q_i - d_i, 0) the part of its own anomaly q_i that no explaining dependency accounts for
      (d_i: the largest anomaly among its anomalous dependencies k that collect at least as many
      anomalous callers besides i, or are at least twice as anomalous, and whose other anomalous
      callers look like i -- i at most 3x their mean; krca_rca_explain).  Symptoms show up upstream
      of a fault (callers -> dependency): a root is anomalous, its callers' mass converges on it, and
      nothing below it explains it.  Recall of the planted roots: C2 1.00 / 0.90
      (default / spread failure model, CPU oracle, 3 seeds), 10k-40k default meshes 1.00, C4 on the
      GPU in profiles/r5;
      "rq": r_i * q_i (propagated mass times own anomaly; rounds 2-4): 1.00 on the default model,
      0.17 / 0.00 at C2 / C4 when the callers carry the larger symptoms."""

    KEYS = ("explained", "rq")

    def __init__(self, window=60, z_threshold=3.0, seed_floor=None, alpha=0.5, iters=30, tol=1e-10, k=10,
                 min_floor=4.0, key="explained"):
        if key not in self.KEYS:
            raise ValueError(f"ranking key {key!r}: one of {self.KEYS}")
        self.window = window
        self.z_threshold = z_threshold
        self.seed_floor = seed_floor
        self.alpha = alpha
        self.iters = iters
        self.tol = tol
        self.k = k
        self.min_floor = min_floor
        self.key = key

    def floor(self, n_pods, n_metrics=1):
        """The seed floor for a mesh of n_pods pods scored over n_metrics metrics each."""
        if self.seed_floor is not None:
            return float(self.seed_floor)
        return null_floor(int(n_pods) * int(n_metrics), self.min_floor)

    def as_dict(self):
        return dict(window=self.window, z_threshold=self.z_threshold, seed_floor=self.seed_floor, alpha=self.alpha,
                    iters=self.iters, tol=self.tol, k=self.k, min_floor=self.min_floor, key=self.key)

    def replace(self, **kw):
        d = self.as_dict()
        d.update(kw)
        return Config(**d)


RANKING = Config()


def step_flags(tol, last):
    """krca_ppr_shard_step flags: under a tolerance every iteration needs the residual and the
    stored ranks; a fixed-iteration solve stores the ranks on its last iteration only."""
    return 3 if tol > 0 else (2 if last else 0)


class Comm:
    """All-gather over torch.distributed (nccl == RCCL on ROCm; gloo in CPU tests).

    collective=True runs the collectives even with one rank (a world-size-1 process group: on a
    one-GPU box this is how the RCCL call sites -- the per-iteration all-gather, the candidate
    merge -- execute on the hardware; tests/test_gpu_rccl.py).  Its shards then use the G > 1 slot
    protocol (DeviceShard(pingpong=False)): the exchange copies send into w_all instead of swapping."""

    def __init__(self, world=1, rank=0, group=None, collective=False):
        self.world, self.rank, self.group = world, rank, group
        self.collective = bool(collective) or world > 1
        self._gloo = None  # the backend, looked up once
        self._direct = None  # RCCL: (process group, options) for the per-iteration all-gather

    def exchange(self, shard):
        """Make every rank's send slice visible in shard.w_all (G = 1: swap the ping-pong pair)."""
        if not self.collective:
            shard.send, shard.w_all = shard.w_all, shard.send
            return
        if self._direct is None:
            self._direct = self._direct_gather()
        if self._direct:
            # the PageRank exchange runs 30 times per solve: the process group's all-gather called
            # directly skips the public wrapper's per-call checks and option building (host time
            # that, at 8 ranks, is of the order of the ~20 us step itself).  A first
            # call that raises (an API this torch does not have) falls back to the public wrapper
            # for good; later failures propagate.
            pg, opts = self._direct
            try:
                work = pg._allgather_base(shard.w_all, shard.send, opts)
                if work is not None:  # asyncOp = False: the group may return no work (already on our stream)
                    work.wait()
                self.direct_calls += 1
                return
            except (AttributeError, TypeError, RuntimeError):
                if self.direct_calls:
                    raise
                self._direct = False
        self.all_gather(shard.w_all, shard.send)

    direct_calls = 0  # exchanges that took the direct entry point (tests)

    def _direct_gather(self):
        """(group, AllgatherOptions) when the backend is RCCL / NCCL and the group has the direct
        entry point, else False (gloo: the list form of all_gather_flat).  AllgatherOptions lives
        in torch.distributed.distributed_c10d (torch 2.10 does not re-export it from
        torch.distributed: ADVICE r4).

        asyncOp = False, as the public all_gather_into_tensor(async_op=False) sets it: the collective
        is enqueued on the caller's stream.  The options' default (True) runs it on the process
        group's internal stream behind an event fork and join; captured into a HIP graph that way,
        the solve replayed correctly once and then diverged (R5j: the second replay's keys differed
        from the eager solve's; tests/test_gpu_rccl.py)."""
        import torch.distributed as dist
        if dist.get_backend(self.group) == "gloo":
            return False
        pg = self.group if self.group is not None else dist.distributed_c10d._get_default_group()
        opts_t = getattr(dist.distributed_c10d, "AllgatherOptions", None)
        if opts_t is None or not hasattr(pg, "_allgather_base"):
            return False
        opts = opts_t()
        if hasattr(opts, "asyncOp"):
            opts.asyncOp = False
        return pg, opts

    def all_gather(self, out, inp):
        if not self.collective:
            if out.data_ptr() != inp.data_ptr():
                out.copy_(inp)
            return
        if self._gloo is None:
            import torch.distributed as dist
            self._gloo = dist.get_backend(self.group) == "gloo"
        all_gather_flat(out, inp, self.world, self.group, self._gloo)


def _collective_dtypes():
    import torch
    return (torch.uint8, torch.int8, torch.int32, torch.int64, torch.float32, torch.float64)


def all_gather_flat(out, inp, world, group=None, gloo=None):
    """out[world * inp.numel()] <- every rank's inp.  RCCL ("nccl") gathers into the flat tensor
    directly; gloo has no all_gather_into_tensor, so it takes the list form.  Chosen once from the
    backend, so a real RCCL failure (timeout, size mismatch) propagates instead of being retried."""
    import torch
    import torch.distributed as dist
    if gloo is None:
        gloo = dist.get_backend(group) == "gloo"
    if out.dtype not in _collective_dtypes():
        # a gather only moves bytes: dtypes the backends lack (RCCL / NCCL have no int16, gloo
        # refuses it: the correlation's fp16 rows travel as int16) go as uint8 views
        out, inp = out.view(torch.uint8), inp.view(torch.uint8)
    if gloo:
        dist.all_gather(list(out.view(world, -1).unbind(0)), inp, group=group)
    else:
        dist.all_gather_into_tensor(out, inp, group=group)


class DeviceShard:
    """Per-rank device state (libkrca kernels on torch's current stream)."""

    def __init__(self, engine, x_local, row_ptr_local, col_local, outdeg_local, N, n_max, world, cfg, pingpong=None):
        """pingpong (default: world == 1): the G = 1 exchange is a swap of two buffers; False with a
        one-rank collective Comm (the exchange copies send into w_all, the G > 1 slot protocol)."""
        import torch
        self.torch, self.eng, self.cfg = torch, engine, cfg
        lib = engine.lib
        dev = engine.device
        self.N, self.n_max, self.world = N, n_max, world
        self.pingpong = (world == 1) if pingpong is None else bool(pingpong)
        if self.pingpong and world != 1:
            raise ValueError("DeviceShard: the ping-pong exchange needs one rank")
        self.host_csr = (row_ptr_local, col_local)  # the whole graph when n == N (Explain's default)
        self.x = x_local
        self.M = int(x_local.shape[2]) if x_local is not None and x_local.dim() == 3 else 1  # metrics per pod
        self.n = int(outdeg_local.shape[0])
        # plan + packed columns (remapped to the exchange layout, dictionary blocks where they pay)
        self.plan, self.plan_len, self.col, self.lane, self.n_dict = (
            engine.ppr_pack(row_ptr_local, col_local, n_max, n_total=max(N, world * n_max)) if self.n
            else (None, 0, None, None, 0))
        self.row_ptr = torch.from_numpy(np.ascontiguousarray(row_ptr_local)).to(dev)
        self.outdeg = torch.from_numpy(np.ascontiguousarray(outdeg_local)).to(dev)
        i64 = dict(dtype=torch.int64, device=dev)
        self.q = torch.zeros(max(self.n, 1), **i64)
        self.r = torch.zeros(max(self.n, 1), **i64)
        self.key = torch.zeros(max(self.n, 1), **i64)
        self.d = torch.zeros(max(self.n, 1), **i64)  # krca_rca_explain's output for these rows
        self.send = torch.zeros(slice_words(n_max), **i64)
        # G = 1: ping-pong pair (the step reads w_all, writes send; the exchange swaps them)
        self.w_all = torch.zeros((1 if world == 1 else world) * slice_words(n_max), **i64)
        self.ctl = torch.zeros(lib.krca_ppr_ctl_size(self.n), dtype=torch.uint8, device=dev)
        self.score_out = None
        # one device: krca_ppr_solo_step launches the step and its reduction (in the step's last
        # workgroup under KRCA_PPR_FUSE); reduce(first=0) is then a no-op.  Its tolerance is the one
        # of the solve's first reduce(first=1).
        self.fused = self.pingpong and n_max == N
        self._tol = 0.0
        # ctypes argument tuples of the per-iteration calls, keyed by the buffers / scalars / stream
        # they bind (at 8 ranks a step is ~5 us of GPU work: rebuilding ~17 ctypes objects per
        # call was host time on the critical path)
        self._argc = {}

    def _cached(self, key, build):
        a = self._argc.get(key)
        if a is None:
            a = self._argc[key] = build()
        return a

    def _chk(self, rc, what):
        from .native import _check
        _check(rc, what, self.eng.lib)

    # -- streaming (krca/stream.py): rolling state of this rank's pods, warm-started ranks ------
    def stream_score(self, x_new, t0, horizon):
        """x_new float32 [delta, n_local, M] (device, time-major): carry the rank's rolling state
        forward by delta steps (krca_stream_score); outputs as the batch scorer over the series so far."""
        torch, e, p = self.torch, self.eng, self.eng.ptr
        d, P, M = x_new.shape
        self.M = int(M)
        if P != self.n:
            raise ValueError(f"stream window has {P} pods, the shard owns {self.n}")
        self._ensure_stream(int(M), horizon)
        o = self.score_out
        self._chk(e.lib.krca_stream_score(p(x_new), P, M, int(d), int(t0), self.cfg.window, int(horizon),
                                          float(self.cfg.z_threshold), p(self._stream_state), p(o["z_last"]), p(o["score"]),
                                          p(o["n_exceed"]), p(o["flags"]), e._stream()), "krca_stream_score")
        return o

    def _ensure_stream(self, M, horizon):
        """The rolling state (krca_stream_state_size bytes) and the score outputs, allocated once."""
        torch, e = self.torch, self.eng
        if getattr(self, "_stream_state", None) is not None:
            return
        P, dev = self.n, e.device
        nbytes = e.lib.krca_stream_state_size(P, M, self.cfg.window, horizon)
        self._stream_state = torch.zeros(max(int(nbytes), 1), dtype=torch.uint8, device=dev)
        self.score_out = dict(z_last=torch.empty((max(P, 1), M), dtype=torch.float32, device=dev),
                              score=torch.empty(max(P, 1), dtype=torch.float32, device=dev),
                              n_exceed=torch.empty(max(P, 1), dtype=torch.int32, device=dev),
                              flags=torch.empty(max(P, 1), dtype=torch.uint8, device=dev))

    # -- snapshots of the stream (krca.stream.StreamingRCA.snapshot / restore) --------------------
    def state_dict(self, M, horizon):
        """The rank's stream state as host arrays: the rolling state bytes (plain data:
        krca_stream_state_size's float64 sums, sample ring and exceedance bits, no pointers) and the
        ranks of the last solve (the next window's warm start)."""
        self.M = int(M)
        self._ensure_stream(self.M, horizon)
        return dict(stream_state=self._stream_state.cpu().numpy(), r=self.r[:self.n].cpu().numpy())

    def load_state_dict(self, st, M, horizon):
        torch = self.torch
        self.M = int(M)
        self._ensure_stream(self.M, horizon)
        ss, r = np.asarray(st["stream_state"], np.uint8), np.asarray(st["r"], np.int64)
        if ss.shape != tuple(self._stream_state.shape) or r.shape != (self.n,):
            raise ValueError(f"snapshot state {ss.shape} / ranks {r.shape} do not fit this shard "
                             f"({tuple(self._stream_state.shape)} / ({self.n},))")
        self._stream_state.copy_(torch.from_numpy(ss))
        self.r[:self.n].copy_(torch.from_numpy(r))

    def init_warm(self, alpha, seed_floor):
        """Re-seed from the current scores, start from the ranks of the previous solve."""
        e, p = self.eng, self.eng.ptr
        self._zero_slots()
        self._chk(e.lib.krca_ppr_shard_init_warm(p(self.score_out["score"]), float(seed_floor), p(self.outdeg), self.n,
                                                 self.n_max, self.N, float(alpha), p(self.ctl), p(self.q), p(self.r),
                                                 p(self.send), e._stream()), "krca_ppr_shard_init_warm")

    def ctl_async(self):
        """Enqueue a copy of (iteration at convergence, iterations done) into pinned host memory and
        an event behind it; ctl_wait(handle) reads it.  Two slots: one poll in flight while the
        caller enqueues the next iterations."""
        torch, e, p = self.torch, self.eng, self.eng.ptr
        if getattr(self, "_poll", None) is None:
            self._poll = [torch.zeros(2, dtype=torch.int32, pin_memory=True) for _ in range(2)]
            self._poll_ev = [torch.cuda.Event() for _ in range(2)]
            self._poll_i = 0
        i = self._poll_i
        self._poll_i ^= 1
        self._chk(e.lib.krca_ppr_ctl_copy(p(self.ctl), self._poll[i].data_ptr(), e._stream()), "krca_ppr_ctl_copy")
        self._poll_ev[i].record(torch.cuda.current_stream(e.device))
        return i

    def ctl_wait(self, handle):
        self._poll_ev[handle].synchronize()
        conv, it = (int(v) for v in self._poll[handle].tolist())
        return (conv or it), bool(conv)

    def ctl_read(self):
        """(iterations done, converged) of the solve in flight (synchronises the stream)."""
        import ctypes
        e, p = self.eng, self.eng.ptr
        it, conv = ctypes.c_int32(0), ctypes.c_int32(0)
        self._chk(e.lib.krca_ppr_ctl_read(p(self.ctl), ctypes.byref(it), ctypes.byref(conv), e._stream()),
                  "krca_ppr_ctl_read")
        return int(it.value), bool(conv.value)

    def score(self):
        self.score_out = self.eng.rolling_score_device(self.x, self.cfg.window, self.cfg.z_threshold, self.score_out)
        return self.score_out

    def _zero_slots(self):
        """Partial-sum slots zeroed before an init adds into send's set 0 (and, with the ping-pong
        exchange, the other buffer's, which the first folded step writes)."""
        e, p = self.eng, self.eng.ptr
        wsl = wslots(self.n_max)
        # by a libkrca kernel, not torch's zero_ (a memset node in a captured solve)
        for buf in (self.send, self.w_all) if self.pingpong else (self.send,):
            tail = buf[wsl:]
            self._chk(e.lib.krca_fill_i64(p(tail), tail.numel(), 0, e._stream()), "krca_fill_i64")

    def init(self, alpha, seed_floor):
        e, p = self.eng, self.eng.ptr
        self._zero_slots()
        self._chk(e.lib.krca_ppr_shard_init(p(self.score_out["score"]), float(seed_floor), p(self.outdeg), self.n,
                                            self.n_max, self.N, float(alpha), p(self.ctl), p(self.q), p(self.r),
                                            p(self.send), e._stream()), "krca_ppr_shard_init")

    def step(self, alpha, flags=3):
        """flags: krca_ppr_shard_step's KRCA_PPR_RESIDUAL (1) | KRCA_PPR_WRITE_R (2)."""
        e, p = self.eng, self.eng.ptr
        if not self.plan_len:
            return
        st = e._stream()
        key = ("step", self.w_all.data_ptr(), self.send.data_ptr(), float(alpha), int(flags), float(self._tol), st.value)
        if self.fused:
            args = self._cached(key, lambda: (p(self.row_ptr), p(self.col), p(self.plan), self.plan_len, p(self.lane),
                                              p(self.w_all), p(self.outdeg), p(self.q), self.N, float(alpha), int(flags),
                                              float(self._tol), p(self.r), p(self.send), p(self.ctl), st))
            self._chk(e.lib.krca_ppr_solo_step(*args), "krca_ppr_solo_step")
        else:
            args = self._cached(key, lambda: (p(self.row_ptr), p(self.col), p(self.plan), self.plan_len, p(self.lane),
                                              p(self.w_all), p(self.outdeg), p(self.q), self.n, self.n_max, self.N,
                                              float(alpha), int(flags), p(self.r), p(self.send), p(self.ctl), st))
            self._chk(e.lib.krca_ppr_shard_step(*args), "krca_ppr_shard_step")

    def step_folded(self, alpha, tol, it, flags):
        """Folded iteration `it` (1-based): the reduction of step it - 1 and the step, one kernel."""
        e, p = self.eng, self.eng.ptr
        st = e._stream()
        nxt = self.w_all if self.pingpong else self.send
        if not self.plan_len:
            # a rank that owns no pods still runs the step's reduction (krca_ppr_shard_step_folded
            # launches it alone for an empty plan): its iteration count and convergence flag must
            # advance with the other ranks', or its convergence poll never stops and the
            # collectives mismatch
            null = ctypes.c_void_p(0)
            self._chk(e.lib.krca_ppr_shard_step_folded(null, null, null, 0, null, p(self.w_all), self.world, null, null,
                                                       0, self.n_max, self.N, float(alpha), float(tol), int(it),
                                                       int(flags), null, p(self.send), p(nxt), p(self.ctl), st),
                      "krca_ppr_shard_step_folded")
            return
        key = ("fold", self.w_all.data_ptr(), self.send.data_ptr(), float(alpha), float(tol), int(it), int(flags), st.value)
        args = self._cached(key, lambda: (p(self.row_ptr), p(self.col), p(self.plan), self.plan_len, p(self.lane),
                                          p(self.w_all), self.world, p(self.outdeg), p(self.q), self.n, self.n_max, self.N,
                                          float(alpha), float(tol), int(it), int(flags), p(self.r), p(self.send), p(nxt),
                                          p(self.ctl), st))
        self._chk(e.lib.krca_ppr_shard_step_folded(*args), "krca_ppr_shard_step_folded")

    def finish(self, alpha, tol, it):
        """The reduction of the last folded step (iteration count, convergence)."""
        e, p = self.eng, self.eng.ptr
        self._chk(e.lib.krca_ppr_shard_finish(p(self.w_all), self.world, self.n_max, self.N, float(alpha), float(tol),
                                              int(it), p(self.ctl), e._stream()), "krca_ppr_shard_finish")

    def reduce(self, alpha, tol, first):
        e, p = self.eng, self.eng.ptr
        if first:
            self._tol = float(tol)
        elif self.fused and self.plan_len:
            return  # launched by krca_ppr_solo_step
        st = e._stream()
        key = ("reduce", self.w_all.data_ptr(), self.send.data_ptr(), float(alpha), float(tol), int(first), st.value)
        args = self._cached(key, lambda: (p(self.w_all), self.world, self.n_max, self.N, float(alpha), float(tol),
                                          int(first), p(self.ctl), p(self.send), st))
        self._chk(e.lib.krca_ppr_shard_reduce(*args), "krca_ppr_shard_reduce")

    def local_topk(self, k):
        """Top-k of the key r_i * q_i (Config key "rq")."""
        e, p = self.eng, self.eng.ptr
        if self.n == 0:
            return np.zeros(0, np.int64), np.zeros(0, np.int64)
        self._chk(e.lib.krca_ppr_rca_key(p(self.r), p(self.q), self.n, p(self.key), e._stream()), "krca_ppr_rca_key")
        idx, val = e.topk_device(self.key[:self.n], min(k, self.n))
        return idx, val

    def local_topk_explained(self, k, score_all, floor, graph, lo):
        """Top-k of the default key (Config key "explained") over this shard's rows, global pods
        [lo, lo + n): krca_rca_explain over the whole graph (an :class:`Explain`) and every pod's
        scores, then krca_rca_key_explained from the finished solve's ranks and ctl."""
        e, p = self.eng, self.eng.ptr
        if self.n == 0:
            return np.zeros(0, np.int64), np.zeros(0, np.int64)
        rp, col = graph.device(e)
        e.rca_explain_device(score_all, floor, rp, col, lo, lo + self.n, out=self.d)
        self._chk(e.lib.krca_rca_key_explained(p(self.r), p(self.q), p(self.d), self.n, self.N, p(self.ctl), p(self.key),
                                               e._stream()), "krca_rca_key_explained")
        idx, val = e.topk_device(self.key[:self.n], min(k, self.n))
        return idx, val


class SplitShard:
    """A rank whose PageRank rows are not its scored pods (bench.py at G >= 4).

    The scoring runs on `scorer` over the rank's range of `spart` (uniform: every rank streams the
    same number of series), ONE all-gather per step moves the scores (4 B per pod, every rank's
    padded slice: pod order, since the ranges are uniform), and the PageRank solve runs on `ppr`
    over the rank's range of `ppart` (Partition.balanced: the hub services' in-edges spread over
    the ranks), seeded from its rows' slice of the gathered scores.  The solve is the same
    pod-sharded one (one all-gather per iteration), so the ranks stay bit-identical to the oracle.
    With a one-range `ppart` (``Partition([0, N])``) the solve is REPLICATED: every rank runs the
    whole mesh's PageRank on the gathered scores with no collective inside the solve (its RcaStep
    takes ``Comm(1, 0)``) and reaches the same top-k on its own -- the measured alternative when the
    per-iteration all-gather costs more than the solve it shards.
    Everything :class:`RcaStep` and :class:`Comm` use besides score() -- init, folded steps, send /
    w_all, top-k, r -- is the PageRank shard's; score_out is the scorer's."""

    def __init__(self, scorer, ppr, spart, ppart, rank, comm):
        import torch
        if (spart.world < 2 and not comm.collective) or ppart.world not in (1, spart.world) or spart.N != ppart.N:
            raise ValueError("SplitShard: two partitions of the same pods over the same G > 1 ranks "
                             "(or one range: the replicated solve; one rank only with a collective Comm)")
        if not np.array_equal(spart.bounds, Partition.uniform(spart.N, spart.world).bounds):
            raise ValueError("SplitShard: the scoring partition must be uniform (its gathered slices are then in pod order)")
        self.scorer, self.ppr, self.comm, self.rank = scorer, ppr, comm, rank
        self.spart, self.ppart = spart, ppart
        lo, hi, s_slot = spart.range(rank)
        self.n_score = hi - lo
        plo, phi, _ = ppart.range(rank if ppart.world > 1 else 0)
        dev = ppr.send.device
        self._pad = torch.zeros(s_slot, dtype=torch.float32, device=dev)
        self._all = torch.zeros(spart.world * s_slot + 1, dtype=torch.float32, device=dev)
        view = self._all[plo:plo + max(phi - plo, 1)]
        ppr.score_out = {"score": view.numpy() if dev.type == "cpu" else view}

    def __getattr__(self, name):  # only reached for names the wrapper does not define
        if name in ("scorer", "ppr"):
            raise AttributeError(name)
        return getattr(self.ppr, name)

    # the exchange buffers are the PageRank shard's, assignments included (a one-rank solve's
    # exchange swaps them: Comm.exchange at world 1)
    @property
    def send(self):
        return self.ppr.send

    @send.setter
    def send(self, v):
        self.ppr.send = v

    @property
    def w_all(self):
        return self.ppr.w_all

    @w_all.setter
    def w_all(self, v):
        self.ppr.w_all = v

    @property
    def M(self):
        return self.scorer.M

    @property
    def score_out(self):
        return getattr(self.scorer, "score_out", None)

    def score(self):
        """The rank's scoring, then the all-gather of every rank's scores."""
        out = self.score_local()
        self.exchange_scores()
        return out

    def score_local(self):
        """The rank's scoring alone (a pipelined caller orders the next step's scoring after this,
        not after the exchange)."""
        return self.scorer.score()

    def scores_all(self):
        """The scores of every pod in pod order (the gathered vector; the uniform ranges put the
        padding at the end)."""
        return self._all[:self.spart.N]

    def exchange_scores(self):
        """Every rank's scores into the PageRank shard's seed vector (one all-gather)."""
        import torch
        s, n = self.scorer.score_out["score"], self.n_score
        if isinstance(s, np.ndarray):
            self._pad[:n] = torch.from_numpy(np.ascontiguousarray(s[:n], np.float32))
        else:
            self._pad[:n].copy_(s[:n])
        self.comm.all_gather(self._all[:-1], self._pad)


class Explain:
    """The whole pull-CSR (global pod ids) that krca_rca_explain walks for the default ranking key:
    host arrays, uploaded once per device on first use and shared by every RcaStep of a process (the
    bench's two pipeline slots)."""

    def __init__(self, row_ptr, col):
        self.row_ptr = np.ascontiguousarray(row_ptr, np.int64)
        self.col = np.ascontiguousarray(col, np.int32)
        self.N = len(self.row_ptr) - 1
        if len(self.col) != int(self.row_ptr[-1]) or (len(self.col) and (int(self.col.min()) < 0 or
                                                                          int(self.col.max()) >= self.N)):
            raise ValueError("Explain: a pull-CSR with columns in [0, N) and row_ptr[N] == len(col)")
        self._dev = {}

    def device(self, engine):
        key = str(engine.device)
        if key not in self._dev:
            self._dev[key] = (engine._dev(self.row_ptr), engine._dev(self.col))
        return self._dev[key]


def graph_default(comm, cfg, shard=None):
    """Whether RcaStep captures its PageRank solve in a HIP graph: only with KRCA_RCA_GRAPH=1, for a
    device shard.  Measured at C4 on one MI355X (`profiles/r3/bench_graph_ab.txt`): the replayed
    graph ran the step 0.26 ms and the one-step latency 0.2 ms SLOWER than the eager launches -- the
    ~13 us per iteration between the step kernels is the GPU's dependent-kernel boundary, not host
    time -- so eager is the default."""
    import os
    if os.environ.get("KRCA_RCA_GRAPH") != "1" or not isinstance(shard, DeviceShard):
        return False
    return True


class RcaStep:
    """One rank's view of the pod-sharded RCA step.

    With `graph` (default: :func:`graph_default`, off) the PageRank solve of n folded steps (init,
    exchange, n x (step, exchange), the last reduction) is captured into a HIP graph on the shard's
    fixed buffers, once per n, and replayed: one launch instead of ~2 host calls per iteration.
    Under the stop rule n is plan_iters() (the previous count + 1: two graphs in practice, the cap's
    for the first solve and the converged count's); the poll of the count and settle()'s rare
    continuation stay eager.  Replays compute exactly the eager sequence: the captured kernels and
    pointers are the same, and G = 1's ping-pong roles after a replay are set to those the captured
    sequence ends with."""

    def __init__(self, shard, comm, cfg, offset, graph=None, explain=None, part=None):
        """explain: the whole pull-CSR (an :class:`Explain` or (row_ptr, col)) for the default key;
        optional when one rank holds the whole graph (its own rows are it).  part: the Partition
        whose padded slices a coupled G > 1 shard's scores are gathered in (default uniform)."""
        self.s, self.comm, self.cfg, self.offset = shard, comm, cfg, offset
        self.graph = graph_default(comm, cfg, shard) if graph is None else bool(graph)
        self._graphs = {}  # n -> (captured graph, the exchange buffers' roles after it)
        if explain is not None and not isinstance(explain, Explain):
            explain = Explain(*explain)
        self.explain = explain
        self.part = part
        self._sall = None
        self.last_iters = 0  # iterations of the last solve (negative: the cap without convergence)
        self._spec = None    # under a tolerance: (steps issued, ctl poll handle) of the solve in flight

    def plan_iters(self):
        """Folded steps the next solve issues: cfg.iters for a fixed-iteration solve; under a
        tolerance the previous solve's count + 1 (the last step finds the count's convergence and
        does nothing), cfg.iters before any history or after a solve that hit the cap."""
        cfg = self.cfg
        if cfg.tol > 0 and self.last_iters > 0:
            return min(self.last_iters + 1, cfg.iters)
        return cfg.iters

    def propagate(self):
        """Seeded PageRank on the current scores: init, exchange, then n x (folded step, exchange)
        and the last step's reduction; under the stop rule n = plan_iters() and a poll of the
        iteration count is enqueued behind them (read by settle())."""
        s, cfg = self.s, self.cfg
        n = self.plan_iters()
        if not self.graph:
            self._solve(n)
        else:
            self._replay(n)
        if cfg.tol > 0:
            self._spec = (n, s.ctl_async())

    def _replay(self, n):
        import gc

        import torch
        s = self.s
        if n not in self._graphs:
            self._solve(n)  # eager warm-up: statics, occupancy queries, workspaces
            g = torch.cuda.CUDAGraph()
            cur = torch.cuda.current_stream(s.eng.device)
            side = torch.cuda.Stream(s.eng.device)
            side.wait_stream(cur)
            # no garbage collection inside the capture: a collected cycle that holds device objects
            # (another graph, events, a communicator's work) would release them mid-capture, which
            # the runtime aborts on (torch.cuda.graph collects once before it begins)
            was = gc.isenabled()
            gc.disable()
            try:
                with torch.cuda.graph(g, stream=side):
                    self._solve(n)
            finally:
                if was:
                    gc.enable()
            cur.wait_stream(side)
            self._graphs[n] = (g, (s.send, s.w_all))
        g, roles = self._graphs[n]
        g.replay()
        s.send, s.w_all = roles

    def _solve(self, n):
        """init, exchange, then n x (folded step, exchange) and the last step's reduction: the same
        results as init / reduce(first) / n x (step, exchange, reduce), one kernel fewer per
        iteration (krca_ppr_shard_step_folded).  Under the stop rule steps past convergence exit on
        the device-held flag, so n may overshoot with no host poll."""
        s, c, cfg = self.s, self.comm, self.cfg
        s.init(cfg.alpha, cfg.floor(s.N, s.M))
        c.exchange(s)
        for it in range(1, n + 1):
            s.step_folded(cfg.alpha, cfg.tol, it, step_flags(cfg.tol, it == n))
            c.exchange(s)
        s.finish(cfg.alpha, cfg.tol, n)

    def settle(self, idx, val):
        """After propagate() + local_candidates() under a tolerance: read the solve's count; if the
        planned steps fell short of convergence (the scores moved), continue in polled batches of 4
        to convergence or the cap and recompute the candidates.  Every rank takes the same branch
        (the counts come from the same gathered slots).  Returns the (possibly new) candidates."""
        if self._spec is None:
            return idx, val
        s, c, cfg = self.s, self.comm, self.cfg
        n, h = self._spec
        self._spec = None
        iters, conv = s.ctl_wait(h)
        if not conv and n < cfg.iters:
            it, pending = n, None
            while it < cfg.iters:
                for _ in range(min(4, cfg.iters - it)):
                    it += 1
                    s.step_folded(cfg.alpha, cfg.tol, it, step_flags(cfg.tol, False))
                    c.exchange(s)
                if pending is not None and s.ctl_wait(pending)[1]:
                    break
                pending = s.ctl_async() if it < cfg.iters else None
            s.finish(cfg.alpha, cfg.tol, it)
            h = s.ctl_async()
            idx, val = self.local_candidates()
            iters, conv = s.ctl_wait(h)
        self.last_iters = iters if conv else -iters
        return idx, val

    def run(self, to_host=True, score_events=None):
        """One RCA step; score_events = (start, end) HIP events recorded around the scoring kernel."""
        if score_events is not None:
            score_events[0].record()
        self.s.score()
        if score_events is not None:
            score_events[1].record()
        self.propagate()
        idx, val = self.settle(*self.local_candidates())
        return self.merge(idx, val) if to_host else (idx, val)

    def local_candidates(self):
        """This rank's top-k (local index, key) under cfg.key, after propagate(): "rq" from the
        ranks alone; "explained" also needs every pod's scores (gathered at G > 1 unless the shard
        already holds them) and the whole graph."""
        s, cfg = self.s, self.cfg
        if cfg.key == "rq":
            return s.local_topk(cfg.k)
        ex = self.explain
        if ex is None:
            if self.comm.world != 1 or s.n != s.N:
                raise ValueError("RcaStep: the 'explained' key needs the whole graph (explain=...) at G > 1")
            ex = self.explain = Explain(*s.host_csr)
        return s.local_topk_explained(cfg.k, self.scores_all(), cfg.floor(s.N, s.M), ex, self.offset)

    def scores_all(self):
        """Every pod's score in pod order: the shard's own at G = 1, the gathered vector of a
        SplitShard, else one all-gather of the ranks' padded slices."""
        s = self.s
        if hasattr(s, "scores_all"):
            return s.scores_all()
        sc = s.score_out["score"]
        if self.comm.world == 1:
            return sc[:s.N]
        import torch
        part = self.part or Partition.uniform(s.N, self.comm.world)
        lo, hi, n_slot = part.range(self.comm.rank)
        host = isinstance(sc, np.ndarray)
        t = torch.from_numpy(np.ascontiguousarray(sc, np.float32)) if host else sc
        if self._sall is None:
            self._sall = (torch.zeros(n_slot, dtype=torch.float32, device=t.device),
                          torch.zeros(self.comm.world * n_slot, dtype=torch.float32, device=t.device))
        pad, out = self._sall
        pad[:hi - lo].copy_(t[:hi - lo])
        self.comm.all_gather(out, pad)
        if np.array_equal(part.bounds, Partition.uniform(s.N, self.comm.world).bounds):
            res = out[:s.N]
        else:
            res = torch.from_numpy(part.unpad(out.cpu().numpy())).to(t.device)
        return res.numpy() if host else res

    def merge(self, idx, val):
        """Gather G x k (global index, key) candidates; identical top-k on every rank."""
        import torch
        k = self.cfg.k
        if not isinstance(idx, torch.Tensor):
            idx = torch.from_numpy(np.asarray(idx, np.int64))
            val = torch.from_numpy(np.asarray(val, np.int64))
        kk = int(idx.numel())
        if not self.comm.collective:  # nothing to gather: one copy of (idx | val) to the host
            a = torch.cat((idx.to(torch.int64), val.to(torch.int64))).cpu().numpy()
            gi, gv = a[:kk] + self.offset, a[kk:]
            ok = a[:kk] >= 0
            gi, gv = gi[ok], gv[ok]
            order = sorted(range(len(gi)), key=lambda j: (-int(gv[j]), int(gi[j])))
            return gi[order[:k]], gv[order[:k]]
        cand = torch.full((2, k), -1, dtype=torch.int64, device=idx.device)
        cand[0, :kk] = idx.to(torch.int64) + self.offset
        cand[1, :kk] = val.to(torch.int64)
        cand[1, kk:] = torch.iinfo(torch.int64).min
        allc = torch.empty((self.comm.world, 2, k), dtype=torch.int64, device=idx.device)
        self.comm.all_gather(allc.view(-1), cand.view(-1))
        a = allc.cpu().numpy()
        gi = a[:, 0, :].reshape(-1)
        gv = a[:, 1, :].reshape(-1)
        ok = gi >= 0
        gi, gv = gi[ok], gv[ok]
        # keys are the bits of non-negative doubles: compare as int64, ties -> lower pod index
        order = sorted(range(len(gi)), key=lambda j: (-int(gv[j]), int(gi[j])))
        sel = order[:k]
        return gi[sel], gv[sel]


def key_to_score(v):
    """int64 root-cause key -> the float64 value r*q it encodes (in 2^-60 * 2^-32 units)."""
    return np.asarray(v, np.int64).view(np.float64) / (2.0 ** 92)
