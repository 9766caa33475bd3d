"""NumPy restatement of krca.rca.DeviceShard — TESTS ONLY.

Same integer/float64 expressions as csrc/ppr.hip (shard kernels) and oracle/krca_oracle.c, so
the distributed orchestration of krca/rca.py (partitioning, column remap, one all-gather per
iteration with the partial sums in the payload, the G = 1 ping-pong swap, candidate merge) can be
exercised on CPU with the gloo backend and compared bit-for-bit with the single-process oracle.
Slot layout of the send tail: residual | dangling | seed total, NSPREAD slots each (the device
spreads its atomics over them; only the sums matter).
"""
import numpy as np
import torch

import oracle
from krca.rca import NSET, NSPREAD, SET_WORDS, remap_cols, slice_words, wslots

FIX = 1152921504606846976.0


def _w(r, deg, alpha):
    """Weight codes (csrc/ppr.hip wenc) of floor(r * alpha / deg)."""
    w = np.zeros(len(r), np.int64)
    nz = deg > 0
    coef = alpha / deg[nz].astype(np.float64)
    w[nz] = (r[nz].astype(np.float64) * coef).astype(np.int64)
    out = w.astype(np.uint32)
    big = w >= (1 << 26)
    sh = np.zeros(len(w), np.int64)
    sh[big] = np.floor(np.log2(w[big].astype(np.float64))).astype(np.int64) - 25
    # log2 of a float64 can land one off near powers of two: fix up with exact integer tests
    sh[big] += (w[big] >> (sh[big] + 25)) >= 2
    sh[big] -= (w[big] >> (sh[big] + 25)) < 1
    out[big] = ((sh[big] << 26) | (w[big] >> sh[big])).astype(np.uint32)
    return out


def _wdec(c):
    c = c.astype(np.int64)
    return (c & 0x3FFFFFF) << (c >> 26)


class NumpyShard:
    def __init__(self, x_local, row_ptr_local, col_local, outdeg_local, N, n_max, world, cfg):
        self.cfg, self.N, self.n_max, self.world = cfg, N, n_max, world
        self.x = np.asarray(x_local, np.float32)
        self.M = int(self.x.shape[2]) if self.x.ndim == 3 else 1  # metrics per pod (the seed floor's scale)
        self.rp = np.asarray(row_ptr_local, np.int64)
        c = np.asarray(col_local, np.int64)
        self.col = remap_cols(c, n_max)
        self.deg = np.asarray(outdeg_local, np.int32)
        self.n = len(self.deg)
        self.rows = np.repeat(np.arange(self.n), np.diff(self.rp))
        self.ws = wslots(n_max)
        self.host_csr = (row_ptr_local, col_local)
        self.recv = np.zeros(self.n, np.int64)  # acc of the last step that updated the rows
        self.send = torch.zeros(slice_words(n_max), dtype=torch.int64)
        self.w_all = torch.zeros((1 if world == 1 else world) * slice_words(n_max), dtype=torch.int64)
        self.ctl = {}

    def score(self):
        self.score_out = oracle.c_rolling_score(self.x, self.cfg.window, self.cfg.z_threshold)
        return self.score_out

    def init(self, alpha, floor):
        s = self.score_out["score"]
        v = s.astype(np.float64) - np.float64(np.float32(floor))
        self.q = np.where(v > 0, (np.maximum(v, 0) * 4294967296.0).astype(np.int64), 0)
        r0 = np.int64(FIX / float(self.N))
        self.r = np.full(self.n, r0, np.int64)
        self.recv = self.r.copy()  # no step yet: no teleport share recorded (the device's is 0)
        snd = self.send.numpy()
        snd[self.ws:] = 0
        if self.world == 1:
            self.w_all.numpy()[self.ws:] = 0  # the first folded step writes the other buffer
        snd.view(np.uint32)[:self.n] = _w(self.r, self.deg, alpha)
        snd[self.ws + NSPREAD] = int(self.r[self.deg == 0].sum())
        snd[self.ws + 2 * NSPREAD] = int(self.q.sum())
        self.ctl = dict(tele=0.0, q_total=0, converged=0, iter=0)

    def _set_sums(self, sset):
        w = self.w_all.numpy().reshape(self.world, slice_words(self.n_max))[:, self.ws + sset * SET_WORDS:]
        return tuple(int(w[:, i * NSPREAD:(i + 1) * NSPREAD].sum()) for i in range(3))

    def step_folded(self, alpha, tol, it, flags=3):
        """krca_ppr_shard_step_folded: the reduction of set (it-1) % NSET, then the step into set
        it % NSET; set (it+1) % NSET of the next write target zeroed."""
        c = self.ctl
        if c["converged"]:
            return
        err, dang, qs = self._set_sums((it - 1) % NSET)
        nxt = self.w_all if self.world == 1 else self.send
        zs = self.ws + ((it + 1) % NSET) * SET_WORDS
        nxt.numpy()[zs:zs + SET_WORDS] = 0
        if it == 1:
            c["q_total"] = qs
        c["iter"] = it - 1
        lim = float(self.N) * tol * FIX if tol > 0 else 0.0
        if it > 1 and lim > 0 and float(err) < lim:
            c["converged"] = it - 1
            return
        c["tele"] = (1.0 - alpha) * FIX + alpha * float(dang)
        self.step(alpha, flags, sset=it % NSET)

    def finish(self, alpha, tol, it):
        c = self.ctl
        if c["converged"]:
            return
        err, dang, _ = self._set_sums(it % NSET)
        c["iter"] = it
        lim = float(self.N) * tol * FIX if tol > 0 else 0.0
        if lim > 0 and float(err) < lim:
            c["converged"] = it
            return
        c["tele"] = (1.0 - alpha) * FIX + alpha * float(dang)

    def step(self, alpha, flags=3, sset=0):
        """Pull SpMV fused with the update: reads w_all, writes r and send (krca_ppr_shard_step)."""
        if self.ctl["converged"]:
            return
        w = self.w_all.numpy().view(np.uint32)
        acc = np.zeros(self.n, np.int64)
        np.add.at(acc, self.rows, _wdec(w[self.col]))
        qt = self.ctl["q_total"]
        tele = self.ctl["tele"]
        # t_i = q_i * (tele / qtot) (csrc/ppr.hip update_row), uniform 1/N when every seed is at the floor
        t = ((self.q.astype(np.float64) * (tele / float(qt))).astype(np.int64) if qt > 0
             else np.full(self.n, np.int64((1.0 / float(self.N)) * tele), np.int64))
        rn = acc + t
        err = int(np.abs(rn - self.r).sum())
        self.r = rn
        self.recv = acc
        snd = self.send.numpy()
        snd.view(np.uint32)[:self.n] = _w(rn, self.deg, alpha)
        o = self.ws + sset * SET_WORDS
        snd[o] += err
        snd[o + NSPREAD] += int(rn[self.deg == 0].sum())

    def reduce(self, alpha, tol, first):
        w = self.w_all.numpy().reshape(self.world, slice_words(self.n_max))[:, self.ws:]
        err, dang, qs = (int(w[:, i * NSPREAD:(i + 1) * NSPREAD].sum()) for i in range(3))
        self.send.numpy()[self.ws:] = 0
        c = self.ctl
        if c["converged"]:
            return
        if first:
            c["q_total"] = qs
        else:
            c["iter"] += 1
            lim = float(self.N) * tol * FIX if tol > 0 else 0.0
            if lim > 0 and float(err) < lim:
                c["converged"] = c["iter"]
                return
        c["tele"] = (1.0 - alpha) * FIX + alpha * float(dang)

    def local_topk(self, k):
        key = (self.r.astype(np.float64) * self.q.astype(np.float64)).view(np.int64)
        return oracle.topk_ref(key, min(k, self.n))

    def local_topk_explained(self, k, score_all, floor, graph, lo):
        """krca_rca_explain (the C restatement over the whole graph) + krca_rca_key_explained."""
        d = oracle.c_rca_explain(np.asarray(score_all, np.float32), floor, graph.row_ptr, graph.col, lo, lo + self.n)
        key = oracle.c_rca_key_explained(self.r, self.recv, self.q, d)
        return oracle.topk_ref(key, min(k, self.n))

    # -- streaming (krca/stream.py): the batch oracle over the series so far ---------------------
    def stream_score(self, x_new, t0, horizon):
        """krca_stream_score's contract restated: outputs of the batch scorer over the whole series
        so far, n_exceed over the last `horizon` evaluated steps (a difference of prefix counts)."""
        x_new = np.asarray(x_new.cpu() if hasattr(x_new, "cpu") else x_new, np.float32)
        self.M = int(x_new.shape[2])
        hist = getattr(self, "_hist", None)
        self._hist = x_new if hist is None else np.concatenate([hist, x_new])
        assert len(self._hist) == t0 + len(x_new)
        W = self.cfg.window
        t = len(self._hist)

        def prefix(tt):
            return oracle.c_rolling_score(self._hist[:tt], W)["n_exceed"] if tt > W else np.zeros(self.n, np.int32)
        out = oracle.c_rolling_score(self._hist, W)  # t <= W: z = 0, no exceedance
        out["n_exceed"] = prefix(t) - prefix(t - horizon) if t - horizon > W else prefix(t)
        self.score_out = out
        return out

    def state_dict(self, M, horizon):
        """Stream snapshot of this restatement: the series so far (its whole rolling state) + ranks."""
        hist = getattr(self, "_hist", None)
        r = getattr(self, "r", None)
        return dict(hist=np.zeros((0, self.n, M), np.float32) if hist is None else hist,
                    r=np.zeros(self.n, np.int64) if r is None else r.copy())

    def load_state_dict(self, st, M, horizon):
        self.M = int(M)
        self._hist = np.asarray(st["hist"], np.float32)
        self.r = np.asarray(st["r"], np.int64).copy()

    def init_warm(self, alpha, floor):
        """krca_ppr_shard_init_warm: new seeds, w and dangling mass from the kept ranks."""
        s = self.score_out["score"]
        v = s.astype(np.float64) - np.float64(np.float32(floor))
        self.q = np.where(v > 0, (np.maximum(v, 0) * 4294967296.0).astype(np.int64), 0)
        snd = self.send.numpy()
        snd[self.ws:] = 0
        if self.world == 1:
            self.w_all.numpy()[self.ws:] = 0
        self.recv = self.r.copy()
        snd.view(np.uint32)[:self.n] = _w(self.r, self.deg, alpha)
        snd[self.ws + NSPREAD] = int(self.r[self.deg == 0].sum())
        snd[self.ws + 2 * NSPREAD] = int(self.q.sum())
        self.ctl = dict(tele=0.0, q_total=0, converged=0, iter=0)

    def ctl_async(self):  # the restatement runs eagerly: the poll is the current state
        return self.ctl_read()

    def ctl_wait(self, handle):
        return handle

    def ctl_read(self):
        c = self.ctl
        return (c["converged"] or c["iter"]), bool(c["converged"])
