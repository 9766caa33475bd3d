"""Pod-sharded cross-pod correlation (a9 on G GPUs).

Rank g of G owns the pods [g*n_max, (g+1)*n_max) (n_max a multiple of the 256-pod tile edge) and
their metric series.  One run (the same result as the single-device krca_corr_topk, bit for bit
whenever no candidate buffer overflows):

1. krca_corr_prepare on the local series; ONE all-gather each of the fp16 screening rows (zh) and
   the fp32 rows (z32) — every rank then holds the full standardized matrix (2.9 GB fp16 + 5.8 GB
   fp32 at 1M pods x 1440 steps, a small fraction of 288 GB of HBM).
2. krca_corr_shard_sample: the threshold sample of the rank's own pods -> phi; all-gather phi.
3. krca_corr_shard_tiles: the rank's share of the upper triangle (every G-th 8x8 super-tile, so
   the MFMA work is balanced and no pair is computed twice); candidates of ANY pod land in the
   rank's append buffers; |r| > tau counts and raw candidate counts are all-reduced (sum).
4. krca_corr_shard_pack_sizes / _pack: candidates grouped by owner; ONE all-to-all over RCCL.
5. krca_corr_shard_unpack + krca_corr_shard_merge: sort, exact float64 re-scoring, top-k and
   certificate of the rank's own pods (the rectangle pass for overflowed pods stays local: every
   rank holds every column).

The collectives go through a small comm object so that tests can run G shards in one process
on one device (tests/test_gpu_corr.py) and the CPU suite can check the partition logic.
"""
import ctypes
import math

import numpy as np

TB = 256  # tile edge of the correlation kernels (pods)


def corr_shard_range(P, world, rank):
    """Pods [lo, hi) of `rank`; n_max is a multiple of TB so every rank starts on a tile."""
    nb2 = max(1, math.ceil(P / TB))
    n_max = math.ceil(nb2 / world) * TB
    lo = min(P, rank * n_max)
    hi = min(P, lo + n_max)
    return lo, hi, n_max


class TorchComm:
    """torch.distributed collectives (nccl == RCCL on ROCm)."""

    def __init__(self, world, rank, group=None):
        self.world, self.rank, self.group = world, rank, group

    def all_gather(self, out, inp):
        from .rca import all_gather_flat
        all_gather_flat(out, inp, self.world, self.group)

    def all_reduce_sum(self, t):
        import torch.distributed as dist
        dist.all_reduce(t, group=self.group)

    def all_to_all(self, recv, send, recv_splits, send_splits):
        import torch.distributed as dist
        dist.all_to_all_single(recv, send, output_split_sizes=list(recv_splits),
                               input_split_sizes=list(send_splits), group=self.group)


class CorrShard:
    """One rank's state and phases (device tensors owned by torch; kernels through libkrca)."""

    def __init__(self, engine, P, T, k, tau, world, rank):
        import torch
        self.torch, self.eng, self.lib = torch, engine, engine.lib
        self.P, self.T, self.k, self.tau = int(P), int(T), int(k), float(tau)
        self.world, self.rank = int(world), int(rank)
        self.lo, self.hi, self.n_max = corr_shard_range(P, world, rank)
        self.n_loc = self.hi - self.lo
        self.Tp = int(self.lib.krca_corr_pad_steps(T))
        dev = engine.device
        rows = world * self.n_max
        self.zh = torch.zeros((rows, self.Tp), dtype=torch.int16, device=dev)
        self.z32 = torch.zeros((rows, self.T), dtype=torch.float32, device=dev)
        self.phi = torch.zeros(rows, dtype=torch.float32, device=dev)
        self.count = torch.zeros(P, dtype=torch.int32, device=dev)
        self.raw = torch.zeros(P, dtype=torch.int32, device=dev)
        words = self.lib.krca_corr_shard_ws_size(P, T, k, self.n_loc, world)
        self.ws = torch.empty(max(int(words), 1) * 4, dtype=torch.uint8, device=dev)
        self.out = dict(idx=torch.empty((max(self.n_loc, 1), k), dtype=torch.int32, device=dev),
                        val=torch.empty((max(self.n_loc, 1), k), dtype=torch.float32, device=dev),
                        cert=torch.empty(max(self.n_loc, 1), dtype=torch.float32, device=dev))

    def _chk(self, rc, what):
        from .native import _check
        _check(rc, what)

    def _args(self):
        return self.P, self.T, self.k, self.n_loc, self.world

    # -- phase 1: local standardization -> this rank's rows of zh / z32 ---------------------------
    def prepare(self, x_local, channel=0):
        """x_local [T, n_loc, M] on the device -> send slices (n_max rows each)."""
        torch = self.torch
        zl = self.eng.corr_prepare_device(x_local, channel) if self.n_loc else None
        zh_s = torch.zeros((self.n_max, self.Tp), dtype=torch.int16, device=self.eng.device)
        z32_s = torch.zeros((self.n_max, self.T), dtype=torch.float32, device=self.eng.device)
        if zl is not None:
            zh_s[:self.n_loc] = zl["zh"][:self.n_loc]
            z32_s[:self.n_loc] = zl["z32"]
        return zh_s, z32_s

    # -- phase 2: threshold sample of the own pods ------------------------------------------------
    def sample(self):
        e, p = self.eng, self.eng.ptr
        self._chk(self.lib.krca_corr_shard_sample(p(self.zh), self.P, self.T, self.k, self.lo, self.n_loc, self.world,
                                                  p(self.ws), p(self.phi), e._stream()), "krca_corr_shard_sample")
        g0 = self.rank * self.n_max  # == lo for every non-empty rank
        return self.phi[g0:g0 + self.n_max].clone()

    # -- phase 3: this rank's share of the upper triangle -----------------------------------------
    def tiles(self):
        e, p = self.eng, self.eng.ptr
        self._chk(self.lib.krca_corr_shard_tiles(p(self.zh), p(self.z32), self.P, self.T, self.k, self.tau, self.world, self.rank,
                                                 p(self.phi), self.n_loc, p(self.ws), p(self.count), p(self.raw),
                                                 e._stream()), "krca_corr_shard_tiles")

    # -- phase 4: candidates grouped by owner -----------------------------------------------------
    def pack(self):
        torch, e, p = self.torch, self.eng, self.eng.ptr
        tot = (ctypes.c_int64 * self.world)()
        P, T, k, n_loc, G = self._args()
        self._chk(self.lib.krca_corr_shard_pack_sizes(P, T, k, n_loc, G, self.n_max, p(self.ws), tot, e._stream()),
                  "krca_corr_shard_pack_sizes")
        sizes = [int(v) for v in tot]
        send = torch.empty((max(sum(sizes), 1), 4), dtype=torch.int32, device=e.device)
        self._chk(self.lib.krca_corr_shard_pack(P, T, k, n_loc, G, self.n_max, p(self.ws), p(send), e._stream()),
                  "krca_corr_shard_pack")
        return send[:sum(sizes)], sizes

    # -- phase 5: own pods ------------------------------------------------------------------------
    def merge(self, recv):
        e, p = self.eng, self.eng.ptr
        P, T, k, n_loc, G = self._args()
        self._chk(self.lib.krca_corr_shard_unpack(P, T, k, n_loc, G, self.lo, p(self.ws), p(recv), int(recv.shape[0]),
                                                  e._stream()), "krca_corr_shard_unpack")
        lcnt = self.raw[self.lo:self.hi].contiguous() if n_loc else self.raw[:1]
        self._chk(self.lib.krca_corr_shard_merge(p(self.zh), p(self.z32), P, T, k, self.tau, self.lo, n_loc, G,
                                                 p(self.phi), p(lcnt), p(self.ws), p(self.out["idx"]),
                                                 p(self.out["val"]), p(self.out["cert"]), e._stream()),
                  "krca_corr_shard_merge")
        return dict(idx=self.out["idx"][:n_loc], val=self.out["val"][:n_loc], cert=self.out["cert"][:n_loc],
                    count=self.count[self.lo:self.hi])

    # -- one full run over torch.distributed ------------------------------------------------------
    def run(self, x_local, comm, channel=0):
        zh_s, z32_s = self.prepare(x_local, channel)
        comm.all_gather(self.zh.view(-1), zh_s.view(-1))
        comm.all_gather(self.z32.view(-1), z32_s.view(-1))
        phi_s = self.sample()
        comm.all_gather(self.phi, phi_s)
        self.tiles()
        comm.all_reduce_sum(self.count)
        comm.all_reduce_sum(self.raw)
        send, sizes = self.pack()
        recv = exchange_candidates(comm, send, sizes, self.world, self.rank, self.eng.device)
        return self.merge(recv)


def exchange_candidates(comm, send, sizes, world, rank, device):
    """All-to-all of int4 candidate entries: sizes[h] = entries this rank sends to rank h (its
    pods' owner); returns the entries every rank sent here, in source-rank order."""
    import torch
    sz = torch.tensor(sizes, dtype=torch.int64, device=device)
    allsz = torch.empty(world * world, dtype=torch.int64, device=device)
    comm.all_gather(allsz, sz)
    m = allsz.view(world, world).cpu().numpy()  # m[src, dst] entries
    recv_sizes = [int(v) for v in m[:, rank]]
    recv = torch.empty((max(sum(recv_sizes), 1), 4), dtype=torch.int32, device=device)
    flat_send = send.reshape(-1) if send.numel() else torch.empty(0, dtype=torch.int32, device=device)
    comm.all_to_all(recv.view(-1)[:4 * sum(recv_sizes)], flat_send, [4 * v for v in recv_sizes],
                    [4 * v for v in sizes])
    return recv[:sum(recv_sizes)]


def run_emulated(engine, x, P, T, k, tau, world, channel=0):
    """TESTS: G shards in ONE process on one device, the collectives done with copies in the
    same order a distributed run uses.  Returns host arrays for all P pods."""
    import torch
    shards = [CorrShard(engine, P, T, k, tau, world, g) for g in range(world)]
    zs = [s.prepare(x[:, s.lo:s.hi, :].contiguous(), channel) for s in shards]
    zh = torch.cat([a for a, _ in zs])
    z32 = torch.cat([b for _, b in zs])
    for s in shards:
        s.zh.copy_(zh)
        s.z32.copy_(z32)
    phis = [s.sample() for s in shards]
    phi = torch.cat(phis)
    for s in shards:
        s.phi.copy_(phi)
    for s in shards:
        s.tiles()
    count = sum(s.count for s in shards)
    raw = sum(s.raw for s in shards)
    for s in shards:
        s.count.copy_(count)
        s.raw.copy_(raw)
    packed = [s.pack() for s in shards]
    outs = []
    for h, s in enumerate(shards):
        segs = []
        for g, (send, sizes) in enumerate(packed):
            o = int(np.sum(sizes[:h]))
            segs.append(send[o:o + sizes[h]])
        recv = torch.cat(segs) if segs else torch.empty((0, 4), dtype=torch.int32, device=engine.device)
        outs.append(s.merge(recv.contiguous()))
    res = {key: torch.cat([o[key] for o in outs]).cpu().numpy() for key in ("idx", "val", "cert", "count")}
    return res
