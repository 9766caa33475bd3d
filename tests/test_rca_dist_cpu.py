"""The pod-sharded RCA step (krca/rca.py) with world_size 2 and 3 over gloo on CPU.

Checks the multi-GPU path by construction: partitioning, column remap, the single all-gather per
PageRank iteration (partial sums in the payload) and the candidate merge must give the SAME bits
as the single-process oracle, for any number of ranks.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import ROOT

N, T, M = 3000, 200, 8


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _mesh():
    from krca import synth
    m = synth.make_graph(N, avg_degree=15, seed=4)
    hops = synth.caller_hops(m, m.roots)
    x = synth.make_metrics(N, M, T, window=60, seed=9, roots=m.roots, hop_sets=hops).numpy()
    return m, x


def _worker(rank, world, port, out_q, balanced=False):
    """balanced: False (uniform ranges), True (Partition.balanced ranges for both halves) or
    "split" (bench.py at G > 1: scoring on uniform ranges, PageRank on balanced ones, the scores
    all-gathered once per step by krca.rca.SplitShard)."""
    sys.path[:0] = [os.path.join(ROOT, "kubernetes-rca-system_amd"), os.path.join(ROOT, "oracle"),
                    os.path.join(ROOT, "tests")]
    import torch.distributed as dist
    from krca.rca import Comm, Config, Partition, RcaStep, SplitShard, shard_graph
    from numpy_shard import NumpyShard
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    m, x = _mesh()
    cfg = Config(iters=12)
    part = Partition.balanced(m.row_ptr, world) if balanced else Partition.uniform(N, world)
    lo, hi, n_max = part.range(rank)
    rp, col, od = shard_graph(m.row_ptr, m.col, m.outdeg, lo, hi, part)
    comm = Comm(world, rank)
    step_comm = comm
    if balanced in ("split", "replicated"):
        spart = Partition.uniform(N, world)
        slo, shi, s_slot = spart.range(rank)
        scorer = NumpyShard(x[:, slo:shi, :], np.zeros(1, np.int64), np.zeros(0, np.int64), np.zeros(0, np.int32), N,
                            s_slot, world, cfg)
        if balanced == "replicated":  # the whole mesh's solve on every rank, no collective inside it
            part = Partition([0, N])
            lo, hi, n_max = 0, N, N
            rp, col, od = shard_graph(m.row_ptr, m.col, m.outdeg, 0, N, part)
            ppr = NumpyShard(x, rp, col, od, N, N, 1, cfg)
            step_comm = Comm(1, 0)
        else:
            ppr = NumpyShard(x[:, lo:hi, :], rp, col, od, N, n_max, world, cfg)
        shard = SplitShard(scorer, ppr, spart, part, rank, comm)
    else:
        shard = NumpyShard(x[:, lo:hi, :], rp, col, od, N, n_max, world, cfg)
    # the default key needs every pod's scores (gathered, or the SplitShard's) and the whole graph
    idx, key = RcaStep(shard, step_comm, cfg, lo, explain=(m.row_ptr, m.col), part=None if balanced in (
        "split", "replicated") else part).run()
    out_q.put((rank, lo, shard.r.copy(), [int(i) for i in idx], [int(k) for k in key]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,balanced", [(2, False), (3, False), (2, True), (4, True), (3, "split"), (7, "split"),
                                           (3, "replicated")])
def test_sharded_rca_matches_single_process_oracle(world, balanced):
    """Uniform ranges and pods + in-edges balanced ranges (krca.rca.Partition: ranges of different
    lengths, columns in the exchange layout's virtual ids), and the split form (scoring uniform,
    PageRank balanced, scores all-gathered; world 7: the last uniform range is short, so the
    gathered scores carry padding), and the replicated solve (scores all-gathered, every rank
    solves the whole mesh): the same bits every way."""
    import oracle
    from krca.rca import Config
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, balanced)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    m, x = _mesh()
    score = oracle.c_rolling_score(x, 60)["score"]
    ridx, rf, r = oracle.rca_rank(m.row_ptr, m.col, m.outdeg, score, 0.5, 12, Config().floor(N, M), 10,
                                  tol=Config().tol)
    if balanced == "replicated":  # every rank holds the whole fixed point
        for _, _, rr, _, _ in res:
            assert np.array_equal(rr, r)
    else:
        r_sharded = np.concatenate([rr for _, _, rr, _, _ in res])
        assert np.array_equal(r_sharded, r)
    for _, _, _, idx, _ in res:  # every rank holds the same merged top-10
        assert idx == [int(i) for i in ridx]


def test_bench_metrics_do_not_depend_on_sharding():
    """bench.py's mesh is generated in fixed pod blocks: any shard holds the rows one GPU holds."""
    import torch
    from krca import synth
    roots, hops = np.array([5, 120, 250]), [np.array([7, 130]), np.array([260])]
    kw = dict(window=20, seed=3, roots=roots, hop_sets=hops, block=100)
    full = synth.make_metrics_range(0, 300, 8, 100, **kw)
    for cuts in ([0, 150, 300], [0, 100, 200, 300], [0, 77, 154, 231, 300]):
        parts = [synth.make_metrics_range(a, b, 8, 100, **kw) for a, b in zip(cuts, cuts[1:])]
        assert torch.equal(full, torch.cat(parts, 1))


def _gather_worker(rank, world, port, out_q):
    sys.path[:0] = [os.path.join(ROOT, "kubernetes-rca-system_amd")]
    import torch
    import torch.distributed as dist
    from krca.rca import all_gather_flat
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    got = {}
    for dt in (torch.int16, torch.float16, torch.int64, torch.float32):
        inp = (torch.arange(6) + 100 * rank).to(dt)
        out = torch.empty(6 * world, dtype=dt)
        all_gather_flat(out, inp, world)
        got[str(dt)] = out.tolist()
    out_q.put((rank, got))
    dist.barrier()
    dist.destroy_process_group()


def test_all_gather_flat_moves_dtypes_the_backends_lack():
    """The correlation's fp16 rows travel as int16 (krca/corr_dist.py), a dtype gloo refuses and
    RCCL / NCCL do not have: all_gather_flat moves such tensors as uint8 views, bit for bit."""
    import torch
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for dt in (torch.int16, torch.float16, torch.int64, torch.float32):
        want = torch.cat([(torch.arange(6) + 100 * r).to(dt) for r in range(world)]).tolist()
        assert res[0][str(dt)] == want and res[1][str(dt)] == want


def test_partition_balanced_ranges():
    """Partition.balanced: contiguous ranges covering [0, N); no range past t x N / G pods or
    t x EDGE_SLACK x E / G in-edges (t from the bisection, within 10 % of the uniform ranges' pod
    balance on this mesh); virtual ids land in the owner's slice; unpad inverts the gather."""
    from krca import synth
    from krca.rca import EDGE_SLACK, Partition, remap_cols, slice_words
    m = synth.make_graph(20000, avg_degree=20, seed=2)
    E = int(m.row_ptr[-1])
    for world in (1, 2, 3, 8):
        p = Partition.balanced(m.row_ptr, world)
        b = p.bounds
        assert b[0] == 0 and b[-1] == 20000 and np.all(np.diff(b) >= 0) and p.world == world
        edges = np.diff(m.row_ptr[b])
        t = max(np.max(np.diff(b)) / (20000 / world), np.max(edges) / (EDGE_SLACK * E / world))
        assert t < 1.5, (world, t)
        j = np.arange(20000)
        g = p.owner(j)
        assert np.all((b[g] <= j) & (j < b[g + 1]))
        v = p.virtual(j).astype(np.int64)
        u = remap_cols(v, p.n_slot)  # uint32 index of the code in w_all[world][slice]
        assert np.array_equal(u // (2 * slice_words(p.n_slot)), g)
        assert np.array_equal(u % (2 * slice_words(p.n_slot)), j - b[g])
        padded = np.full(world * p.n_slot, -1)
        for r in range(world):
            padded[r * p.n_slot:r * p.n_slot + b[r + 1] - b[r]] = np.arange(b[r], b[r + 1])
        assert np.array_equal(p.unpad(padded), j)
    u = Partition.uniform(20000, 3)
    assert np.array_equal(u.virtual(np.arange(20000)), np.arange(20000))
    hub = Partition.balanced(m.row_ptr, 8)  # the hub services at low ids: a short first range
    assert hub.bounds[1] < 20000 // 8 and np.max(np.diff(m.row_ptr[hub.bounds])) <= 1.5 * EDGE_SLACK * E / 8


def test_split_shard_rejects_partitions_it_cannot_gather():
    """SplitShard needs uniform scoring ranges (the gathered scores are then in pod order), two
    partitions of the same pods over the same ranks, and more than one rank."""
    import torch
    from krca.rca import Comm, Partition, SplitShard

    class Stub:
        def __init__(self):
            self.send = torch.zeros(4, dtype=torch.int64)

    m, _ = _mesh()
    bal = Partition.balanced(m.row_ptr, 3)
    uni = Partition.uniform(N, 3)
    assert not np.array_equal(bal.bounds, uni.bounds)
    for spart, ppart, world in ((bal, bal, 3), (uni, Partition.uniform(N, 2), 3), (Partition.uniform(N, 1),
                                                                                   Partition.uniform(N, 1), 1)):
        with pytest.raises(ValueError):
            SplitShard(Stub(), Stub(), spart, ppart, 0, Comm(world, 0))
    s = SplitShard(Stub(), Stub(), uni, bal, 1, Comm(3, 1))
    lo, hi, _ = bal.range(1)
    assert s.ppr.score_out["score"].shape == (hi - lo,)
