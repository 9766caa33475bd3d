"""The C5 streaming replay (krca/stream.py) pod-sharded over gloo on CPU, world sizes 1-3.

Each rank owns a pod range: its rolling state, its rows of the pull-CSR; every re-ranking
iteration is one all-gather.  After every window the sharded ranks, iteration counts and merged
top-10 must equal the single-process oracle chain (oracle.c_ppr_warm from the previous window's
ranks; scores = the batch C scorer over the series so far), bit for bit, for any number of ranks.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import ROOT

N, M, W, H = 2500, 8, 30, 90
WINDOWS = [W + 40, 5, 1, 1, 17, 1]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _mesh():
    from krca import synth
    m = synth.make_graph(N, n_edges=15 * N, seed=8)
    x = synth.make_metrics(N, M, sum(WINDOWS), window=W, seed=10, roots=m.roots,
                           hop_sets=synth.caller_hops(m, m.roots)).numpy()
    return m, x


def _worker(rank, world, port, out_q, snap_dir=None, snap_at=2, short_at=None):
    sys.path[:0] = [os.path.join(ROOT, "kubernetes-rca-system_amd"), os.path.join(ROOT, "oracle"),
                    os.path.join(ROOT, "tests")]
    import torch.distributed as dist
    from krca.rca import Comm, Config, shard_graph, shard_range
    from krca.stream import StreamingRCA
    from numpy_shard import NumpyShard
    if world > 1:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
    m, x = _mesh()
    cfg = Config(window=W)
    lo, hi, n_max = shard_range(N, world, rank)
    rp, col, od = shard_graph(m.row_ptr, m.col, m.outdeg, lo, hi)

    def fresh():
        shard = NumpyShard(np.zeros((0, hi - lo, M), np.float32), rp, col, od, N, n_max, world, cfg)
        return shard, StreamingRCA(None, m.row_ptr, m.col, m.outdeg, M, cfg, horizon=H, tol=1e-9, max_iter=60,
                                   comm=Comm(world, rank), shard=shard)
    shard, s = fresh()
    t, rows = 0, []
    for wi, d in enumerate(WINDOWS):
        if snap_dir is not None and wi == snap_at:
            # checkpoint between windows, continue in a new stream object restored from the file
            path = os.path.join(snap_dir, f"stream_rank{rank}.npz")
            s.snapshot(path)
            shard, s = fresh()
            s.restore(path)
        if short_at is not None and wi == short_at:
            # the re-rank's speculative first batch is the previous count + 1 steps: make it fall
            # short, so the window continues in the polled batches after a dropped merge
            s.last_iters = 2
        out = s.window(x[t:t + d, lo:hi, :])
        t += d
        rows.append((shard.r.copy(), out["iters"], [int(i) for i in out["top"][0]],
                     np.asarray(out["scores"]["n_exceed"]).copy()))
    out_q.put((rank, rows))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


@pytest.mark.parametrize("world,snap,short", [(1, False, False), (2, False, False), (3, False, False), (2, True, False),
                                              (2, False, True)])
def test_sharded_stream_matches_oracle_chain(world, snap, short, tmp_path):
    """snap: every rank snapshots its stream after window 2 and continues in a restored object.
    short: window 3's speculative first batch is too short (the fallback path)."""
    import oracle
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, str(tmp_path) if snap else None, 2, 3 if short else None))
             for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    m, x = _mesh()
    from krca.rca import Config
    FLOOR = Config().floor(x.shape[1], x.shape[2])  # the scale-aware floor of krca.rca.Config
    r_ref, t = None, 0
    for wi, d in enumerate(WINDOWS):
        t += d
        score = oracle.c_rolling_score(x[:t], W)["score"]
        # cold, then warm from the previous window's ranks; the default key of krca.rca.Config
        o = oracle.c_ppr_ex(m.row_ptr, m.col, m.outdeg, score, 0.5, 60, 1e-9, FLOOR, r_start=r_ref)
        r_ref, it = o["r"], o["it"]
        top = oracle.topk_ref(oracle.rca_keys_from(o, score, FLOOR, m.row_ptr, m.col), 10)[0].tolist()
        r_sh = np.concatenate([res[g][wi][0] for g in range(world)])
        assert np.array_equal(r_sh, r_ref), (world, wi)
        for g in range(world):
            assert res[g][wi][1] == it, (world, wi, res[g][wi][1], it)
            assert res[g][wi][2] == top, (world, wi)


def test_snapshot_refuses_another_stream(tmp_path):
    """A snapshot restores only into a stream of the same mesh, partition, horizon and config."""
    sys.path[:0] = [os.path.join(ROOT, "tests")]
    from krca.rca import Comm, Config, shard_graph, shard_range
    from krca.stream import StreamingRCA
    from numpy_shard import NumpyShard
    m, x = _mesh()

    def make(cfg, horizon):
        lo, hi, n_max = shard_range(N, 1, 0)
        rp, col, od = shard_graph(m.row_ptr, m.col, m.outdeg, lo, hi)
        sh = NumpyShard(np.zeros((0, N, M), np.float32), rp, col, od, N, n_max, 1, cfg)
        return StreamingRCA(None, m.row_ptr, m.col, m.outdeg, M, cfg, horizon=horizon, tol=1e-9, max_iter=60,
                            comm=Comm(1, 0), shard=sh)
    s = make(Config(window=W), H)
    s.window(x[:W + 5])
    path = str(tmp_path / "s.npz")
    s.snapshot(path)
    for other in (make(Config(window=W, alpha=0.6), H), make(Config(window=W), H + 1)):
        with pytest.raises(ValueError, match="differ"):
            other.restore(path)
    ok = make(Config(window=W), H)
    ok.restore(path)
    assert ok.t == W + 5 and ok.solved
