"""RCCL on the hardware: a world-size-1 "nccl" process group on the one GPU of the box.

RCCL refuses two ranks on one device, so the multi-rank runs are the driver's; but a one-rank
communicator is legal, and with krca.rca.Comm(collective=True) every call site of the multi-GPU
path runs its collective through RCCL even with one rank:

* RcaStep, PageRank rows on the scoring's range and on a SplitShard (score all-gather): the
  per-iteration all-gather (the process group's _allgather_base), the candidate merge's all-gather;
* krca/corr_dist.py: the all-gathers of the fp16 / fp32 rows (the uint8-view dtype trick), phi,
  the count all-reduces and the candidate all-to-all;
* one StreamingRCA window (warm re-rank under the L1 stop rule, speculative batch);
* the HIP-graph capture of the solve with the RCCL all-gather inside (KRCA_RCA_GRAPH path).
Every result bit-identical to the oracle (or the single-device path).
"""
import socket

import numpy as np
import pytest
import torch

import oracle
from krca import native, synth
from krca.rca import Comm, Config, DeviceShard, Partition, RcaStep, SplitShard, all_gather_flat, shard_graph

pytestmark = pytest.mark.gpu

N = 20_000


@pytest.fixture(scope="module")
def eng():
    return native.NativeEngine()


@pytest.fixture(scope="module")
def pg():
    import torch.distributed as dist
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    assert dist.get_backend() == "nccl"
    yield dist.group.WORLD
    dist.destroy_process_group()


@pytest.fixture(scope="module")
def mesh():
    m = synth.make_graph(N, n_edges=20 * N, seed=12)
    x = synth.make_metrics(N, 8, 300, seed=12, roots=m.roots, hop_sets=synth.caller_hops(m, m.roots)).cuda()
    return m, x


def _oracle_top(m, score, cfg):
    return oracle.rca_rank(m.row_ptr, m.col, m.outdeg, score, cfg.alpha, cfg.iters, cfg.floor(N, 8), cfg.k, tol=cfg.tol)


def test_rccl_dtype_views(pg):
    """all_gather_flat over RCCL: int16 / fp16 travel as uint8 views, int64 / f32 as they are."""
    for dt in (torch.int16, torch.float16, torch.int64, torch.float32, torch.uint8):
        inp = (torch.arange(37, device="cuda") * 3 - 5).to(dt)
        out = torch.empty(37, dtype=dt, device="cuda")
        all_gather_flat(out, inp, 1)
        assert torch.equal(out, inp), dt


def test_rccl_rca_step_uniform(eng, pg, mesh):
    """The pod-sharded step with one rank over RCCL: 31 all-gathers through _allgather_base, the
    candidate merge's all-gather; ranks and top-10 bit-identical to the oracle."""
    m, x = mesh
    cfg = Config()
    comm = Comm(1, 0, collective=True)
    sh = DeviceShard(eng, x, *shard_graph(m.row_ptr, m.col, m.outdeg, 0, N), N, N, 1, cfg, pingpong=False)
    assert not sh.fused
    step = RcaStep(sh, comm, cfg, 0)
    idx, _ = step.run()
    # init's exchange + one per issued step (the stop rule's count is unknown to the first solve: the
    # cap), all through the direct entry point
    assert comm.direct_calls == cfg.iters + 1 and step.last_iters > 0
    idx2, _ = step.run()  # the second solve issues the count + 1 steps
    assert comm.direct_calls == cfg.iters + 1 + step.last_iters + 2 and list(idx2) == list(idx)
    score = sh.score_out["score"].cpu().numpy()
    ridx, _, r = _oracle_top(m, score, cfg)
    assert np.array_equal(sh.r[:N].cpu().numpy(), r)
    assert [int(i) for i in idx] == ridx.tolist()


@pytest.mark.parametrize("mode", ["balanced", "replicated"])
def test_rccl_split_shard(eng, pg, mesh, mode):
    """SplitShard with one rank over RCCL: the score all-gather (and, balanced, the solve's)."""
    m, x = mesh
    cfg = Config()
    comm = Comm(1, 0, collective=True)
    spart = Partition.uniform(N, 1)
    ppart = Partition([0, N])
    nograph = (np.zeros(1, np.int64), np.zeros(0, np.int32), np.zeros(0, np.int32))
    scorer = DeviceShard(eng, x, *nograph, N, N, 1, cfg, pingpong=False)
    replicated = mode == "replicated"
    ppr = DeviceShard(eng, None, *shard_graph(m.row_ptr, m.col, m.outdeg, 0, N, ppart), N, N, 1, cfg,
                      pingpong=replicated)
    sh = SplitShard(scorer, ppr, spart, ppart, 0, comm)
    idx, _ = RcaStep(sh, Comm(1, 0) if replicated else comm, cfg, 0, explain=(m.row_ptr, m.col)).run()
    score = scorer.score_out["score"].cpu().numpy()
    ridx, _, r = _oracle_top(m, score, cfg)
    assert np.array_equal(ppr.r[:N].cpu().numpy(), r)
    assert [int(i) for i in idx] == ridx.tolist()


def test_rccl_corr_dist(eng, pg):
    """krca/corr_dist.py with one rank over RCCL (all-gathers, all-reduces, the all-to-all) equals
    the single-device correlation bit for bit."""
    from krca.corr_dist import CorrShard, TorchComm
    P, T, k, tau = 6000, 720, 10, 0.5
    x = synth.make_metrics(P, 1, T, seed=5, group_size=20).cuda()
    z = eng.corr_prepare_device(x, 0)
    ref = eng.corr_topk_device(z, k, tau)
    got = CorrShard(eng, P, T, k, tau, 1, 0).run(x, TorchComm(1, 0))
    for key in ("idx", "val", "count", "cert"):
        assert torch.equal(got[key][:P], ref[key][:P]), key


def test_rccl_stream_window(eng, pg, mesh):
    """Two StreamingRCA windows (cold, then warm under the L1 stop rule with the speculative batch)
    with one rank over RCCL: ranks, iteration counts and top-10 = the oracle chain."""
    from krca.stream import StreamingRCA
    m, x = mesh
    cfg = Config()
    s = StreamingRCA(eng, m.row_ptr, m.col, m.outdeg, 8, cfg, horizon=240, tol=1e-9, max_iter=60,
                     comm=Comm(1, 0, collective=True))
    assert not s.shard.pingpong
    r_ref, t = None, 0
    for d in (290, 1, 9):
        out = s.window(x[t:t + d].contiguous())
        t += d
        score = out["scores"]["score"].cpu().numpy()
        o = oracle.c_ppr_ex(m.row_ptr, m.col, m.outdeg, score, cfg.alpha, 60, 1e-9, cfg.floor(N, 8), r_start=r_ref)
        r_ref = o["r"]
        assert np.array_equal(s.shard.r[:N].cpu().numpy(), r_ref), t
        assert out["iters"] == o["it"], t
        top = oracle.topk_ref(oracle.rca_keys_from(o, score, cfg.floor(N, 8), m.row_ptr, m.col), cfg.k)[0]
        assert [int(i) for i in out["top"][0]] == top.tolist(), t


@pytest.mark.parametrize("producer", [False, True])
@pytest.mark.parametrize("direct", [False, True])
def test_rccl_graph_capture_plain_allgather(pg, direct, producer):
    """One all-gather captured into a HIP graph and replayed after its input changed (the public
    all_gather_into_tensor, or the process group's _allgather_base as Comm.exchange calls it);
    producer: a kernel that writes the input is captured before it (the graph must order the two)."""
    import torch.distributed as dist
    inp = torch.arange(1000, dtype=torch.int64, device="cuda")
    out = torch.zeros(1000, dtype=torch.int64, device="cuda")
    pgd = dist.distributed_c10d._get_default_group()
    opts = dist.distributed_c10d.AllgatherOptions()

    def gather():
        if producer:
            inp.mul_(3).add_(1)
        if direct:
            pgd._allgather_base(out, inp, opts).wait()
        else:
            dist.all_gather_into_tensor(out, inp)
        if producer:
            out.add_(5)  # a consumer after it
    gather()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.graph(g, stream=side):
        gather()
    torch.cuda.current_stream().wait_stream(side)
    inp.add_(7)
    out.zero_()
    want = inp * 3 + 1 if producer else inp.clone()
    g.replay()
    torch.cuda.synchronize()
    got = out - 5 if producer else out
    assert torch.equal(got, want), (got[:5].tolist(), want[:5].tolist())


@pytest.mark.parametrize("tol", [0.0, 1e-10])
def test_rccl_graph_capture_with_allgather(eng, pg, mesh, tol):
    """The solve captured into a HIP graph with the RCCL all-gather inside (RcaStep graph=True),
    replayed: the same bits as the eager collective sequence, also after the scores change, with a
    fixed iteration count and under the stop rule (graphs per step count)."""
    m, x0 = mesh
    cfg = Config(tol=tol)
    res = {}
    for graph in (False, True):
        x = x0.clone()
        comm = Comm(1, 0, collective=True)
        sh = DeviceShard(eng, x, *shard_graph(m.row_ptr, m.col, m.outdeg, 0, N), N, N, 1, cfg, pingpong=False)
        step = RcaStep(sh, comm, cfg, 0, graph=graph)
        out = []
        for shift in (0.0, 3.0):
            x.copy_(x0)
            x[-1, :50] += shift * 10.0  # new scores under the captured buffers
            idx, key = step.run()
            out.append(([int(i) for i in idx], sh.r[:N].cpu().numpy().copy()))
        res[graph] = out
    for (ia, ra), (ib, rb) in zip(res[False], res[True]):
        assert ia == ib and np.array_equal(ra, rb)
    assert not np.array_equal(res[True][0][1], res[True][1][1])


class _CopyExchange:
    """The exchange as a device copy (what a one-rank all-gather does), for the capture diagnostic."""
    world, rank, collective = 1, 0, True

    def exchange(self, shard):
        shard.w_all.copy_(shard.send)

    def all_gather(self, out, inp):
        out.copy_(inp)


@pytest.mark.parametrize("how", ["copy", "public", "direct"])
def test_rccl_graph_capture_interleaved(eng, pg, mesh, how):
    """An eager collective solve and a captured one (the exchange a device copy, the public all-gather
    or the direct one) run alternately, the scores changing between rounds: ranks, keys and top-10
    equal after every replay.  (With the runtime's graph packet capture on, the second replay ran
    with clobbered arguments -- a garbage ctl header -- R5k-R5m; tests/conftest.py turns it off.)"""
    m, x0 = mesh
    cfg = Config(tol=0.0)
    xe, xg = x0.clone(), x0.clone()
    sh_e = DeviceShard(eng, xe, *shard_graph(m.row_ptr, m.col, m.outdeg, 0, N), N, N, 1, cfg, pingpong=False)
    st_e = RcaStep(sh_e, Comm(1, 0, collective=True), cfg, 0)
    comm = _CopyExchange() if how == "copy" else Comm(1, 0, collective=True)
    if how == "public":
        comm._direct = False
    sh = DeviceShard(eng, xg, *shard_graph(m.row_ptr, m.col, m.outdeg, 0, N), N, N, 1, cfg, pingpong=False)
    step = RcaStep(sh, comm, cfg, 0, graph=True)
    report = []
    for shift in (0.0, 3.0):
        for x in (xe, xg):
            x[-1, :50] += shift * 10.0
        ie, _ = st_e.run()
        ig, _ = step.run()
        torch.cuda.synchronize()
        diff = {name: int((getattr(sh_e, name)[:N] != getattr(sh, name)[:N]).sum().item())
                for name in ("r", "q", "d", "key")}
        diff["score"] = int((sh_e.score_out["score"] != sh.score_out["score"]).sum().item())
        ce, cg = sh_e.ctl.cpu().numpy(), sh.ctl.cpu().numpy()
        he, hg = ce[:48].view(np.uint8), cg[:48].view(np.uint8)
        diff["ctl_head"] = [(f, float(np.frombuffer(he[o:o + 8].tobytes(), t)[0]), float(np.frombuffer(hg[o:o + 8].tobytes(), t)[0]))
                            for f, o, t in (("tele", 0, np.float64), ("q_total", 8, np.int64), ("tele_used", 32, np.float64))
                            if he[o:o + 8].tobytes() != hg[o:o + 8].tobytes()]
        diff["ctl_head"] += [("conv_iter", ce[16:24].tolist(), cg[16:24].tolist())] if ce[16:24].tobytes() != cg[16:24].tobytes() else []
        diff["ctl_rest"] = int((ce[48:] != cg[48:]).sum())
        diff["top"] = [int(i) for i in ie] == [int(i) for i in ig]
        report.append((shift, diff))
    assert torch.equal(sh.w_all, sh.send), how
    assert all(d["top"] and d["r"] == 0 and d["key"] == 0 for _, d in report), f"{how}: {report!r}"
