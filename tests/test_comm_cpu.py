"""krca.rca.Comm's per-iteration exchange on CPU with a mocked process group: the
RCCL path calls the group's _allgather_base(w_all, send, AllgatherOptions) directly -- the options
class comes from torch.distributed.distributed_c10d, where torch 2.10 keeps it -- and falls back
to the public all-gather for good when the first direct call raises; later failures propagate.
A one-rank Comm(collective=True) runs the collective too (the world-size-1 RCCL tests).  The
options carry asyncOp = False (the collective on the caller's stream, as the public wrapper's)."""
import types

import pytest
import torch
import torch.distributed as dist

from krca import rca


class FakeWork:
    def wait(self):
        return True


class FakePG:
    def __init__(self, fail=0):
        self.calls, self.fail = [], fail

    def _allgather_base(self, out, inp, opts):
        self.calls.append((out, inp, type(opts).__name__, getattr(opts, "asyncOp", None)))
        if self.fail:
            self.fail -= 1
            raise RuntimeError("no such collective")
        out.copy_(inp.repeat(out.numel() // inp.numel()))
        return FakeWork()


def _shard(n=6):
    return types.SimpleNamespace(send=torch.arange(n, dtype=torch.int64), w_all=torch.zeros(2 * n, dtype=torch.int64))


def _patch(monkeypatch, pg, backend="nccl"):
    monkeypatch.setattr(dist, "get_backend", lambda group=None: backend)
    monkeypatch.setattr(dist.distributed_c10d, "_get_default_group", lambda: pg)
    gathered = []

    def fake_flat(out, inp, world, group=None, gloo=None):
        gathered.append((out, inp))
        out.copy_(inp.repeat(world))
    monkeypatch.setattr(rca, "all_gather_flat", fake_flat)
    return gathered


def test_allgather_options_come_from_c10d():
    assert getattr(dist.distributed_c10d, "AllgatherOptions", None) is not None


def test_exchange_calls_allgather_base(monkeypatch):
    pg = FakePG()
    gathered = _patch(monkeypatch, pg)
    c, sh = rca.Comm(2, 0), _shard()
    for _ in range(3):
        c.exchange(sh)
    assert len(pg.calls) == 3 and c.direct_calls == 3 and not gathered
    out, inp, opts, async_op = pg.calls[0]
    assert out is sh.w_all and inp is sh.send and opts == "AllgatherOptions"
    assert async_op is False  # enqueued on the caller's stream (HIP-graph capture safe)
    assert sh.w_all.tolist() == list(range(6)) * 2


def test_exchange_accepts_no_work_object(monkeypatch):
    """asyncOp = False: the process group may return None instead of a work object (torch 2.10's
    all_gather_into_tensor checks for it too); that is a completed direct call, not a failure."""
    class NoWorkPG(FakePG):
        def _allgather_base(self, out, inp, opts):
            super()._allgather_base(out, inp, opts)
            return None
    pg = NoWorkPG()
    gathered = _patch(monkeypatch, pg)
    c, sh = rca.Comm(2, 0), _shard()
    c.exchange(sh)
    c.exchange(sh)
    assert c.direct_calls == 2 and len(pg.calls) == 2 and not gathered


def test_exchange_falls_back_once_then_for_good(monkeypatch):
    pg = FakePG(fail=1)
    gathered = _patch(monkeypatch, pg)
    c, sh = rca.Comm(2, 0), _shard()
    c.exchange(sh)  # the direct call raises: the public all-gather does the exchange
    c.exchange(sh)  # and every later one
    assert len(pg.calls) == 1 and c.direct_calls == 0 and len(gathered) == 2
    assert sh.w_all.tolist() == list(range(6)) * 2


def test_exchange_failure_after_success_propagates(monkeypatch):
    pg = FakePG()
    _patch(monkeypatch, pg)
    c, sh = rca.Comm(2, 0), _shard()
    c.exchange(sh)
    pg.fail = 1
    with pytest.raises(RuntimeError):
        c.exchange(sh)


def test_gloo_takes_the_public_path(monkeypatch):
    pg = FakePG()
    gathered = _patch(monkeypatch, pg, backend="gloo")
    c, sh = rca.Comm(2, 0), _shard()
    c.exchange(sh)
    assert not pg.calls and len(gathered) == 1


def test_one_rank_swap_or_collective(monkeypatch):
    pg = FakePG()
    _patch(monkeypatch, pg)
    sh = _shard()
    send, w_all = sh.send, sh.w_all
    rca.Comm(1, 0).exchange(sh)  # the ping-pong swap, no collective
    assert sh.send is w_all and sh.w_all is send and not pg.calls
    sh = types.SimpleNamespace(send=torch.arange(4, dtype=torch.int64), w_all=torch.zeros(4, dtype=torch.int64))
    c = rca.Comm(1, 0, collective=True)
    c.exchange(sh)
    assert len(pg.calls) == 1 and sh.w_all.tolist() == [0, 1, 2, 3]

