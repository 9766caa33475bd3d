"""f4 on the device: krca_group_reduce vs the oracle, EventsAgent / Coordinator vs the reference goldens."""
import numpy as np
import pytest

import agent_cases as A
import oracle
from krca import eventcols, native
from oracle_engine import OracleEngine

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    return native.NativeEngine()


def _records(rng, N, S, hot=0.0, p_sel=0.7):
    slot = rng.integers(-1, S + 2, N).astype(np.int32)  # includes ignored -1 and out-of-range slots
    if hot:
        h = rng.random(N) < hot
        slot[h] = rng.integers(0, min(S, 4), int(h.sum()))
    idx = np.arange(N, dtype=np.int64)
    ts = rng.integers(0, 7, N).astype(np.int64)  # heavy timestamp ties
    key = np.where(rng.random(N) < p_sel, (ts << 32) | (0x7FFFFFFF - idx), -1)
    return slot, key


@pytest.mark.parametrize("N,S,R,hot,ranked", [(1, 1, 1, 0, 1), (63, 5, 3, 0, 1), (5000, 40, 3, 0.5, 1),
                                              (20000, 3000, 3, 0.1, 0.5), (70000, 2, 6, 0, 1),
                                              (70000, 50000, 2, 0, 0.3), (9000, 100, 4, 0.2, 0)])
def test_group_reduce_vs_oracle(eng, N, S, R, hot, ranked):
    rng = np.random.default_rng(N + S + R)
    slot, key = _records(rng, N, S, hot)
    n_ranked = int(N * ranked)
    got = eng.group_reduce(slot, key, S, R, n_ranked=n_ranked)
    ref = oracle.group_reduce_ref(slot, key, S, R, n_ranked)
    for g, r, what in zip(got, ref, ("first", "count", "n_key", "top")):
        assert np.array_equal(g, r), what


def test_group_reduce_empty(eng):
    first, count, n_key, top = eng.group_reduce(np.zeros(0, np.int32), np.zeros(0, np.int64), 7, 3)
    assert (first == 2**31 - 1).all() and (count == 0).all() and (n_key == 0).all() and (top == -1).all()
    assert all(len(x) == 0 for x in eng.group_reduce(np.zeros(3, np.int32), np.zeros(3, np.int64), 0, 1)[:3])


def test_group_reduce_4m_records(eng):
    """Full-size property check: numpy's scatter-min / bincount / sorted top-3 of every slot."""
    rng = np.random.default_rng(7)
    N, S = 4_000_000, 300_000
    slot, key = _records(rng, N, S, hot=0.05)
    first, count, n_key, top = eng.group_reduce(slot, key, S, 3)
    ok = (slot >= 0) & (slot < S)
    s, k, i = slot[ok], key[ok], np.nonzero(ok)[0]
    f = np.full(S, 2**31 - 1, np.int64)
    np.minimum.at(f, s, i)
    assert np.array_equal(first, f)
    assert np.array_equal(count, np.bincount(s, minlength=S))
    sel = k >= 0
    assert np.array_equal(n_key, np.bincount(s[sel], minlength=S))
    o = np.lexsort((-k[sel], s[sel]))
    ss, kk = s[sel][o], k[sel][o]
    start = np.searchsorted(ss, np.arange(S))
    end = np.searchsorted(ss, np.arange(S), side="right")
    for r in range(3):
        exp = np.where(start + r < end, kk[np.minimum(start + r, len(kk) - 1)], -1)
        assert np.array_equal(top[r], exp), r


def test_events_goldens(eng):
    assert A.check_events(eng) == []
    assert A.check_events_random(eng) == []


def test_correlate_goldens(eng):
    assert A.check_correlate(eng) == []


class _Bulk(A.DictClient):
    def __init__(self, cols):
        super().__init__()
        self.cols = cols

    def get_event_columns(self, ns):
        return self.cols


def test_events_bulk_columns_vs_oracle_engine(eng):
    """200k columnar events (bulk accessor): device findings == the oracle engine's."""
    cols = eventcols.make_events(200_000, seed=5, n_obj=20_000, n_hosts=32)
    dev = A.EventsAgent(_Bulk(cols), engine=eng).analyze("x")
    ref = A.EventsAgent(_Bulk(cols), engine=OracleEngine()).analyze("x")
    assert "error" not in dev
    assert A.strip(dev) == A.strip(ref)
    assert len(dev["findings"]) > 1000
