"""f2 service-graph construction on the device (csrc/topograph.hip) — SURVEY.md §8f.

* the agents' graph build and ResourceAnalyzer's selector matches through libkrca against the
  reference's graphs (tests/golden/topograph_cases.json);
* krca_selector_match against the oracle on random id sets, and bit-exact at 1M objects against a
  vectorised restatement (ids drawn from a 64-id universe, so every set is a 64-bit mask and the
  test is (obj & sel) == sel);
* krca_substr_match against Python's ``in``: every returned pair is verified, and a sample of
  values is checked for completeness against all keys."""
import random

import numpy as np
import pytest

import agent_cases as A
import oracle
from krca import native, topograph

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    return native.NativeEngine()


def test_graph_build_goldens_on_device(eng):
    assert A.check_topograph(eng) == []


def _rand_sets(rng, n, lo, hi, universe):
    sizes = rng.integers(lo, hi + 1, n)
    off = np.zeros(n + 1, np.int64)
    off[1:] = np.cumsum(sizes)
    ids = np.concatenate([rng.choice(universe, s, replace=False) for s in sizes]).astype(np.int32) \
        if off[-1] else np.zeros(0, np.int32)
    return ids, off


def test_selector_match_random_vs_oracle(eng):
    rng = np.random.default_rng(3)
    lab, lab_off = _rand_sets(rng, 1500, 0, 6, 40)
    sel, sel_off = _rand_sets(rng, 321, 0, 3, 40)
    got = eng.selector_match(lab, lab_off, sel, sel_off)
    assert np.array_equal(got, oracle.selector_match_ref(lab, lab_off, sel, sel_off))


def test_selector_match_1m_objects_bit_exact(eng):
    import torch
    rng = np.random.default_rng(4)
    D, S, U = 1_000_000, 200, 64
    lab, lab_off = _rand_sets(rng, D, 0, 8, U)
    sel, sel_off = _rand_sets(rng, S, 1, 3, U)

    def masks(ids, off):
        owner = np.repeat(np.arange(len(off) - 1), np.diff(off))
        m = np.zeros(len(off) - 1, np.uint64)
        np.bitwise_or.at(m, owner, np.left_shift(np.uint64(1), ids.astype(np.uint64)))
        return m

    om, sm = masks(lab, lab_off), masks(sel, sel_off)
    t0 = torch.cuda.Event(enable_timing=True)
    t1 = torch.cuda.Event(enable_timing=True)
    eng.selector_match(lab, lab_off, sel, sel_off)  # warm
    t0.record()
    got = eng.selector_match(lab, lab_off, sel, sel_off)
    t1.record()
    t1.synchronize()
    print(f"selector_match D={D} S={S}: {t0.elapsed_time(t1):.2f} ms incl. H2D/D2H")
    want = np.zeros_like(got)
    for s in range(S):
        hit = (om & sm[s]) == sm[s]
        want[:, s // 64] |= hit.astype(np.uint64) << np.uint64(s % 64)
    assert np.array_equal(got, want)
    assert 0 < int(np.count_nonzero(got)) < got.size


def test_substr_match_vs_python_in(eng):
    rng = random.Random(11)
    names = ["svc%d" % i for i in range(1000)] + ["a", "ab", "ü-db", "db"]
    keys = []
    for n in names:
        keys += [n, n + ".shop", n + ".shop.svc", n + ".shop.svc.cluster.local"]
    keys.append("")
    values = []
    for i in range(200_000):
        r = rng.random()
        n = rng.choice(names)
        if r < 0.4:
            values.append("http://%s.shop.svc.cluster.local:%d/x" % (n, rng.randint(1, 99999)))
        elif r < 0.6:
            values.append("%s,%s.shop" % (n, rng.choice(names)))
        elif r < 0.7:
            values.append("")
        elif r < 0.75:
            values.append("ünï " * rng.randint(1, 30) + n)
        else:
            values.append("plain-%d-%s" % (rng.randint(0, 10**6), "x" * rng.randint(0, 100)))
    values.append(" ".join(names))  # one long value holding every name
    got = topograph.substring_matches(eng, values, keys)
    n_pairs = 0
    for v, ks in enumerate(got):
        assert ks == sorted(set(ks))
        for k in ks:
            assert keys[k] in values[v]
        n_pairs += len(ks)
    for v in rng.sample(range(len(values)), 1500) + [len(values) - 1]:
        assert got[v] == [k for k, key in enumerate(keys) if key in values[v]], v
    assert n_pairs > len(values)
