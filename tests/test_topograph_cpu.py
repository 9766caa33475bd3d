"""f2 service-graph construction on CPU: the agents' host replay with the oracle
engine against the reference's graphs, and the interning / packing of krca/topograph.py against
the reference's own Python expressions on hazard inputs (ref:agents/topology_agent.py:133,257,
ref:agents/resource_analyzer.py:851)."""
import random

import numpy as np

import agent_cases as A
import oracle
from oracle_engine import OracleEngine

from krca import topograph

ENG = OracleEngine()


def test_graph_build_matches_reference_goldens():
    assert A.check_topograph(ENG) == []


def test_host_loop_matches_reference_goldens():
    assert A.check_topograph(ENG, force_host=True) == []


HAZARD_VALUES = [1, 1.0, True, 0, False, "1", "a", "", None, float("nan"), [1], (1,), "ü", 2]


def _rand_dict(rng, n):
    return {rng.choice(["a", "b", 1, True, "c"]): rng.choice(HAZARD_VALUES) for _ in range(n)}


def _bits_to_sets(bits, S):
    return [set(r.tolist()) for r in topograph.match_rows(bits, S)]


def test_selector_interning_matches_itemsview_and_eq_semantics():
    rng = random.Random(5)
    nan = float("nan")
    objs = [_rand_dict(rng, rng.randint(0, 4)) for _ in range(150)] + [{"a": nan}, {}]
    sels = [_rand_dict(rng, rng.randint(0, 2)) for _ in range(70)] + [{"a": nan}, {}]
    objs[-2]["a"] = sels[-2]["a"]  # the same NaN object: ItemsView matches it (identity), == does not
    for identity in (True, False):
        bits = topograph.selector_bits(ENG, [o.items() for o in objs], [s.items() for s in sels], identity)
        got = _bits_to_sets(bits, len(sels))
        for d, o in enumerate(objs):
            if identity:
                want = {s for s, sel in enumerate(sels) if all(it in o.items() for it in sel.items())}
            else:
                want = {s for s, sel in enumerate(sels) if all(k in o and o[k] == v for k, v in sel.items())}
            assert got[d] == want, (identity, d, o)
    cols = topograph.match_cols(topograph.selector_bits(ENG, [o.items() for o in objs], [s.items() for s in sels]),
                                len(sels))
    rows = _bits_to_sets(topograph.selector_bits(ENG, [o.items() for o in objs], [s.items() for s in sels]), len(sels))
    for s in range(len(sels)):
        assert cols[s] == sorted(d for d in range(len(objs)) if s in rows[d])


def test_substring_matches_equal_python_in():
    rng = random.Random(9)
    alphabet = ["a", "b", ".", "ü", "é", " ", "x", "svc", "\ud800"]
    keys = ["", "a", "ab", "a.b", "ü", "üé", "svc", "b.svc", "aaaa", "\ud800", "xx" * 20] + \
           ["".join(rng.choice(alphabet) for _ in range(rng.randint(1, 5))) for _ in range(40)]
    values = ["", "a", "aaaaaaa"] + ["".join(rng.choice(alphabet) for _ in range(rng.randint(0, 30)))
                                     for _ in range(300)] + ["xx" * 25]
    got = topograph.substring_matches(ENG, values, keys)
    for v, val in enumerate(values):
        assert got[v] == [k for k, key in enumerate(keys) if key in val], (v, val)


def test_oracle_kernel_semantics_small():
    lab = np.array([0, 1, 2, 1], np.int32)
    lab_off = np.array([0, 3, 4, 4], np.int64)
    sel = np.array([1, 0, 2, 3], np.int32)
    sel_off = np.array([0, 1, 3, 3, 4], np.int64)
    bits = oracle.selector_match_ref(lab, lab_off, sel, sel_off)
    assert bits.tolist() == [[0b0111], [0b0101], [0b0100]]
    assert oracle.substr_match_ref(b"abcab", [0, 5], b"abzc", [0, 2, 3, 4]).tolist() == [0, 2]
