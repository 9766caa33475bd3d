"""The C-ABI library: it loads without a GPU and exports every symbol include/krca.h declares;
host-only helpers (sizes, plans) are callable on CPU."""
import ctypes
import os
import re

import numpy as np

from conftest import ROOT
from krca import native


def header_symbols():
    with open(os.path.join(ROOT, "include", "krca.h")) as f:
        src = f.read()
    return sorted(set(re.findall(r"^\s*(?:int|int32_t|int64_t|uint64_t|float|const char\*)\s+(krca_\w+)\s*\(", src, re.M)))


def test_library_exports_every_header_symbol():
    lib = native.load_library()
    syms = header_symbols()
    assert len(syms) >= 15
    for s in syms:
        assert hasattr(lib, s), s
    assert set(syms) == set(native.SIGNATURES), "ctypes signatures out of sync with include/krca.h"


def test_version_and_host_helpers():
    lib = native.load_library()
    assert lib.krca_version() == 100
    assert lib.krca_log_index_size(0) > 0
    assert lib.krca_log_index_size(1 << 30) > lib.krca_log_index_size(1 << 20)
    assert lib.krca_topk_workspace_size(1 << 20, 10) > 0
    assert lib.krca_ppr_workspace_size(1000) >= 4 * 1000 * 8
    from krca.rca import NSLOT, slice_words
    assert lib.krca_ppr_nslot() == NSLOT  # send-slice layout shared by the kernels and krca/rca.py
    for n_max in (1, 2, 7, 1000, 999999):
        assert lib.krca_ppr_slice_words(n_max) == slice_words(n_max)
    assert lib.krca_ppr_ctl_size(1000) >= 12 * 1000  # long-row accumulators + tickets
    assert lib.krca_group_max_rank() == 6  # 64-byte slot records: first, counts, 6 ranks
    assert lib.krca_template_huge_ws_size(5000) >= 2 * 5000 * 12  # distinct-hash table of >= 2n slots


def test_ppr_plan_blocks_cover_rows():
    lib = native.load_library()
    rng = np.random.default_rng(0)
    deg = rng.integers(0, 40, 5000)
    deg[[7, 999]] = [5000, 2049]  # long rows -> chunked
    rp = np.zeros(len(deg) + 1, np.int64)
    np.cumsum(deg, out=rp[1:])
    n = lib.krca_ppr_plan_size(rp.ctypes.data_as(ctypes.c_void_p), len(deg))
    plan = np.zeros(n, np.int64)
    assert lib.krca_ppr_plan(rp.ctypes.data_as(ctypes.c_void_p), len(deg), plan.ctypes.data_as(ctypes.c_void_p), n) == 0
    covered = np.zeros(len(deg), np.int64)
    for rb, code, e0, e1 in plan.reshape(-1, 4):
        if code > 0:
            assert code - rb <= 256 and rp[code] - rp[rb] <= 2048
            assert (e0, e1) == (rp[rb], rp[code])
            covered[rb:code] += 1
        else:
            assert deg[rb] > 2048
            assert e0 == rp[rb] + 2048 * (-code) and e1 == min(rp[rb + 1], e0 + 2048)
            covered[rb] += (-code == 0)
    assert (covered == 1).all()


def test_no_cpu_fallback_without_device():
    import torch
    if torch.cuda.is_available():
        return
    try:
        native.NativeEngine()
    except native.KrcaError as e:
        assert "no CPU fallback" in str(e)
    else:
        raise AssertionError("NativeEngine must refuse to run without a HIP device")


def test_corr_shard_ranges_tile_aligned_and_cover():
    from krca.corr_dist import TB, corr_shard_range
    for P in (2, 255, 256, 257, 6000, 100_000, 1_000_000):
        for G in (1, 2, 3, 8):
            spans = [corr_shard_range(P, G, g) for g in range(G)]
            assert spans[0][0] == 0 and spans[-1][1] == P
            for (lo, hi, n_max), (lo2, _, _) in zip(spans, spans[1:]):
                assert hi == lo2 and n_max % TB == 0 and (lo % TB == 0 or lo == hi == P)
    lib = native.load_library()
    assert lib.krca_corr_shard_ws_size(100_000, 1440, 10, 12_544, 8) > lib.krca_corr_shard_ws_size(100_000, 1440, 10,
                                                                                                     0, 8)


def test_tuning_knobs_and_score_variant():
    """A/B knobs are read once at load and changed only through krca_tune_set; the scoring variant
    query reports the pipelined kernel at C4 and the per-row-descriptor form past 2^31 bytes."""
    lib = native.load_library()
    v = ctypes.c_int32(-1)
    assert lib.krca_tune_get(b"KRCA_SCORE_IMPL", ctypes.byref(v)) == 0 and v.value == 0
    assert lib.krca_tune_set(b"NO_SUCH_KNOB", 1) != 0
    assert b"NO_SUCH_KNOB" in lib.krca_last_error()
    assert native.SCORE_VARIANTS[lib.krca_rolling_score_variant(1_000_000, 8, 1440, 60)] == "pipe"
    assert native.SCORE_VARIANTS[lib.krca_rolling_score_variant(4_000_000, 8, 1440, 60)] == "pipe_rows"
    assert native.SCORE_VARIANTS[lib.krca_rolling_score_variant(1000, 8, 50, 60)] == "ring"    # T <= W
    assert native.SCORE_VARIANTS[lib.krca_rolling_score_variant(1000, 8, 500, 7)] == "reread"  # any W
    with native.tune(lib, KRCA_SCORE_IMPL=2):
        assert native.SCORE_VARIANTS[lib.krca_rolling_score_variant(1000, 8, 1440, 60)] == "ring_buf"
    with native.tune(lib, KRCA_SCORE_IMPL=5):
        assert native.SCORE_VARIANTS[lib.krca_rolling_score_variant(1_000_000, 8, 1440, 60)] == "lds"
        assert native.SCORE_VARIANTS[lib.krca_rolling_score_variant(1000, 8, 500, 30)] == "ring"  # W != 60
    with native.tune(lib, KRCA_SCORE_IMPL=4):
        assert native.SCORE_VARIANTS[lib.krca_rolling_score_variant(1000, 8, 1440, 60)] == "pipe_rows"
    assert lib.krca_tune_get(b"KRCA_SCORE_IMPL", ctypes.byref(v)) == 0 and v.value == 0  # restored


def test_ppr_pack_decodes_to_the_remapped_columns():
    """krca_ppr_pack (host): every edge of every block decodes to its remapped column, through the
    block's sorted distinct-column list (dictionary blocks) or directly (direct / long-row blocks)."""
    from krca import synth
    from krca.rca import remap_cols
    lib = native.load_library()
    vp = ctypes.c_void_p
    m = synth.make_graph(6000, n_edges=120_000, seed=2)
    rp, col = m.row_ptr.copy(), m.col.copy()
    # a long row (> 2048 callers) and a row with many distinct callers
    for n_max in (6000, 2500):
        n = lib.krca_ppr_plan_size(rp.ctypes.data_as(vp), len(rp) - 1)
        plan = np.zeros(n, np.int64)
        pk = np.zeros(len(col), np.int32)
        lane = np.zeros(lib.krca_ppr_lane_size(n), np.uint16)
        nd = lib.krca_ppr_pack(rp.ctypes.data_as(vp), col.ctypes.data_as(vp), len(rp) - 1, n_max,
                               plan.ctypes.data_as(vp), n, pk.ctypes.data_as(vp), lane.ctypes.data_as(vp))
        assert nd > 0.5 * (n // 4), nd  # most blocks of a service mesh are dictionary blocks
        want = remap_cols(col, n_max)
        got = np.full(len(col), -1, np.int64)
        for bi, (h, code, e0, e1) in enumerate(plan.reshape(-1, 4)):
            nu = int(h) >> 32
            if code > 0:  # lane words: (slot of the row holding edge 8t) << 8 | row-start bits
                rb = int(h) & 0xFFFFFFFF
                ne = int(e1 - e0)
                deg = np.diff(rp[rb:code + 1])
                slots = lane[bi * 512 + 256:bi * 512 + 256 + (code - rb)].astype(np.int64)
                # non-empty rows: consecutive slots in row order; rows without edges: slot 256
                assert np.array_equal(slots[deg > 0], np.arange(int((deg > 0).sum())))
                assert np.all(slots[deg == 0] == 256)
                holder = np.repeat(slots, deg)  # the slot of the row holding each edge
                starts = set((rp[rb:code][deg > 0] - e0).tolist())
                assert len(holder) == ne
                for t in range(0, (ne + 7) // 8):
                    li = int(lane[bi * 512 + t])
                    assert li >> 8 == holder[8 * t], (bi, t)
                    assert li & 0xFE == sum(1 << k for k in range(1, 8) if 8 * t + k in starts), (bi, t)
            if nu == 0:
                got[e0:e1] = pk[e0:e1]
                continue
            assert code > 0
            uniq = pk[e0:e0 + nu].astype(np.int64)
            assert np.all(np.diff(uniq) > 0)
            dw = ((e0 + nu + 3) & ~3) - e0
            words = pk[e0 + dw:e1].view(np.uint32)
            slots = np.stack([words & 0xFFFF, words >> 16], 1).reshape(-1)[:e1 - e0]
            assert slots.max() < nu
            got[e0:e1] = uniq[slots]
        assert np.array_equal(got, want)


def test_log_matcher_identity_matches_this_interpreter():
    """The DFA tables record the Unicode version they were generated under and the digest of the
    13 patterns; both must match this interpreter and krca/patterns.py (the reference declares
    Python >= 3.11, whose Unicode 14/15 tables may fold or classify non-ASCII differently)."""
    import unicodedata
    from krca import patterns
    lib = native.load_library()
    assert lib.krca_log_dfa_unicode().decode() == unicodedata.unidata_version
    assert int(lib.krca_log_dfa_digest()) == patterns.pattern_digest()
