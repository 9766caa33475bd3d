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
    return sorted(set(re.findall(r"^\s*(?:int|int32_t|int64_t|float|const char\*)\s+(krca_\w+)\s*\(", src, re.M)))


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
    from krca.rca import NSLOT
    assert lib.krca_ppr_nslot() == NSLOT  # send-slice layout shared by the kernels and krca/rca.py
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
    with native.tune(lib, KRCA_SCORE_IMPL=4):
        assert native.SCORE_VARIANTS[lib.krca_rolling_score_variant(1000, 8, 1440, 60)] == "pipe_rows"
    assert lib.krca_tune_get(b"KRCA_SCORE_IMPL", ctypes.byref(v)) == 0 and v.value == 0  # restored
