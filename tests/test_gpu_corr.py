"""a9 cross-pod Pearson correlation (krca_corr_prepare + krca_corr_topk) against the oracle.

The oracle (oracle/krca_oracle.c krco_corr_z32) restates krca_corr_prepare bit for bit: the
standardized fp32 rows z32.  On those rows r(p, q) = sum_t z32[p,t] z32[q,t] in float64 (every product
exact; two summation orders differ by <= T 2^-53 ~ 1.6e-13), and the device's outputs are checked
against that definition:
- z32 / mean / scale: bit-identical to the twin;
- |r| > tau counts: EXACT for every pod, except partners within 1e-12 of tau (where another float64
  summation order may land on the other side): those are counted and printed, and the device count
  must lie within them;
- the top-k set: exact wherever the k-th and (k+1)-th |r| are more than 1e-12 apart;
- reported r: the float32 rounding of the float64 value (1.2e-7 relative);
- every certificate positive.
C3 (100k pods) is checked on EVERY row, and a 1M-pod run (C4's correlation half, tau = 0.5) on 4096
sampled rows, both against float64 references on the device built from the twin's z32.
"""
import numpy as np
import pytest
import torch

import oracle
from krca import native, synth

pytestmark = pytest.mark.gpu
TAU = 0.5
BAND = 1e-12  # float64 summation-order band around tau
OLD_BAND = 1e-6  # the round-2 tolerance (fp32 vs float64 standardisation), reported for comparison


@pytest.fixture(scope="module")
def eng():
    return native.NativeEngine()


def twin_z(x, channel=0):
    x = x.cpu().numpy() if hasattr(x, "cpu") else np.asarray(x)
    return oracle.c_corr_z32(x, channel)[0]


def check_rows(res, z32, rows, k, tau=TAU):
    """Host check of `rows` against the twin rows z32 (float64 products via BLAS)."""
    z = z32.astype(np.float64)
    gi, gv, gc, cert = res["idx"][rows], res["val"][rows], res["count"][rows], res["cert"][rows]
    R = z[rows] @ z.T
    R[np.arange(len(rows)), rows] = 0.0
    a = np.abs(R)
    # reported values: float32 of the exact r of the reported partners
    rv = np.take_along_axis(R, gi.astype(np.int64), axis=1)
    assert np.all(np.abs(gv - rv) <= 1.2e-7 * np.abs(rv) + 1e-12), np.max(np.abs(gv - rv))
    assert np.all(np.diff(np.abs(gv.astype(np.float64)), axis=1) <= 1.2e-7)
    # counts: exact outside the float64 band
    lo, hi = (a > tau + BAND).sum(1), (a > tau - BAND).sum(1)
    assert np.all((gc >= lo) & (gc <= hi)), np.nonzero((gc < lo) | (gc > hi))[0][:10]
    banded = int((hi - lo).sum())
    old = int(((a > tau - OLD_BAND).sum(1) - (a > tau + OLD_BAND).sum(1)).sum())
    # the set: the k best |r| (self excluded), wherever the k-th is not tied within BAND
    a[np.arange(len(rows)), rows] = -1.0
    kk = min(k + 1, z.shape[0] - 1)
    for n in range(len(rows)):
        part = np.argpartition(-a[n], kk - 1)[:kk]
        o = part[np.lexsort((part, -a[n][part]))]
        gap = a[n][o[k - 1]] - (a[n][o[k]] if len(o) > k else -1.0)
        if gap > BAND:
            assert set(gi[n].tolist()) == set(o[:k].tolist()), (rows[n], gi[n], o[:k], gap)
    assert np.all(cert > 0), np.nonzero(cert <= 0)[0][:10]
    print(f"rows {len(rows)}: pairs within {BAND:g} of tau {banded}, within {OLD_BAND:g} {old}")
    return banded, old


def device_check(res, z32d, rows_iter, k, tau=TAU, block=2048):
    """Device check (float64 torch) of the rows in rows_iter (arrays of pod ids) against the twin
    rows z32d (float64 on the device).  Returns (banded pairs, pairs within OLD_BAND, bad)."""
    gi_all = torch.from_numpy(res["idx"]).to(z32d.device).long()
    gv_all = torch.from_numpy(res["val"]).to(z32d.device).double()
    cnt_all = torch.from_numpy(res["count"]).to(z32d.device)
    banded = old = bad_cnt = bad_set = bad_val = 0
    for rows in rows_iter:
        rr = torch.as_tensor(rows, device=z32d.device).long()
        R = z32d[rr] @ z32d.T
        R[torch.arange(len(rr), device=R.device), rr] = 0.0
        a = R.abs()
        cnt = cnt_all[rr]
        lo, hi = (a > tau + BAND).sum(1), (a > tau - BAND).sum(1)
        bad_cnt += int(((cnt < lo) | (cnt > hi)).sum())
        banded += int((hi - lo).sum())
        old += int(((a > tau - OLD_BAND).sum(1) - (a > tau + OLD_BAND).sum(1)).sum())
        gi = gi_all[rr]
        ex = torch.gather(R, 1, gi)
        bad_val += int(((gv_all[rr] - ex).abs() > 1.2e-7 * ex.abs() + 1e-12).sum())
        a[torch.arange(len(rr), device=R.device), rr] = -1.0
        top = torch.topk(a, k + 1, dim=1)
        gap = top.values[:, k - 1] - top.values[:, k]
        want = torch.sort(top.indices[:, :k], dim=1).values
        got = torch.sort(gi, dim=1).values
        bad_set += int(((want != got).any(1) & (gap > BAND)).sum())
        del R, a
    return banded, old, (bad_cnt, bad_set, bad_val)


def test_corr_prepare_matches_twin(eng):
    """krca_corr_prepare's z32, mean and scale are the C twin's bits (flat series included)."""
    x = synth.make_metrics(3000, 3, 1440, seed=21, group_size=20)
    x[:, 7, 1] = 55.0
    for ch in (0, 1):
        z = eng.corr_prepare_device(x.cuda(), ch)
        z32, mean, scale = oracle.c_corr_z32(x.numpy(), ch)
        assert np.array_equal(z["mean"].cpu().numpy().view(np.uint32), mean.view(np.uint32))
        assert np.array_equal(z["scale"].cpu().numpy().view(np.uint32), scale.view(np.uint32))
        assert np.array_equal(z["z32"].cpu().numpy().view(np.uint32), z32.view(np.uint32))


@pytest.mark.parametrize("P,T,group,k", [(6000, 1440, 20, 10), (130, 200, 7, 16), (257, 64, 0, 5), (2, 30, 0, 1),
                                         (1000, 100, 50, 10), (60, 3, 0, 4), (33, 5, 0, 7), (300, 17, 0, 9)])
def test_corr_full_vs_oracle(eng, P, T, group, k):
    x = synth.make_metrics(P, 2, T, seed=P + T, group_size=group)
    x[:, 3 % P, 0] = 42.0  # a flat series: r = 0 with everything
    if P > 20:
        x[:, 17, 0] = x[:, 5, 0]  # duplicate pods: r = 1, tie broken by index
        x[:, 18, 0] = x[:, 5, 0]
    res = eng.corr_topk(x, k=k, tau=TAU, channel=0)
    check_rows(res, twin_z(x, 0), np.arange(P), k)
    if P > 20:
        assert res["idx"][5][:2].tolist() == [17, 18] and abs(res["val"][5][0] - 1) < 1e-6
        assert res["idx"][17][:2].tolist() == [5, 18]


def test_corr_channel_and_determinism(eng):
    x = synth.make_metrics(777, 3, 300, seed=9, group_size=10).cuda()
    a = eng.corr_topk(x, k=8, tau=0.3, channel=2)
    b = eng.corr_topk(x, k=8, tau=0.3, channel=2)
    for key in a:
        assert np.array_equal(a[key], b[key])
    check_rows(a, twin_z(x, 2), np.arange(777), 8, 0.3)


def test_corr_c3_every_row(eng):
    """C3 (100k pods x 1440 steps, k = 10, tau = 0.5): every one of the 100k rows against a float64
    reference on the device built from the twin's z32 — counts exact outside the 1e-12 band."""
    P, T, k = 100_000, 1440, 10
    x = synth.make_metrics(P, 1, T, seed=1, group_size=20, device="cuda")
    res = eng.corr_topk(x, k=k, tau=TAU)
    z32 = twin_z(x)
    del x
    assert (res["cert"] > 0).all(), np.nonzero(res["cert"] <= 0)[0][:10]
    z = torch.from_numpy(z32).cuda().double()
    banded, old, bad = device_check(res, z, (np.arange(r0, min(P, r0 + 2048)) for r0 in range(0, P, 2048)), k)
    print(f"C3: (pod, partner) pairs within {BAND:g} of tau: {banded}; within the round-2 band {OLD_BAND:g}: {old}")
    assert bad == (0, 0, 0), bad
    assert banded <= 1000


@pytest.mark.parametrize("T,k,tau", [(1001, 10, 0.5), (1437, 16, 0.6)])
def test_corr_odd_steps_every_row(eng, T, k, tau):
    """T not a multiple of 4 (the projection kernel's scalar-load form, corr_proj<false>) and of 64 (a
    partial last chunk), at 30k pods: every row against the float64 reference on the device, so the
    projection bound, the packed deep merge and the certificates are exercised away from T = 1440."""
    P = 30_000
    x = synth.make_metrics(P, 1, T, seed=T, group_size=20, device="cuda")
    res = eng.corr_topk(x, k=k, tau=tau)
    z32 = twin_z(x)
    del x
    assert (res["cert"] > 0).all(), np.nonzero(res["cert"] <= 0)[0][:10]
    z = torch.from_numpy(z32).cuda().double()
    _, _, bad = device_check(res, z, (np.arange(r0, min(P, r0 + 2048)) for r0 in range(0, P, 2048)), k, tau)
    assert bad == (0, 0, 0), bad


@pytest.mark.parametrize("tau,k", [(0.3, 1), (0.7, 8), (0.9, 12), (0.123456789, 5), (0.95, 16)])
def test_corr_tau_not_float32_every_row(eng, tau, k):
    """tau values a float32 cannot hold (0.3, 0.7, 0.9, ...) and the smallest / largest k: every row of
    a 20k-pod run against the float64 reference on the device (the counts compare the float64 r with
    the float64 tau; a float tau missed pairs just above it, R8c)."""
    P, T = 20_000, 500
    x = synth.make_metrics(P, 1, T, seed=int(tau * 1000) + k, group_size=20, device="cuda")
    res = eng.corr_topk(x, k=k, tau=tau)
    z32 = twin_z(x)
    del x
    assert (res["cert"] > 0).all(), np.nonzero(res["cert"] <= 0)[0][:10]
    z = torch.from_numpy(z32).cuda().double()
    _, _, bad = device_check(res, z, (np.arange(r0, min(P, r0 + 2048)) for r0 in range(0, P, 2048)), k, tau)
    assert bad == (0, 0, 0), bad


def test_corr_odd_sample_self_products(eng):
    """An odd threshold sample (P = 120k, k = 10: 19 blocks of 128 pods) leaves the second half of
    its last 256-block unscanned, and that block is nobody's own block either: the self products
    of its pods (2432 .. 2559) must still be recorded -- a missed one read a stale value and could
    turn a live pod "flat" (top-k = the lowest indices).  A flat pod inside that half (2500) must
    still be handled as flat; the whole half and 512 random rows are checked exactly."""
    P, T, k = 120_000, 256, 10
    x = synth.make_metrics(P, 1, T, seed=5, group_size=20, device="cuda")
    x[:, 2500, 0] = 42.0
    res = eng.corr_topk(x, k=k, tau=TAU)
    z = torch.from_numpy(twin_z(x)).cuda().double()
    del x
    assert (res["cert"] > 0).all(), np.nonzero(res["cert"] <= 0)[0][:10]
    assert res["idx"][2500].tolist() == list(range(k)) and not res["val"][2500].any()
    rows = np.concatenate([np.arange(2432, 2560), np.random.default_rng(1).choice(P, 512, replace=False)])
    _, _, bad = device_check(res, z, [rows], k)
    assert bad == (0, 0, 0), bad


def test_corr_batches_and_full_lists_identical(eng):
    """The main pass in many batches (KRCA_CORR_BATCH) and with ambiguous lists that fill at once
    (KRCA_CORR_AMB_TILE = 0: every tile decides its pairs in place; 8: mixed), and the list re-scored
    pair by pair instead of grouped by row pod (KRCA_CORR_RS_GROUP = 0), or grouped from the fp32
    partner rows instead of the int16 ones (KRCA_CORR_RS_Q16 = 0), give the same outputs bit for
    bit as the default run (the same float64 re-score in the tile and in either list kernel)."""
    P, T, k = 40_000, 1440, 10
    x = synth.make_metrics(P, 1, T, seed=3, group_size=20, device="cuda")
    ref = eng.corr_topk(x, k=k, tau=TAU)
    lib = eng.lib
    try:
        # (KRCA_CORR_SIDE: the re-scores beside the next batch, after each batch, or after each but the last)
        # (KRCA_CORR_RS_Q16 = 0: the grouped re-score reads the fp32 partner rows, not the int16 ones)
        for batch, per_tile, group, side, q16 in ((4, -1, 1, 0, 1), (0, 0, 1, 0, 1), (3, 8, 1, 0, 1), (0, -1, 0, 0, 1),
                                                  (4, -1, 0, 0, 1), (4, -1, 1, 1, 1), (4, -1, 1, 2, 1), (3, 8, 1, 2, 1),
                                                  (0, -1, 1, 0, 0), (4, -1, 1, 0, 0)):
            assert lib.krca_tune_set(b"KRCA_CORR_BATCH", batch) == 0
            assert lib.krca_tune_set(b"KRCA_CORR_AMB_TILE", per_tile) == 0
            assert lib.krca_tune_set(b"KRCA_CORR_RS_GROUP", group) == 0
            assert lib.krca_tune_set(b"KRCA_CORR_SIDE", side) == 0
            assert lib.krca_tune_set(b"KRCA_CORR_RS_Q16", q16) == 0
            got = eng.corr_topk(x, k=k, tau=TAU)
            for key in ref:
                assert np.array_equal(got[key], ref[key]), (batch, per_tile, group, side, q16, key)
    finally:
        lib.krca_tune_set(b"KRCA_CORR_RS_Q16", 1)
        lib.krca_tune_set(b"KRCA_CORR_BATCH", 0)
        lib.krca_tune_set(b"KRCA_CORR_AMB_TILE", -1)
        lib.krca_tune_set(b"KRCA_CORR_RS_GROUP", 1)
        lib.krca_tune_set(b"KRCA_CORR_SIDE", 0)
    # performance knobs that must not change a result: the grouped re-score's grid, and how many
    # candidates past the k-th the merge re-scores (fewer: more pods take the deep merge; the
    # certificate margins may differ, the sets, values and counts not)
    # (KRCA_CORR_PROJ = 0 / 1: the grouped re-score never with the projection bound / only when the
    # main pass runs in several batches -- the default uses it always; counts must not move)
    # (KRCA_CORR_PERSIST = 1: persistent main-pass workgroups instead of one per tile)
    for knob, val in (("KRCA_CORR_RSG_GRID", 256), ("KRCA_CORR_KM_EXTRA", 2), ("KRCA_CORR_PROJ", 0),
                      ("KRCA_CORR_PROJ", 1), ("KRCA_CORR_PERSIST", 1)):
        with native.tune(lib, **{knob: val}):
            got = eng.corr_topk(x, k=k, tau=TAU)
        for key in ("idx", "val", "count"):
            assert np.array_equal(got[key], ref[key]), (knob, val, key)
        assert (got["cert"] > 0).all(), (knob, val)
    z = torch.from_numpy(twin_z(x)).cuda().double()
    rows = np.random.default_rng(0).choice(P, 2048, replace=False)
    _, _, bad = device_check(ref, z, [rows], k)
    assert bad == (0, 0, 0), bad


def test_corr_c4_1m_pods(eng):
    """C4's correlation half on one GPU: 1M pods x 1440 steps, k = 10, C3's tau = 0.5 (~6e8 pairs
    within eps of tau: the main pass runs in batches, their ambiguous lists re-scored in turn).
    4096 sampled rows against a float64 device reference on the twin's z32: sets, values and
    counts exact; every row certified."""
    import time
    P, T, k = 1_000_000, 1440, 10
    x = synth.make_metrics(P, 1, T, seed=2, group_size=20, device="cuda")
    eng.corr_topk(x[:, :4096], k=k, tau=TAU)  # warm the kernels
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = eng.corr_topk(x, k=k, tau=TAU)
    dt = time.perf_counter() - t0
    print(f"1M pods tau={TAU}: {dt:.3f} s (incl. result copy)")
    z32 = twin_z(x)
    del x
    torch.cuda.empty_cache()
    assert (res["cert"] > 0).all(), np.nonzero(res["cert"] <= 0)[0][:10]
    z = torch.from_numpy(z32).cuda().double()
    del z32
    rows = np.sort(np.random.default_rng(7).choice(P, 4096, replace=False))
    banded, old, bad = device_check(res, z, (rows[i:i + 512] for i in range(0, len(rows), 512)), k)
    print(f"1M sample: pairs within {BAND:g} of tau {banded}, within {OLD_BAND:g} {old}")
    assert bad == (0, 0, 0), bad


def test_corr_sample_in_chunks(eng):
    """P * k past 16 * 64,000 grows the threshold sample beyond one chunk of 16 column blocks (the
    running top-k merge of corr_theta): every row still exact against a float64 device reference."""
    P, T, k = 140_000, 256, 10
    x = synth.make_metrics(P, 1, T, seed=4, group_size=20, device="cuda")
    res = eng.corr_topk(x, k=k, tau=TAU)
    z = torch.from_numpy(twin_z(x)).cuda().double()
    assert (res["cert"] > 0).all()
    _, _, bad = device_check(res, z, (np.arange(r0, min(P, r0 + 4096)) for r0 in range(0, P, 4096)), k)
    assert bad == (0, 0, 0), bad


def test_corr_list_overflow_refill(eng):
    """Two groups of 600 identical series: every in-group pair is a candidate of both pods, so the
    LDS lists of the in-group tiles pass their capacity and those tiles run again for the next
    windows of list slots.  Every row equals the oracle (ties at r = 1 go to the lower index)."""
    P, T, k = 1800, 256, 10
    base = synth.make_metrics(P, 1, T, seed=11, group_size=0)
    x = base.clone()
    for g0 in (0, 600):
        x[:, g0:g0 + 600, 0] = base[:, g0:g0 + 1, 0]
    res = eng.corr_topk(x, k=k, tau=TAU)
    check_rows(res, twin_z(x), np.arange(P), k)
    # in-group pairs tie exactly (identical rows; the float64 oracle's BLAS breaks them by rounding
    # noise): the device keeps the k lowest indices of the group
    for p in range(1200):
        g0 = p // 600 * 600
        want = [q for q in range(g0, g0 + 600) if q != p][:k]
        assert res["idx"][p].tolist() == want, (p, res["idx"][p])
    assert np.all(res["count"][:1200] >= 599)


def test_corr_candidate_buffer_overflow(eng):
    """Candidate buffers that overflow (KRCA_CORR_CAPC = 128 of the krca_corr_cand_cap() slots: a
    few hundred pods of this mesh pass it) take phi2 from the entries that landed, the rectangle pass over their
    rows and the second merge -- on one device and through the sharded path's pack / all-to-all /
    unpack (emulated, G = 2).  Partners, values and counts equal the run whose buffers hold every
    candidate; every row certified."""
    from krca.corr_dist import run_emulated
    P, T, k = 20_000, 720, 10
    x = synth.make_metrics(P, 1, T, seed=8, group_size=20, device="cuda")
    ref = eng.corr_topk(x, k=k, tau=TAU)
    cap = eng.lib.krca_corr_cand_cap()
    raw = eng._ws["corr_cand"].view(torch.int32)[2 * P * cap: 2 * P * cap + P].cpu().numpy()
    assert (raw > 128).sum() > P // 100, (raw > 128).sum()
    lib = eng.lib
    try:
        assert lib.krca_tune_set(b"KRCA_CORR_CAPC", 128) == 0
        got = eng.corr_topk(x, k=k, tau=TAU)
        emu = run_emulated(eng, x, P, T, k, TAU, 2)
    finally:
        lib.krca_tune_set(b"KRCA_CORR_CAPC", 0)
    for res in (got, emu):
        for key in ("idx", "val", "count"):
            assert np.array_equal(res[key], ref[key]), key
        assert (res["cert"] > 0).all(), np.nonzero(res["cert"] <= 0)[0][:10]


def test_corr_every_pair_at_tau(eng):
    """600 series x_i = u + v_i from orthogonal Hadamard rows: every in-group pair has r = 0.5 = tau
    (up to the fp32 rounding of the rows), so each in-group tile has 65,536 pairs within eps of tau:
    its LDS lists pass their capacity (the tile runs again per window) and the batch's ambiguous list
    (32,768 entries at this size) fills, so the remaining tiles decide their pairs in place.  Counts
    exact; every row certified."""
    T, G, R = 1024, 600, 100
    H = np.array([[1.0]])
    while H.shape[0] < T:
        H = np.block([[H, H], [H, -H]])
    rng = np.random.default_rng(5)
    x = np.empty((T, G + R, 1), np.float32)
    x[:, :G, 0] = (H[1][:, None] + H[2:G + 2].T) * 3.0 + 10.0
    x[:, G:, 0] = np.cumsum(rng.standard_normal((T, R)), axis=0)
    x = torch.from_numpy(x)
    res = eng.corr_topk(x, k=10, tau=TAU)
    check_rows(res, twin_z(x), np.arange(G + R), 10)
    assert np.all(res["count"][:G] <= G - 1 + R)


def test_corr_rejects_bad_k(eng):
    x = torch.rand(50, 10, 1)
    with pytest.raises(native.KrcaError):
        eng.corr_topk(x, k=17)
    with pytest.raises(native.KrcaError):
        eng.corr_topk(x, k=10)  # k must be < P


@pytest.mark.parametrize("P,T,G", [(6000, 1440, 2), (6000, 1440, 3), (1000, 100, 4), (300, 64, 2), (100_000, 1440, 2)])
def test_corr_sharded_path_emulated_on_one_gpu(eng, P, T, G):
    """The pod-sharded correlation (krca/corr_dist.py: G super-tile shares of the triangle, one
    all-to-all of candidates by owner) with the collectives done by copies: every output equals
    the single-device run (same screening products, same candidate sets, same merge).  The one
    exception is the certificate MARGIN of a pod whose 2,048-entry candidate buffer overflowed: its
    second threshold phi2 is the k-th best of the candidates that landed first, and arrival order
    differs between one device and the all-to-all.  Its partners, values and count are still
    identical and both certificates positive."""
    from krca.corr_dist import run_emulated
    x = synth.make_metrics(P, 2, T, seed=P + G, group_size=20, device="cuda")
    x[:, 3, 0] = 42.0  # a flat series
    ref = eng.corr_topk(x, k=10, tau=TAU, channel=0)
    got = run_emulated(eng, x, P, T, 10, TAU, G, channel=0)
    for key in ("idx", "val", "count"):
        assert np.array_equal(got[key], ref[key]), key
    assert (got["cert"] > 0).all() and (ref["cert"] > 0).all()
    diff = int((got["cert"] != ref["cert"]).sum())
    print(f"P={P} G={G}: certificate margins differing (overflowed buffers): {diff}")
    assert diff <= P // 100, diff
