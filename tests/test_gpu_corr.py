"""a9 cross-pod Pearson correlation (krca_corr_prepare + krca_corr_topk) against the float64 oracle.

Tolerances ("1e-5 rel on reported r"): reported r within 1e-5 relative (plus
2e-6 absolute for |r| near 0) of float64; the top-k SET equals the oracle's wherever the oracle's
k-th and (k+1)-th |r| are more than 2e-4 apart (closer than that, either pod is a valid k-th);
|r| > tau counts exact (the device re-scores in float64 every pair whose fp16 screening value is
within krca_corr_eps(T) of tau; it works from the fp32 rows z32, so a pair within 1e-6 of tau may
land on either side against the float64 oracle); every certificate positive (pods whose first merge
cannot prove the set have all candidates re-scored), and every certified row matches exactly.
C3 (100k pods) is checked on EVERY row against a float64 torch reference on the device.
"""
import numpy as np
import pytest
import torch

import oracle
from krca import native, synth

pytestmark = pytest.mark.gpu
TAU = 0.5


@pytest.fixture(scope="module")
def eng():
    return native.NativeEngine()


def check_rows(res, z, rows, k, tau=TAU):
    eps = native.load_library().krca_corr_eps(z.shape[1])
    assert 9e-4 < eps < 2e-3
    oi, orr, oc, gap = oracle.corr_rows(z, rows, k, tau)
    gi, gv, gc, cert = res["idx"][rows], res["val"][rows], res["count"][rows], res["cert"][rows]
    # reported values: exact re-scoring of the reported partners
    rv = np.einsum("nt,nkt->nk", z[rows], z[gi])
    assert np.all(np.abs(gv - rv) <= 1e-5 * np.abs(rv) + 2e-6), np.max(np.abs(gv - rv))
    clear = gap > 2e-4
    for n in np.nonzero(clear)[0]:
        assert set(gi[n].tolist()) == set(oi[n].tolist()), (rows[n], gi[n], oi[n], gap[n])
    # descending |r| in the output
    assert np.all(np.diff(np.abs(gv), axis=1) <= 1e-6)
    # certified rows are exact (up to the fp32 rounding of z the device re-scores from: a
    # k-th / (k+1)-th pair closer than 1e-6 in float64 may swap)
    for n in np.nonzero((cert > 0) & (gap > 1e-6))[0]:
        assert set(gi[n].tolist()) == set(oi[n].tolist()), (rows[n], gap[n])
    Rn = z[rows] @ z.T
    Rn[np.arange(len(rows)), rows] = 0
    a = np.abs(Rn)
    lo, hi = (a > tau + 1e-6).sum(1), (a > tau - 1e-6).sum(1)
    assert np.all((gc >= lo) & (gc <= hi)), np.nonzero((gc < lo) | (gc > hi))[0][:10]
    assert np.all(cert > 0), np.nonzero(cert <= 0)[0][:10]
    return clear.mean(), (cert > 0).mean()


@pytest.mark.parametrize("P,T,group,k", [(6000, 1440, 20, 10), (130, 200, 7, 16), (257, 64, 0, 5), (2, 30, 0, 1),
                                         (1000, 100, 50, 10)])
def test_corr_full_vs_oracle(eng, P, T, group, k):
    x = synth.make_metrics(P, 2, T, seed=P + T, group_size=group)
    x[:, 3 % P, 0] = 42.0  # a flat series: r = 0 with everything
    if P > 20:
        x[:, 17, 0] = x[:, 5, 0]  # duplicate pods: r = 1, tie broken by index
        x[:, 18, 0] = x[:, 5, 0]
    res = eng.corr_topk(x, k=k, tau=TAU, channel=0)
    z = oracle.corr_standardize(x.numpy(), 0)
    clear, certified = check_rows(res, z, np.arange(P), k)
    if P > 20:
        assert res["idx"][5][:2].tolist() == [17, 18] and abs(res["val"][5][0] - 1) < 1e-6
        assert res["idx"][17][:2].tolist() == [5, 18]


def test_corr_channel_and_determinism(eng):
    x = synth.make_metrics(777, 3, 300, seed=9, group_size=10).cuda()
    a = eng.corr_topk(x, k=8, tau=0.3, channel=2)
    b = eng.corr_topk(x, k=8, tau=0.3, channel=2)
    for key in a:
        assert np.array_equal(a[key], b[key])
    z = oracle.corr_standardize(x.cpu().numpy(), 2)
    check_rows(a, z, np.arange(777), 8, 0.3)


def test_corr_c3_every_row(eng):
    """C3 (100k pods x 1440 steps, k = 10, tau = 0.5), all 100k rows against a float64 reference
    computed on the device with torch (z from the oracle's standardisation, R in 2048-row blocks)."""
    P, T, k = 100_000, 1440, 10
    x = synth.make_metrics(P, 1, T, seed=1, group_size=20, device="cuda")
    res = eng.corr_topk(x, k=k, tau=TAU)
    z = torch.from_numpy(oracle.corr_standardize(x.cpu().numpy(), 0)).cuda()
    del x
    gi = torch.from_numpy(res["idx"]).cuda().long()
    gv = torch.from_numpy(res["val"]).cuda().double()
    assert (res["cert"] > 0).all(), np.nonzero(res["cert"] <= 0)[0][:10]
    bad_set = bad_cnt = 0
    for r0 in range(0, P, 2048):
        r1 = min(P, r0 + 2048)
        R = z[r0:r1] @ z.T
        rr = torch.arange(r0, r1, device="cuda")
        R[rr - r0, rr] = 0.0
        a = R.abs()
        cnt = torch.from_numpy(res["count"][r0:r1]).cuda()
        lo, hi = (a > TAU + 1e-6).sum(1), (a > TAU - 1e-6).sum(1)
        bad_cnt += int(((cnt < lo) | (cnt > hi)).sum())
        # reported values: the exact r of the reported partners
        ex = torch.gather(R, 1, gi[r0:r1])
        assert torch.all((gv[r0:r1] - ex).abs() <= 1e-5 * ex.abs() + 2e-6)
        # the set: the k best by |r| (self excluded: -1), wherever the k-th is not tied within 1e-6
        a[rr - r0, rr] = -1.0
        top = torch.topk(a, k + 1, dim=1)
        gap = top.values[:, k - 1] - top.values[:, k]
        want = torch.sort(top.indices[:, :k], dim=1).values
        got = torch.sort(gi[r0:r1], dim=1).values
        bad_set += int(((want != got).any(1) & (gap > 1e-6)).sum())
        del R, a
    assert bad_cnt == 0 and bad_set == 0, (bad_cnt, bad_set)


def test_corr_sample_in_chunks(eng):
    """P * k past 16 * 64,000 grows the threshold sample beyond one chunk of 16 column blocks (the
    running top-k merge of corr_theta): every row still exact against a float64 device reference."""
    P, T, k = 140_000, 256, 10
    x = synth.make_metrics(P, 1, T, seed=4, group_size=20, device="cuda")
    res = eng.corr_topk(x, k=k, tau=TAU)
    z = torch.from_numpy(oracle.corr_standardize(x.cpu().numpy(), 0)).cuda()
    assert (res["cert"] > 0).all()
    gi = torch.from_numpy(res["idx"]).cuda().long()
    bad = 0
    for r0 in range(0, P, 4096):
        r1 = min(P, r0 + 4096)
        a = (z[r0:r1] @ z.T).abs()
        rr = torch.arange(r0, r1, device="cuda")
        a[rr - r0, rr] = -1.0
        top = torch.topk(a, k + 1, dim=1)
        gap = top.values[:, k - 1] - top.values[:, k]
        want = torch.sort(top.indices[:, :k], dim=1).values
        got = torch.sort(gi[r0:r1], dim=1).values
        bad += int(((want != got).any(1) & (gap > 1e-6)).sum())
        cnt = torch.from_numpy(res["count"][r0:r1]).cuda()
        a[rr - r0, rr] = 0.0
        lo, hi = (a > TAU + 1e-6).sum(1), (a > TAU - 1e-6).sum(1)
        bad += int(((cnt < lo) | (cnt > hi)).sum())
    assert bad == 0


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
    z = oracle.corr_standardize(x.numpy(), 0)
    check_rows(res, z, np.arange(P), k)
    # in-group pairs tie exactly (identical rows; the float64 oracle's BLAS breaks them by rounding
    # noise): the device keeps the k lowest indices of the group
    for p in range(1200):
        g0 = p // 600 * 600
        want = [q for q in range(g0, g0 + 600) if q != p][:k]
        assert res["idx"][p].tolist() == want, (p, res["idx"][p])
    assert np.all(res["count"][:1200] >= 599)


def test_corr_every_pair_at_tau(eng):
    """600 series x_i = u + v_i from orthogonal Hadamard rows: every in-group pair has r = 0.5 = tau
    exactly, so each in-group tile lists 65,536 pairs within eps of tau (past the 8,191 a tile ranks:
    the rest take one global slot each) and the lists pass their capacity.  Counts of the other pairs
    exact, in-group pairs (within 1e-6 of tau) on either side; every row certified."""
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
    z = oracle.corr_standardize(x.numpy(), 0)
    check_rows(res, z, np.arange(G + R), 10)
    assert np.all(res["count"][:G] <= G - 1 + R)


def test_corr_rejects_bad_k(eng):
    x = torch.rand(50, 10, 1)
    with pytest.raises(native.KrcaError):
        eng.corr_topk(x, k=17)
    with pytest.raises(native.KrcaError):
        eng.corr_topk(x, k=10)  # k must be < P


@pytest.mark.parametrize("P,T,G", [(6000, 1440, 2), (6000, 1440, 3), (1000, 100, 4), (300, 64, 2)])
def test_corr_sharded_path_emulated_on_one_gpu(eng, P, T, G):
    """The pod-sharded correlation (krca/corr_dist.py: G super-tile shares of the triangle, one
    all-to-all of candidates by owner) with the collectives done by copies: every output equals
    the single-device run (same screening products, same candidate sets, same merge)."""
    from krca.corr_dist import run_emulated
    x = synth.make_metrics(P, 2, T, seed=P + G, group_size=20).cuda()
    x[:, 3, 0] = 42.0  # a flat series
    ref = eng.corr_topk(x, k=10, tau=TAU, channel=0)
    got = run_emulated(eng, x, P, T, 10, TAU, G, channel=0)
    for key in ("idx", "val", "count", "cert"):
        assert np.array_equal(got[key], ref[key]), key
