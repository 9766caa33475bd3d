"""The oracle against the scale goldens of tests/golden/capture_scale.py (networkx 3.4.2 PageRank
on 2k / 20k-node meshes; the C2-mini fixture of SURVEY.md §8c golden #7), and the one ranking
definition (krca.rca.Config) shared by the bench path and Coordinator.ranked_root_causes."""
import os

import numpy as np
import pytest

import oracle
from conftest import GOLDEN

import c2mini as C  # tests/golden/c2mini.py (conftest puts tests/ on the path; golden/ below)
from krca.rca import RANKING, Config


def _csr(edges, n):
    src, dst = edges[:, 0].astype(np.int64), edges[:, 1].astype(np.int64)
    o = np.lexsort((src, dst))
    rp = np.zeros(n + 1, np.int64)
    np.cumsum(np.bincount(dst, minlength=n), out=rp[1:])
    return rp, src[o].astype(np.int32), np.bincount(src, minlength=n).astype(np.int32)


@pytest.fixture(scope="module")
def meshes():
    return np.load(os.path.join(GOLDEN, "ppr_nx_meshes.npz"))


def test_ranking_definition_is_shared():
    """bench.py, RcaStep, StreamingRCA and the Coordinator all default to krca.rca.RANKING."""
    import inspect
    from krca.agents.coordinator import Coordinator
    from krca.stream import StreamingRCA
    assert (RANKING.alpha, RANKING.seed_floor, RANKING.iters, RANKING.tol, RANKING.k, RANKING.key) == (
        0.5, None, 30, 1e-10, 10, "explained")  # iters: the cap of networkx's L1 stop rule
    # the scale-aware floor: 4 up to ~16k series, the null max of P*M series beyond (C2 4.369, C4 5.286)
    assert RANKING.floor(2000, 8) == 4.003 and RANKING.floor(1000, 8) == 4.0
    assert RANKING.floor(10_000, 8) == 4.369 and RANKING.floor(1_000_000, 8) == 5.286
    c = Coordinator(None, engine=object())
    assert c.rank_config is RANKING
    assert (c.metrics_agent.window, c.metrics_agent.z_threshold) == (RANKING.window, RANKING.z_threshold)
    assert "cfg or Config()" in inspect.getsource(StreamingRCA.__init__)
    import bench
    a = bench.parse([])
    assert (a.alpha, a.seed_floor, a.iters, a.window) == (RANKING.alpha, RANKING.seed_floor, RANKING.iters,
                                                          RANKING.window)


@pytest.mark.parametrize("name", ["m2k", "m20k"])
def test_oracle_ppr_matches_networkx_meshes(meshes, name):
    """C twin (30 fixed iterations, alpha 0.5, floor 4) = networkx's converged PageRank within
    1e-5 relative on every node holding >= 1e-12 of the mass; top-10 by r*p identical."""
    e, s = meshes[f"{name}_edges"], meshes[f"{name}_seed"]
    n = len(s)
    rp, col, od = _csr(e, n)
    rf, r, it, q = oracle.c_ppr(rp, col, od, s, RANKING.alpha, RANKING.iters, 0.0, 4.0,  # the floor the goldens were captured at
                                return_q=True)
    x = r.astype(np.float64) / 2.0 ** 60
    ref = meshes[f"{name}_rank"]
    big = ref >= 1e-12
    assert np.max(np.abs(x[big] - ref[big]) / ref[big]) < 1e-5
    assert np.max(np.abs(x[~big] - ref[~big])) < 1e-12
    idx, _ = oracle.topk_ref(oracle.c_rca_key(r, q), 10)
    assert idx.tolist() == meshes[f"{name}_top10"].tolist()
    # the networkx defaults (alpha 0.85, raw seeds as personalization), iterated to convergence
    rf, r85, it = oracle.c_ppr(rp, col, od, s, 0.85, 500, 1e-13, 0.0)
    x85 = r85.astype(np.float64) / 2.0 ** 60
    ref85 = meshes[f"{name}_rank_a085"]
    assert np.max(np.abs(x85 - ref85) / ref85) < 1e-5


def test_c2mini_inputs_reproduce():
    g = np.load(os.path.join(GOLDEN, "c2mini.npz"))
    e, x, blob, off = C.inputs()
    assert C.sha(e, x, off) == str(g["sha"]), "numpy changed the C2-mini input streams"
    assert np.array_equal(e, g["edges"]) and len(e) == C.N_EDGES and x.shape == (C.T, C.P, C.M)


def test_c2mini_oracle_outputs():
    g = np.load(os.path.join(GOLDEN, "c2mini.npz"))
    e, x, blob, off = C.inputs()
    sc = oracle.c_rolling_score(x, C.W)
    for k in ("z_last", "score", "n_exceed", "flags"):
        assert np.array_equal(sc[k], g[k]), k
    assert np.allclose(sc["z_last"], g["z_last_f64"], rtol=1e-5, atol=1e-5)
    assert np.array_equal(sc["n_exceed"], g["n_exceed_f64"])  # no sample within rounding of |z| = 3
    # a10 under the ranking definition, against networkx
    rp, col, od = _csr(e, C.P)
    rf, r, it, q = oracle.c_ppr(rp, col, od, g["score"], RANKING.alpha, RANKING.iters, 0.0, 4.0,
                                return_q=True)
    xr = r.astype(np.float64) / 2.0 ** 60
    ref = g["ppr_rank"]
    big = ref >= 1e-12
    assert np.max(np.abs(xr[big] - ref[big]) / ref[big]) < 1e-5
    assert oracle.topk_ref(oracle.c_rca_key(r, q), 10)[0].tolist() == g["ppr_top10"].tolist()
    assert set(C.ROOTS) <= set(g["ppr_top10"].tolist())
    # a12: the literal restatement against the reference's own patterns
    for d in range(C.P):
        n, h, _ = oracle.log_hist(blob[off[d]:off[d + 1]].decode("utf-8", "surrogatepass"))
        assert n == g["log_lines"][d] and h == g["log_hist"][d].tolist(), d
    # a9: float64 correlation
    z = oracle.corr_standardize(x, 0)
    idx, rr, cnt, gap = oracle.corr_rows(z, np.arange(C.P), 10, 0.5)
    assert np.array_equal(idx, g["corr_idx"]) and np.array_equal(cnt, g["corr_count"])
    assert np.allclose(rr, g["corr_r"], rtol=1e-12, atol=1e-12)


def test_coordinator_ranking_equals_bench_ranking_cpu():
    """Coordinator.ranked_root_causes on a mesh client == oracle.rca_rank (the bench's checker)."""
    from krca import synth
    from krca.agents.coordinator import Coordinator
    from krca.mock import MeshClient
    from oracle_engine import OracleEngine
    m = synth.make_graph(3000, n_edges=60_000, seed=5)
    x = synth.make_metrics(3000, 8, 300, seed=5, roots=m.roots, hop_sets=synth.caller_hops(m, m.roots)).numpy()
    res = Coordinator(MeshClient(m, x), engine=OracleEngine()).run_analysis("comprehensive", "test-microservices")
    got = [int(r["component"].split("-")[-1]) for r in res["ranked_root_causes"]]
    score = oracle.c_rolling_score(x, RANKING.window)["score"]
    idx, _, _ = oracle.rca_rank(m.row_ptr, m.col, m.outdeg, score, RANKING.alpha, RANKING.iters,
                                RANKING.floor(3000, 8), RANKING.k, tol=RANKING.tol)
    assert got == idx.tolist()
    assert Config().as_dict() == RANKING.as_dict()
