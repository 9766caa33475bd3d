"""f3: krca_betweenness against networkx 3.4.2 betweenness_centrality (the reference's SPOF check,
ref:agents/topology_agent.py:329).  Same float64 formulas; the dependency sum runs in CSR order
instead of networkx's stack order, so values agree to 1e-12 relative, and the SPOF decision
(value > 0.5) is identical wherever a value is not within 1e-9 of 0.5.  Exact ties (chains)
come out exact.  At 20k nodes the total is checked against the path-length identity
sum_v bc(v) = sum over reachable ordered pairs (s, t) of (d(s, t) - 1), computed exactly by
scipy's BFS."""
import networkx as nx
import numpy as np
import pytest

from krca import native

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    return native.NativeEngine()


def _csr(g, nodes):
    pos = {n: i for i, n in enumerate(nodes)}
    rp, col = [0], []
    nb = g.successors if g.is_directed() else g.neighbors
    for n in nodes:
        col.extend(pos[m] for m in nb(n))
        rp.append(len(col))
    return rp, col


def _check(eng, g, batch=1024):
    nodes = list(g.nodes)
    rp, col = _csr(g, nodes)
    got = eng.betweenness(rp, col, normalized=True, directed=g.is_directed(), batch=batch)
    ref = nx.betweenness_centrality(g)
    want = np.array([ref[n] for n in nodes])
    assert np.allclose(got, want, rtol=1e-12, atol=1e-15), np.max(np.abs(got - want))
    clear = np.abs(want - 0.5) > 1e-9
    assert np.array_equal((got > 0.5)[clear], (want > 0.5)[clear])
    return got, want


@pytest.mark.parametrize("n,p,seed", [(30, 0.1, 1), (200, 0.02, 2), (1000, 0.004, 3), (1500, 0.002, 4)])
def test_betweenness_random_digraphs(eng, n, p, seed):
    _check(eng, nx.gnp_random_graph(n, p, seed=seed, directed=True))


def test_betweenness_undirected_and_small_batches(eng):
    _check(eng, nx.gnp_random_graph(300, 0.02, seed=5), batch=7)
    _check(eng, nx.barabasi_albert_graph(500, 2, seed=6))


def test_betweenness_exact_ties_and_degenerate(eng):
    chain = nx.DiGraph([(0, 1), (1, 2)])  # middle node exactly 0.5: not critical
    got, want = _check(eng, chain)
    assert got[1] == 0.5 and want[1] == 0.5
    _check(eng, nx.DiGraph([(i, 0) for i in range(1, 6)] + [(0, j) for j in range(6, 9)]))
    _check(eng, nx.DiGraph([(0, 1)]))
    _check(eng, nx.empty_graph(4, create_using=nx.DiGraph))


def test_betweenness_20k_path_length_identity(eng):
    from scipy.sparse import csr_matrix
    from scipy.sparse.csgraph import shortest_path
    g = nx.barabasi_albert_graph(20000, 2, seed=7).to_directed()
    nodes = list(g.nodes)
    rp, col = _csr(g, nodes)
    n = len(nodes)
    got = eng.betweenness(rp, col)
    A = csr_matrix((np.ones(len(col)), np.asarray(col), np.asarray(rp)), shape=(n, n))
    total = 0.0
    for s0 in range(0, n, 2000):
        d = shortest_path(A, directed=True, unweighted=True, indices=np.arange(s0, min(n, s0 + 2000)))
        d = d[np.isfinite(d)]
        total += float(np.sum(np.maximum(d - 1, 0)))
    assert got.min() >= 0 and np.isfinite(got).all()
    assert abs(got.sum() * (n - 1) * (n - 2) - total) / total < 1e-9
