"""The drop-in agents on the device path (libkrca) against the reference goldens."""
import pytest

import agent_cases as A
from krca import native

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    return native.NativeEngine()


def test_c1_raw(eng):
    assert A.check_c1(eng, "c1_raw.json", A.MockK8sClient) == []


def test_c1_shim(eng):
    assert A.check_c1(eng, "c1_shim.json", A.Shim) == []


def test_c1_other(eng):
    assert A.check_c1_other(eng) == []


def test_logs_corpus(eng):
    assert A.check_logs_corpus(eng) == []


def test_metrics_scaled(eng):
    assert A.check_metrics_scaled(eng) == []


def test_topology(eng):
    assert A.check_topology(eng) == []


def test_resource_analyzer_c1(eng):
    assert A.check_resource(eng) == []


def test_pod_classify_random_dicts(eng):
    """f1 kernel on every branch of the reference's categorisation (dict walk restated in oracle)."""
    import oracle
    from krca import podstate
    pods = A.random_pods(5000, seed=9)
    mask, hist = eng.pod_classify(*podstate.encode_pods(pods))
    assert podstate.groups_from_masks(list(range(len(pods))), mask) == oracle.categorize_pods_ref(pods)
    ref_mask, ref_hist = oracle.pod_classify_ref(*podstate.encode_pods(pods))
    assert (mask == ref_mask).all() and (hist == ref_hist).all()


@pytest.mark.parametrize("P", [0, 1, 255, 300_000, 3_000_000])
def test_pod_classify_columnar_scale(eng, P):
    import numpy as np

    import oracle
    from krca import podstate
    pc, off, cc = podstate.make_pod_states(P, seed=P)
    mask, hist = eng.pod_classify(pc, off, cc)
    sample = np.arange(P) if P <= 300_000 else np.random.default_rng(0).choice(P, 20000, replace=False)
    if P <= 300_000:
        ref_mask, ref_hist = oracle.pod_classify_ref(pc, off, cc)
        assert (mask == ref_mask).all() and (hist == ref_hist).all()
    else:  # sampled rows exact; histogram = the popcount of the kernel's own masks
        sub_off = np.concatenate([[0], np.cumsum(off[sample + 1] - off[sample])])
        sub_cc = np.concatenate([cc[off[i]:off[i + 1]] for i in sample])
        ref_mask, _ = oracle.pod_classify_ref(pc[sample], sub_off, sub_cc)
        assert (mask[sample] == ref_mask).all()
        assert hist.tolist() == [int(((mask >> b) & 1).sum()) for b in range(12)]


def test_ranked_root_causes_c1(eng):
    """The device ranking of the C1 mock equals the oracle engine's (tests/test_agents_cpu.py pins the
    order and explains it), scores included; with key "rq" the rounds-2-4 order is kept too."""
    from oracle_engine import OracleEngine
    from krca.rca import RANKING
    res = A.Coordinator(A.Shim(), engine=eng).run_analysis("comprehensive", A.NS)
    ref = A.Coordinator(A.Shim(), engine=OracleEngine()).run_analysis("comprehensive", A.NS)
    assert [r["component"] for r in res["ranked_root_causes"]] == [
        "Service/database", "Service/api-gateway", "Service/frontend", "Service/backend", "Service/resource-service"]
    assert [r["score"] for r in res["ranked_root_causes"]] == [r["score"] for r in ref["ranked_root_causes"]]
    rq = A.Coordinator(A.Shim(), engine=eng, rank_config=RANKING.replace(key="rq")).run_analysis("comprehensive", A.NS)
    assert [r["component"] for r in rq["ranked_root_causes"]] == [
        "Service/api-gateway", "Service/database", "Service/backend", "Service/resource-service", "Service/frontend"]


def test_default_engine_is_native():
    e = native.default_engine()
    assert isinstance(e, native.NativeEngine)
    assert e.lib.krca_version() == 100
