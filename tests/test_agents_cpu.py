"""Host logic of the drop-in agents against the reference goldens, on CPU.

The device kernels are replaced by the oracle engine (tests/oracle_engine.py); the same cases
run through libkrca on the GPU in tests/test_gpu_agents.py.
"""
import agent_cases as A
from oracle_engine import OracleEngine

ENG = OracleEngine()


def test_c1_raw_mock_all_types():
    assert A.check_c1(ENG, "c1_raw.json", A.MockK8sClient) == []


def test_c1_shimmed_mock_all_types():
    assert A.check_c1(ENG, "c1_shim.json", A.Shim) == []


def test_c1_other_namespaces_and_unknown_type():
    assert A.check_c1_other(ENG) == []


def test_resource_analyzer():
    assert A.check_resource(ENG) == []


def test_pod_status_columns_restate_the_reference():
    """f1: the columnar encoding + classification rules (oracle) == the reference's dict walk."""
    import oracle
    from krca import podstate
    pods = A.random_pods(3000, seed=5)
    ref = oracle.categorize_pods_ref(pods)
    mask, hist = oracle.pod_classify_ref(*podstate.encode_pods(pods))
    got = podstate.groups_from_masks(list(range(len(pods))), mask)
    assert got == ref
    assert hist.tolist() == [len(ref[g]) for g in oracle.POD_GROUPS]
    assert all(len(ref[g]) for g in oracle.POD_GROUPS)  # every group exercised


def test_logs_corpus_findings():
    assert A.check_logs_corpus(ENG) == []


def test_topology_small_clusters():
    assert A.check_topology(ENG) == []


def test_metrics_scaled_boundaries():
    assert A.check_metrics_scaled(ENG) == []


def test_events_cases():
    assert A.check_events(ENG) == []


def test_events_random_reference_cases():
    assert A.check_events_random(ENG) == []


def test_correlate_random_reference_cases():
    assert A.check_correlate(ENG) == []


def test_correlate_bad_severity_raises_like_reference():
    co = A.Coordinator(A.DictClient(), engine=ENG)
    ok = {"component": "x", "severity": "high"}
    assert co._correlate_findings([ok, {"component": "y", "severity": "bogus"}]) == []  # singleton: never checked
    try:
        co._correlate_findings([ok, {"component": "x", "severity": "bogus"}])
        raise AssertionError("expected ValueError")
    except ValueError as e:
        assert str(e) == "'bogus' is not in list"


def test_events_columns_match_host_loop():
    """The columnar replay == the reference's loops (_host_analyze) on synthetic columns."""
    from krca import eventcols
    cols = eventcols.make_events(3000, seed=3, n_obj=200, n_hosts=8)
    evs = []
    for e in range(len(cols)):
        ev = {"involvedObject": {"kind": cols.kinds[cols.kind[e]], "name": cols.names[cols.name[e]]},
              "type": "Warning" if cols.warn[e] else "Normal", "message": cols.messages[cols.message[e]],
              "count": int(cols.count[e]), "lastTimestamp": "%08d" % cols.ts[e],
              "source": {"host": cols.hosts[cols.host[e]]}}
        if cols.reason[e] >= 0:
            ev["reason"] = cols.reasons[cols.reason[e]]
        if cols.comp[e] >= 0:
            ev["source"]["component"] = cols.comps[cols.comp[e]]
        evs.append(ev)
    a = A.EventsAgent(A.DictClient(events=evs), engine=ENG)
    dev = a.analyze("x")
    a.reset()
    a._host_analyze(evs)
    host = a.get_results()
    assert A.strip(dev["findings"]) == A.strip(host["findings"])
    assert len(dev["findings"]) > 50


def test_events_bulk_columns_equal_dict_path():
    """A client's get_event_columns (bulk accessor) gives the same findings as its event dicts."""
    from krca import eventcols

    class Bulk(A.DictClient):
        def get_event_columns(self, ns):
            return self.cols

    evs = A.load("events_random.json")["events"]["medium"]["events"]
    cols = eventcols.encode_events(evs)
    assert cols is not None
    c = Bulk(events=evs)
    c.cols = cols
    assert A.strip(A.EventsAgent(c, engine=ENG).analyze("x")) == A.strip(
        A.EventsAgent(A.DictClient(events=evs), engine=ENG).analyze("x"))
    assert eventcols.encode_events([{"involvedObject": {"name": 3}}]) is None  # non-str: reference loops


def test_comprehensive_roots_order():
    res = A.Coordinator(A.Shim(), engine=ENG).run_analysis("comprehensive", A.NS)
    assert [r["component"] for r in res["root_causes"]] == [
        "Pod/database-7c9f8b6d5e-3x5qp/database", "Pod/api-gateway-6b7c8d9e5f-4q3zx/api-gateway"]
    ranked = [r["component"] for r in res["ranked_root_causes"]]
    # the ranking definition of krca.rca.Config (alpha 0.5, 30 iterations, key "explained"; the
    # mock's per-service error rates as seeds, floor 0) on the mock's trace dependency map.  The
    # database is the deepest anomalous service (api-gateway -> backend -> database) and explains
    # nothing below it; api-gateway keeps 0.20 of its 0.25 after the backend's 0.05; backend is
    # explained by the database (0.15 >= 2 x 0.05) and the rest carry no unexplained anomaly, so they
    # follow at key 0 in index order.  Not networkx's pagerank order (tests/golden/ppr_known.json:
    # database > backend > api-gateway at alpha 0.85, r alone), whose vector is pinned separately
    # (test_gpu_kernels.py::test_ppr_known_answer); its top-1 is the same service.
    assert ranked == ["Service/database", "Service/api-gateway", "Service/frontend", "Service/backend",
                      "Service/resource-service"]
    score = [r["score"] for r in res["ranked_root_causes"]]
    assert score[0] > score[1] > 0 and score[2:] == [0.0, 0.0, 0.0]


def test_threshold_safe_conversion():
    import numpy as np
    from krca.agents.metrics import to_f32_threshold_safe
    v = np.array([80.0, 80.0000001, 80.00000000001, 90.0000000001, 79.99999999, 90.0, np.nan, 1e300])
    f = to_f32_threshold_safe(v)
    assert list(f > 80) == list(v > 80)
    assert list(f > 90) == list(v > 90)


def test_topology_cycles_valid():
    gold = A.load("topology_small.json")
    for name, case in gold.items():
        agent = A.TopologyAgent(A.DictClient(**case["inputs"]), engine=ENG)
        res = agent.analyze("shop")
        for f in res["findings"]:
            if f["evidence"].startswith("Dependency cycle: "):
                nodes = f["evidence"][len("Dependency cycle: "):].split(" → ")
                assert nodes[0] == nodes[-1]
                for u, v in zip(nodes, nodes[1:]):
                    assert agent.service_graph.has_edge(u, v), (name, u, v)


def test_logs_agent_refuses_edited_error_patterns():
    """The reference matches whatever LogsAgent.error_patterns holds (ref:agents/logs_agent.py:20,
    147-149); the device matcher is compiled, so an edited dict is refused through the agent's
    error contract instead of giving silently different histograms."""
    agent = A.LogsAgent(A.Shim(), engine=ENG)
    ok = agent.analyze(A.NS)
    assert "error" not in ok
    agent.error_patterns["timeout"] = r"(deadline)"
    res = agent.analyze(A.NS)
    assert "error_patterns differs" in res.get("error", "")
    del agent.error_patterns["timeout"]
    assert "error_patterns differs" in agent.analyze(A.NS).get("error", "")
