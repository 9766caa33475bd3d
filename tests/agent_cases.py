"""Golden-vector cases for the drop-in agents, shared by the CPU (oracle engine) and the GPU
(libkrca) test modules.  Expected outputs were captured from the reference itself by
tests/golden/capture_reference.py (timestamps stripped)."""
import copy
import json
import os

from conftest import GOLDEN

from krca.agents import Coordinator, EventsAgent, LogsAgent, MetricsAgent, ResourceAnalyzer, TopologyAgent
from krca.mock import MockK8sClient

NS = "test-microservices"
TYPES = ["metrics", "logs", "topology", "events", "traces", "comprehensive"]


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def strip(obj, drop=("timestamp",)):
    if isinstance(obj, dict):
        return {k: strip(v, drop) for k, v in obj.items() if k not in drop}
    if isinstance(obj, list):
        return [strip(v, drop) for v in obj]
    return obj


def normalize(obj):
    """View of a result that is independent of PYTHONHASHSEED.  Two reference outputs depend on
    string-hash order, so they differ between two runs of the reference itself:
      * ref:agents/topology_agent.py:483-487 prints ', '.join(set difference)  -> names sorted;
      * ref:agents/topology_agent.py:268-270 reports cycles[0] of nx.simple_cycles, whose
        start node comes from set iteration inside networkx              -> cycle masked
        (test_topology_cycles_valid checks the build's cycle is a real cycle of the graph)."""
    if isinstance(obj, dict):
        out = {k: normalize(v) for k, v in obj.items()}
        ev = out.get("evidence")
        if isinstance(ev, str) and ev.startswith("Services without network policies: "):
            names = ev[len("Services without network policies: "):].split(", ")
            out["evidence"] = "Services without network policies: " + ", ".join(sorted(names))
        if isinstance(ev, str) and ev.startswith("Dependency cycle: "):
            out["evidence"] = "Dependency cycle: <cycle>"
        return out
    if isinstance(obj, list):
        return [normalize(v) for v in obj]
    return obj


def same(actual, expected):
    return normalize(strip(actual)) == normalize(expected)


class Shim(MockK8sClient):
    """SURVEY.md §8c test double (same class name as in the capture): adds get_recently_terminated_pods and fixes the argument order."""

    def get_recently_terminated_pods(self, namespace):
        return []

    def get_pod_logs(self, pod_name, namespace, container_name=None, tail_lines=100, previous=False):
        return MockK8sClient.get_pod_logs(self, namespace, pod_name, container_name, tail_lines, previous)


class DictClient:
    def __init__(self, **kw):
        self.d = kw

    def set_context(self, c):
        return True

    def get_current_context(self):
        return "fixture-context"

    def get_current_time(self):
        return "T"

    def get_pods(self, ns):
        return copy.deepcopy(self.d.get("pods", []))

    def get_services(self, ns):
        return self.d.get("services", [])

    def get_deployments(self, ns):
        return self.d.get("deployments", [])

    def get_ingresses(self, ns):
        return self.d.get("ingresses", [])

    def get_configmaps(self, ns):
        return self.d.get("configmaps", [])

    def get_secrets(self, ns):
        return self.d.get("secrets", [])

    def get_network_policies(self, ns):
        return self.d.get("network_policies", [])

    def get_pod_metrics(self, ns):
        return self.d.get("pod_metrics", {})

    def get_node_metrics(self):
        return self.d.get("node_metrics", {})

    def get_hpas(self, ns):
        return self.d.get("hpas", [])

    def get_events(self, ns):
        return self.d.get("events", [])


def check_c1(engine, golden_name, client_cls):
    gold = load(golden_name)
    bad = []
    for t in TYPES:
        res = Coordinator(client_cls(), engine=engine).run_analysis(t, NS)
        res.pop("ranked_root_causes", None)  # additive key
        if not same(res, gold[t]):
            bad.append(t)
    return bad


def check_c1_other(engine):
    gold = load("c1_raw.json")
    bad = []
    for key in ["unknown", "comprehensive@default", "comprehensive@kube-system", "comprehensive@nope"]:
        t, _, ns = key.partition("@")
        res = Coordinator(MockK8sClient(), engine=engine).run_analysis("bogus" if t == "unknown" else t, ns or NS)
        res.pop("ranked_root_causes", None)
        if not same(res, gold[key]):
            bad.append(key)
    return bad


def check_resource(engine):
    gold = load("c1_resource.json")
    return [ns for ns in gold
            if not same(ResourceAnalyzer(MockK8sClient(), engine=engine).analyze_namespace_resources(ns), gold[ns])]


def random_pods(n, seed=0):
    """Pod dicts covering every branch of the reference's categorisation (f1 parity cases)."""
    import random
    rnd = random.Random(seed)
    phases = ['Pending', 'Running', 'Running', 'Running', 'Succeeded', 'Failed', 'Unknown', 'CrashLoopBackOff', None]
    waits = ['CrashLoopBackOff', 'ImagePullBackOff', 'ErrImagePull', 'ContainerCreating', 'PodInitializing', '']
    terms = ['Completed', 'Error', 'OOMKilled', '']

    def status(name):
        st = {}
        r = rnd.random()
        if r < 0.3:
            st['waiting'] = {'reason': rnd.choice(waits)} if rnd.random() < 0.9 else {}
        elif r < 0.5:
            st['terminated'] = {'reason': rnd.choice(terms)} if rnd.random() < 0.9 else {}
        elif r < 0.9:
            st['running'] = {}
        if rnd.random() < 0.05:
            st['waiting'] = {'reason': rnd.choice(waits)}
            st['terminated'] = {'reason': rnd.choice(terms)}
        cs = {'name': name, 'state': st}
        if rnd.random() < 0.9:
            cs['ready'] = rnd.random() < 0.8
        return cs

    pods = []
    for i in range(n):
        st = {}
        ph = rnd.choice(phases)
        if ph is not None:
            st['phase'] = ph
        conds = []
        for _ in range(rnd.randint(0, 3)):
            conds.append({'type': rnd.choice(['Ready', 'PodScheduled', 'Initialized']),
                          'status': rnd.choice(['True', 'False', 'Unknown'])})
        st['conditions'] = conds
        if rnd.random() < 0.9:
            st['containerStatuses'] = [status(rnd.choice(['app', 'sidecar', 'init-db'])) for _ in range(rnd.randint(0, 3))]
        if rnd.random() < 0.4:
            st['initContainerStatuses'] = [status(rnd.choice(['init-x', 'setup'])) for _ in range(rnd.randint(0, 2))]
        if rnd.random() < 0.05:
            st['reason'] = 'Evicted'
        pods.append({'metadata': {'name': f'pod-{i}'}, 'status': st})
    return pods


def check_logs_corpus(engine):
    gold = load("logs_corpus.json")
    bad = []
    agent = LogsAgent(DictClient(), engine=engine)
    from krca.agents.logs import pack_documents
    texts = [c["text"] for c in gold["containers"]]
    scan = engine.log_scan(*pack_documents(texts))
    for i, c in enumerate(gold["containers"]):
        agent.reset()
        agent._report_container(scan, i, c["pod"], c["container"])
        if strip(agent.get_results()) != c["result"]:
            bad.append(i)
    return bad


def check_topology(engine):
    gold = load("topology_small.json")
    bad = []
    for name, case in gold.items():
        res = TopologyAgent(DictClient(**case["inputs"]), engine=engine).analyze("shop")
        if not same(res, case["result"]):
            bad.append(name)
    return bad


def check_metrics_scaled(engine):
    gold = load("metrics_scaled.json")
    bad = []
    res = MetricsAgent(DictClient(pod_metrics=gold["pod_metrics"], node_metrics=gold["node_metrics"]),
                       engine=engine).analyze("scaled")
    if not same(res, gold["result"]):
        bad.append("scaled")
    first50 = {k: {"cpu": {"usage_percentage": 10}} for k in list(gold["pod_metrics"])[:50]}
    res = MetricsAgent(DictClient(pod_metrics=first50, node_metrics={}), engine=engine).analyze("quiet")
    if not same(res, gold["quiet_result"]):
        bad.append("quiet")
    return bad


def check_events(engine):
    gold = load("events_cases.json")
    bad = []
    if not same(EventsAgent(DictClient(events=gold["events"]), engine=engine).analyze("x"), gold["result"]):
        bad.append("events")
    if not same(EventsAgent(DictClient(events=[]), engine=engine).analyze("x"), gold["empty"]):
        bad.append("empty")
    return bad


def check_events_random(engine):
    """f4: reference EventsAgent outputs on random event lists with hazards (capture_events.py)."""
    gold = load("events_random.json")
    bad = []
    for name, case in gold["events"].items():
        if not same(EventsAgent(DictClient(events=case["events"]), engine=engine).analyze("x"), case["result"]):
            bad.append(name)
    return bad


def check_correlate(engine):
    """f4: reference _correlate_findings / _identify_root_causes on random finding lists."""
    gold = load("events_random.json")
    bad = []
    co = Coordinator(DictClient(), engine=engine)
    for name, case in gold["correlate"].items():
        corr = co._correlate_findings(*case["lists"])
        if corr != case["correlated"] or co._identify_root_causes(corr) != case["root_causes"]:
            bad.append(name)
    return bad


def _jsonable(x):
    return json.loads(json.dumps(x))


def check_topograph(engine, force_host=False):
    """f2: the build's service-graph construction and the ResourceAnalyzer selector
    matches against the reference's graphs on seeded random clusters (topograph_cases.json,
    captured by tests/golden/capture_topograph.py).  Returns a list of mismatches."""
    bad = []
    for name, case in load("topograph_cases.json").items():
        sc = case["inputs"]
        ag = TopologyAgent(DictClient(**sc), engine=engine)
        if force_host:
            ag._selector_rows = lambda *a: None
            ag._env_hits = lambda *a: None
        ag._build_service_graph(sc["deployments"], sc["services"], sc["pods"], sc["ingresses"], sc["configmaps"],
                                sc["secrets"])
        g = ag.service_graph
        nodes = _jsonable([[n, dict(a)] for n, a in g.nodes(data=True)])
        edges = [[u, v, a.get("type")] for u, v, a in g.edges(data=True)]
        if nodes != case["nodes"]:
            bad.append((name, "nodes"))
        if edges != case["edges"]:
            bad.append((name, "edges", len(edges), len(case["edges"])))
        ra = ResourceAnalyzer(DictClient(**sc), engine=engine)
        dev = ra._service_matches(sc["services"], "shop")
        if dev is None:
            bad.append((name, "service matches not on the device path"))
        else:
            idx = {p["metadata"]["name"]: i for i, p in enumerate(sc["pods"])}
            got = [[idx[p["metadata"]["name"]] for p in m] for m in dev]
            if got != case["service_pods"]:
                bad.append((name, "service_pods"))
    return bad
