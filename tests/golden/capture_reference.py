#!/usr/bin/env python3
"""Golden-vector capture: run the REFERENCE (vobbilis/kubernetes-rca-system, read-only at
/root/reference) in THIS container and record its outputs as small JSON fixtures.

This script is test infrastructure.  It is run by hand in the build container only
(`python tests/golden/capture_reference.py`); nothing on the GPU box runs it and no
reference source is copied anywhere: the outputs below are data (inputs + expected outputs).

What it records (SURVEY.md §8c "Goldens to capture"):
  mock_cluster.json        the MockK8sClient fixture data (utils/mock_k8s_client.py:28-798,
                           plus the constant returns of :1146-1272), re-typed as JSON so the
                           build's own MockK8sClient can serve the identical cluster
  c1_raw.json              Coordinator.run_analysis for every type on the raw mock
  c1_shim.json             same with the test double that fixes the mock's API gaps (§4)
  c1_resource.json         ResourceAnalyzer.analyze_namespace_resources on the mock
  logs_corpus.json         13-pattern per-line masks + _analyze_container_logs outputs on a
                           stress corpus (ASCII + non-ASCII / splitlines hazards)
  topology_small.json      TopologyAgent findings on hand-built small clusters
  metrics_scaled.json      MetricsAgent findings on a 2,000-pod dict cluster with boundary values
  events_cases.json        EventsAgent findings on synthetic event lists
  ppr_known.json           nx.pagerank on the mock's trace dependency map (networkx 3.4.2)

Timestamps (datetime.now()) are stripped from every finding / reasoning step / metadata.
"""
import copy
import json
import os
import random
import re
import sys
import tempfile
import types

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
PKG_DATA = os.path.join(HERE, "..", "..", "kubernetes-rca-system_amd", "krca", "data")


def install_stubs():
    """Empty modules for third-party packages the reference imports but the path never uses."""
    for name in ["kubernetes", "kubernetes.client", "kubernetes.config", "streamlit"]:
        sys.modules[name] = types.ModuleType(name)
    sys.modules["kubernetes"].client = sys.modules["kubernetes.client"]
    sys.modules["kubernetes"].config = sys.modules["kubernetes.config"]


def strip_ts(obj):
    if isinstance(obj, dict):
        return {k: strip_ts(v) for k, v in obj.items() if k != "timestamp"}
    if isinstance(obj, list):
        return [strip_ts(v) for v in obj]
    return obj


def dump(name, obj):
    path = os.path.join(HERE, name)
    with open(path, "w") as f:
        json.dump(obj, f, indent=1, sort_keys=False, ensure_ascii=True)
    print("wrote", path, os.path.getsize(path), "bytes")


class DictClient:
    """A minimal duck-typed client over plain dicts (the L1 methods the classic agents call)."""

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


# ----------------------------------------------------------------------------------------
# log stress corpus (own generator; only the EXPECTED masks come from the reference)
# ----------------------------------------------------------------------------------------
ERR_TEMPLATES = [
    "Out of memory: Kill process {n} (java) score {m}",
    "Container {w} was OOMKilled (exit code 137)",
    "worker {n} terminated: signal: killed",
    "process {n} KILLED by supervisor",
    "dial tcp 10.0.{n}.{m}:5432: connect: connection refused",
    "upstream Connection Refused after {n} retries",
    "open /var/lib/{w}/data: permission denied",
    "HTTP 403 Forbidden for /api/{w}",
    "access DENIED for user {w}",
    "context deadline exceeded (Client.Timeout exceeded while awaiting headers)",
    "request to {w} timed out after {n}ms",
    "read tcp 10.1.{n}.{m}:443: ETIMEDOUT",
    "Back-off restarting failed container {w}",
    "pod {w} in CrashLoopBackOff",
    "API server error: etcdserver: request timed out",
    "upstream returned StatusCode={s}",
    "Unable to mount volumes for pod {w}",
    "MountVolume.SetUp failed for volume pvc-{n}",
    "MountVolumeXSetUp failed for volume {w}",
    "Failed to pull image {w}:{n}: ErrImagePull",
    "image {w} ImagePullBackOff",
    "DNS resolution failed for {w}.svc",
    "could not resolve host {w}.example",
    "401 Unauthorized: token expired",
    "Authentication failed for user {w}",
    "Invalid configuration: key {w} missing",
    "configmap not found: {w}-config",
    "Secret not found: {w}-tls",
    "500 Internal Server Error from {w}",
    "InternalServerError: {w}",
    "Exception in thread main java.lang.NullPointerException",
    "ERROR: failed to process batch {n}",
    "Traceback (most recent call last):",
    "FATAL: database {w} does not exist",
    "CRITICAL: disk quota {n}% used",
    "panic: runtime error: index out of range [{n}]",
    "StatusCode=5{n}0 retrying",
    "statuscode=5ab invalid",
    "errImagepull backoff",
]
BENIGN_TEMPLATES = [
    "INFO: GET /api/v1/items 200 {n}ms",
    "DEBUG: cache hit ratio 0.{n}",
    "Starting worker {n} for queue {w}",
    "healthcheck ok ({n} checks)",
    "INFO: request id={h} user={w} latency={n}ms",
    "Reconciling {w}/{w2} generation {n}",
    "listening on 0.0.0.0:{n}",
    "WARN: slow query took {n}ms on {w}",
    "connected to {w}:{n}",
]
HAZARDS = [
    "Process Killed by kernel",            # KELVIN SIGN folds to k under re.IGNORECASE
    "Connection refuſed by peer",          # LATIN SMALL LONG S folds to s
    "upstream StatusCode=5٣٤",         # Arabic-Indic digits match \d
    "ünicöde message without issues",
    "tïmeout but with diaeresis",
    "timeout second half after LINE SEPARATOR",
    "panic\u0085after NEL",
    "AUTHENTİCATION FAİLED dotted I",
    "ok paragraph sep Forbidden",
    "café server error=none",
    "MountVolume·SetUp failed middle dot wildcard",
]
WORDS = ["frontend", "backend", "db", "cache", "payments", "auth", "queue", "search", "gateway"]


def gen_line(rng):
    r = rng.random()
    w = rng.choice(WORDS)
    w2 = rng.choice(WORDS)
    n = rng.randint(0, 99999)
    m = rng.randint(0, 255)
    s = rng.choice(["500", "502", "503", "504", "599", "5x3", "404", "5"])
    h = "%016x" % rng.getrandbits(64)
    if r < 0.35:
        t = rng.choice(ERR_TEMPLATES)
    elif r < 0.97:
        t = rng.choice(BENIGN_TEMPLATES)
    else:
        t = rng.choice(HAZARDS)
    line = t.format(w=w, w2=w2, n=n, m=m, s=s, h=h)
    # random case mangling exercises IGNORECASE
    if rng.random() < 0.1:
        line = "".join(c.upper() if rng.random() < 0.5 else c.lower() for c in line)
    if rng.random() < 0.02:
        line = line + " " + ("x" * rng.randint(150, 300))  # >200 char evidence truncation
    ts = "2024-05-%02dT%02d:%02d:%02d.%03dZ " % (rng.randint(1, 28), rng.randint(0, 23), rng.randint(0, 59),
                                                 rng.randint(0, 59), rng.randint(0, 999))
    return ts + line


SEPS = ["\n"] * 40 + ["\r\n"] * 4 + ["\r", "\x0b", "\x0c", "\x1c", "\x1d", "\x1e", "\x85", " ", "\n\n"]


def gen_container_text(rng, nlines):
    parts = []
    for i in range(nlines):
        parts.append(gen_line(rng))
        if i + 1 < nlines or rng.random() < 0.5:
            parts.append(rng.choice(SEPS))
    return "".join(parts)


def main():
    sys.dont_write_bytecode = True
    install_stubs()
    sys.path.insert(0, REF)
    work = tempfile.mkdtemp(prefix="krca_ref_")
    os.chdir(work)  # the reference writes resource_analysis.log / logs/ into the CWD

    from utils.mock_k8s_client import MockK8sClient  # noqa: E402
    from agents.coordinator import Coordinator  # noqa: E402
    from agents.logs_agent import LogsAgent  # noqa: E402
    from agents.metrics_agent import MetricsAgent  # noqa: E402
    from agents.topology_agent import TopologyAgent  # noqa: E402
    from agents.events_agent import EventsAgent  # noqa: E402
    from agents.resource_analyzer import ResourceAnalyzer  # noqa: E402
    import networkx as nx  # noqa: E402

    # ---- 1. mock fixture data -------------------------------------------------------
    mk = MockK8sClient()
    data = {
        "current_context": mk.current_context,
        "available_contexts": mk.available_contexts,
        "namespaces": mk.namespaces,
        "pods": mk.pods,
        "services": mk.services,
        "deployments": mk.deployments,
        "pod_metrics": mk.pod_metrics,
        "node_metrics": mk.node_metrics,
        "events": mk.events,
        "logs": mk.logs,
        "network_policies": mk.network_policies,
        "endpoints": mk.endpoints,
        "hpas": mk.hpas,
        "trace_ids": mk.get_trace_ids(limit=100),
        "trace_details_template": mk.get_trace_details("TRACE_ID"),
        "service_latency_stats": mk.get_service_latency_stats(),
        "error_rate_by_service": mk.get_error_rate_by_service(),
        "service_dependencies": mk.get_service_dependencies(),
        "slow_operations": mk.find_slow_operations(),
    }
    os.makedirs(PKG_DATA, exist_ok=True)
    with open(os.path.join(PKG_DATA, "mock_cluster.json"), "w") as f:
        json.dump(data, f, indent=1, ensure_ascii=True)
    print("wrote mock_cluster.json")

    ns = "test-microservices"
    types_ = ["metrics", "logs", "topology", "events", "traces", "comprehensive"]

    # ---- 2. C1 raw ------------------------------------------------------------------
    out = {}
    for t in types_:
        out[t] = strip_ts(Coordinator(MockK8sClient()).run_analysis(t, ns))
    out["unknown"] = Coordinator(MockK8sClient()).run_analysis("bogus", ns)
    for other_ns in ["default", "kube-system", "nope"]:
        out["comprehensive@" + other_ns] = strip_ts(Coordinator(MockK8sClient()).run_analysis("comprehensive", other_ns))
    dump("c1_raw.json", out)

    # ---- 3. C1 shimmed (SURVEY §8c test double) ------------------------------------
    class Shim(MockK8sClient):
        def get_recently_terminated_pods(self, namespace):
            return []

        def get_pod_logs(self, pod_name, namespace, container_name=None, tail_lines=100, previous=False):
            return MockK8sClient.get_pod_logs(self, namespace, pod_name, container_name, tail_lines, previous)

    out = {}
    for t in types_:
        out[t] = strip_ts(Coordinator(Shim()).run_analysis(t, ns))
    dump("c1_shim.json", out)

    # ---- 4. ResourceAnalyzer -------------------------------------------------------
    out = {}
    for n_ in [ns, "default"]:
        out[n_] = strip_ts(ResourceAnalyzer(MockK8sClient()).analyze_namespace_resources(n_))
    dump("c1_resource.json", out)

    # ---- 5. logs stress corpus -----------------------------------------------------
    rng = random.Random(20240515)
    la = LogsAgent(DictClient())
    patterns = list(la.error_patterns.items())
    containers = []
    total_lines = 0
    for ci in range(96):
        nlines = rng.choice([1, 2, 3, 5, 40, 150, 200, 250, 300])
        text = gen_container_text(rng, nlines)
        lines = text.splitlines()
        masks = []
        for line in lines:
            mm = 0
            for b, (_, p) in enumerate(patterns):
                if re.search(p, line, re.IGNORECASE):
                    mm |= 1 << b
            masks.append(mm)
        total_lines += len(lines)
        la.reset()
        la._analyze_container_logs("pod-%d" % ci, "c%d" % (ci % 3), text)
        containers.append({
            "pod": "pod-%d" % ci, "container": "c%d" % (ci % 3), "text": text,
            "masks": masks, "result": strip_ts(la.get_results()),
        })
    dump("logs_corpus.json", {
        "patterns": [[k, p] for k, p in patterns],
        "severity": {k: la._determine_error_severity(k) for k, _ in patterns},
        "title": {k: la._format_error_type(k) for k, _ in patterns},
        "recommendation": {k: la._get_recommendation_for_error(k) for k, _ in patterns},
        "total_lines": total_lines,
        "containers": containers,
    })

    # ---- 6. topology small clusters --------------------------------------------------
    def svc(name, sel, typ="ClusterIP", nsname="shop"):
        return {"metadata": {"name": name, "namespace": nsname}, "spec": {"selector": sel, "type": typ, "ports": [{"port": 80}]}}

    def dep(name, labels, env=None, replicas=1, volumes=None, env_from=None):
        c = {"name": name, "image": "img"}
        if env is not None:
            c["env"] = env
        if env_from is not None:
            c["envFrom"] = env_from
        spec = {"containers": [c]}
        if volumes is not None:
            spec["volumes"] = volumes
        md = {"name": name}
        if labels is not None:
            md["labels"] = labels
        return {"metadata": md, "spec": {"replicas": replicas, "template": {"spec": spec}}}

    def url(s, nsname="shop"):
        return [{"name": "UPSTREAM", "value": "http://%s.%s.svc.cluster.local:80" % (s, nsname)}]

    scenarios = {}
    # chain: svc-i selects dep-i; dep-i depends on svc-(i+1)
    n = 6
    scenarios["chain"] = dict(
        services=[svc("s%d" % i, {"app": "s%d" % i}) for i in range(n)],
        deployments=[dep("d%d" % i, {"app": "s%d" % i}, env=url("s%d" % (i + 1)) if i + 1 < n else [],
                         replicas=1 if i % 2 else 3) for i in range(n)],
    )
    scenarios["cycle"] = dict(
        services=[svc(x, {"app": x}) for x in ["a", "b", "c"]],
        deployments=[dep(x + "-dep", {"app": x}, env=url(y)) for x, y in [("a", "b"), ("b", "c"), ("c", "a")]],
    )
    scenarios["hub"] = dict(
        services=[svc("db", {"app": "db"})] + [svc("web%d" % i, {"app": "web%d" % i}) for i in range(5)],
        deployments=[dep("db-dep", {"app": "db"}, replicas=1)] +
                    [dep("web%d-dep" % i, {"app": "web%d" % i}, env=url("db")) for i in range(5)],
        ingresses=[{"metadata": {"name": "edge"}, "spec": {"rules": [{"http": {"paths": [
            {"backend": {"serviceName": "web0"}}, {"backend": {"serviceName": "ghost"}}]}}]}}],
    )
    scenarios["isolates_and_config"] = dict(
        services=[svc("lonely-api", {"app": "none"}), svc("ui", {"app": "ui"}), svc("web-frontend", {"app": "wf"}, typ="NodePort")],
        deployments=[dep("worker", None), dep("ui", {"app": "ui"},
                                              env=[{"name": "X", "valueFrom": {"configMapKeyRef": {"name": "cm1"}}},
                                                   {"name": "Y", "valueFrom": {"secretKeyRef": {"name": "missing-sec"}}}],
                                              volumes=[{"name": "v", "configMap": {"name": "cm-missing"}},
                                                       {"name": "s", "secret": {"secretName": "sec1"}}],
                                              env_from=[{"configMapRef": {"name": "cm1"}}, {"secretRef": {"name": "nosec"}}])],
        configmaps=[{"metadata": {"name": "cm1"}}],
        secrets=[{"metadata": {"name": "sec1"}}],
        network_policies=[{"metadata": {"name": "allow-all"}, "spec": {"podSelector": {"matchLabels": {"app": "ui"}},
                                                                        "ingress": [{}, {"from": []}]}}],
    )
    # hub whose service and deployment share one name (nodes merge, selector self-loop,
    # ref:agents/topology_agent.py:107-134): every leaf pair routes through it -> SPOF
    scenarios["spof"] = dict(
        services=[svc("core", {"app": "core"})] + [svc("l%d" % i, {"app": "l%d" % i}) for i in range(4)],
        deployments=[dep("core", {"app": "core"}, replicas=1,
                         env=[{"name": "L%d" % i, "value": "l%d.shop:80" % i} for i in range(4)])] +
                    [dep("l%d-dep" % i, {"app": "l%d" % i}, env=url("core"), replicas=1) for i in range(4)],
    )
    scenarios["empty"] = dict()
    topo = {}
    for name, sc in scenarios.items():
        res = TopologyAgent(DictClient(**sc)).analyze("shop")
        topo[name] = {"inputs": sc, "result": strip_ts(res)}
    dump("topology_small.json", topo)

    # ---- 7. metrics scaled (dict path, boundary values) ----------------------------
    rng = random.Random(7)
    pods = {}
    specials = [80, 80.0, 80.0000001, 80.05, 79.99, 90, 90.0000001, 90.05, 100, 0, 80.00000000001]
    for i in range(2000):
        def u():
            r = rng.random()
            if r < 0.05:
                return rng.choice(specials)
            return round(rng.uniform(0, 100), rng.choice([0, 1, 2, 3, 6]))
        m = {}
        if rng.random() > 0.01:
            m["cpu"] = {"usage": rng.randint(0, 400), "usage_percentage": u()}
        if rng.random() > 0.01:
            m["memory"] = {"usage": rng.randint(0, 1 << 30), "usage_percentage": u()}
        pods["pod-%05d" % i] = m
    nodes = {"n%d" % i: {"cpu": {"usage_percentage": u()}, "memory": {"usage_percentage": u()}} for i in range(20)}
    res = MetricsAgent(DictClient(pod_metrics=pods, node_metrics=nodes)).analyze("scaled")
    res_quiet = MetricsAgent(DictClient(pod_metrics={k: {"cpu": {"usage_percentage": 10}} for k in list(pods)[:50]},
                                        node_metrics={})).analyze("quiet")
    dump("metrics_scaled.json", {"pod_metrics": pods, "node_metrics": nodes, "result": strip_ts(res),
                                 "quiet_result": strip_ts(res_quiet)})

    # ---- 8. events cases -------------------------------------------------------------
    rng = random.Random(11)
    reasons = ["BackOff", "Failed", "FailedScheduling", "FailedMount", "NodeNotReady", "Unhealthy", "Pulled",
               "MemoryPressure", "DiskPressure", "Evicted", "FailedAttachVolume", "CPUThrottling"]
    msgs = ["0/3 nodes are available: 3 Insufficient cpu.", "0/3 nodes: Insufficient memory",
            "node(s) had taint {x}", "node(s) didn't match node selector", "persistentvolumeclaim data is Pending",
            "MountVolume timeout expired", "no such file or directory", "permission denied", "pvc claim not found",
            "kubelet stopped posting node status", "readiness probe failed"]
    evs = []
    for i in range(60):
        kind = rng.choice(["Pod", "Pod", "Node", "Deployment"])
        evs.append({
            "involvedObject": {"kind": kind, "name": "%s-%d" % (kind.lower(), rng.randint(0, 5))},
            "type": rng.choice(["Warning", "Warning", "Normal"]),
            "reason": rng.choice(reasons),
            "message": rng.choice(msgs),
            "count": rng.randint(1, 30),
            "lastTimestamp": "2024-01-01T00:%02d:%02dZ" % (rng.randint(0, 59), rng.randint(0, 59)),
            "source": {"component": rng.choice(["kubelet", "kube-scheduler", "kube-controller-manager", "etcd"]),
                       "host": "node-%d" % rng.randint(0, 3)},
        })
    ev_out = {"events": evs, "result": strip_ts(EventsAgent(DictClient(events=evs)).analyze("x")),
              "empty": strip_ts(EventsAgent(DictClient(events=[])).analyze("x"))}
    dump("events_cases.json", ev_out)

    # ---- 9. PPR known answer (networkx 3.4.2 on reference fixture data) ----------------
    g = nx.DiGraph()
    deps = mk.get_service_dependencies()
    for s in deps:
        g.add_node(s)
    for s, ds in deps.items():
        for d in ds:
            g.add_edge(s, d)
    pers = mk.get_error_rate_by_service()
    pr = nx.pagerank(g, alpha=0.85, personalization=pers)
    dump("ppr_known.json", {"nodes": list(g.nodes()), "edges": [list(e) for e in g.edges()],
                            "personalization": pers, "alpha": 0.85, "pagerank": pr,
                            "ranking": sorted(pr, key=lambda k: -pr[k])})


if __name__ == "__main__":
    main()
