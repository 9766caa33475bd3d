#!/usr/bin/env python3
"""Golden capture for service-graph construction — TEST INFRASTRUCTURE.

Runs the REFERENCE's TopologyAgent._build_service_graph (ref:agents/topology_agent.py:94-260)
and ResourceAnalyzer._find_matching_pods (ref:agents/resource_analyzer.py:835-854) on seeded
random clusters (own generator below) and records, as data, the graph's node list with its
attributes and its edge list with edge types, both in insertion order, and each service's
matching pod indices.  Run by hand in the build container only
(`python tests/golden/capture_topograph.py`); writes tests/golden/topograph_cases.json.
"""
import json
import os
import random
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from capture_reference import REF, DictClient, dump, install_stubs  # noqa: E402

KEYS = ["app", "tier", "team", "version", "zone"]
VALS = ["a", "b", "web", "db", "v1", "v2", "blue", "ü", ""]
WORDS = ["api", "api-gw", "db", "db-main", "cache", "web", "pay", "payments", "auth", "q", "search", "a", "ab"]


def gen_cluster(rng, n_svc, n_dep, n_pod, n_cm=3, n_sec=3, nsname="shop"):
    def items(lo, hi):
        return {k: rng.choice(VALS) for k in rng.sample(KEYS, rng.randint(lo, hi))}

    svc_names = []
    for i in range(n_svc):
        base = rng.choice(WORDS)
        svc_names.append(base if rng.random() < 0.3 else "%s-%d" % (base, i))
    services = []
    for i, name in enumerate(svc_names):
        ns = nsname if rng.random() < 0.9 else "other"
        services.append({"metadata": {"name": name, "namespace": ns},
                         "spec": {"selector": items(0, 2), "type": "ClusterIP", "ports": [{"port": 80}]}})
    deployments = []
    for i in range(n_dep):
        name = rng.choice(svc_names) if rng.random() < 0.1 else "%s-dep-%d" % (rng.choice(WORDS), i)
        md = {"name": name}
        if rng.random() < 0.85:
            md["labels"] = items(0, 4)
        env = []
        for _ in range(rng.randint(0, 4)):
            r = rng.random()
            s = rng.choice(svc_names)
            if r < 0.3:
                v = "http://%s.%s.svc.cluster.local:%d" % (s, nsname, rng.randint(1, 9999))
            elif r < 0.45:
                v = "%s.%s" % (s, rng.choice([nsname, "other"]))
            elif r < 0.55:
                v = "%s,%s.%s.svc" % (s, rng.choice(svc_names), nsname)
            elif r < 0.65:
                v = "x" + s[: max(1, len(s) - 1)]
            elif r < 0.75:
                v = "ünï-%s-é" % s
            elif r < 0.8:
                v = ""
            else:
                v = "plain-%d" % rng.randint(0, 99)
            var = {"name": "E%d" % len(env)}
            if rng.random() < 0.9:
                var["value"] = v
            else:
                var["valueFrom"] = {"configMapKeyRef": {"name": "cm%d" % rng.randint(0, n_cm)}}
            env.append(var)
        spec = {"containers": [{"name": "c", "image": "img", "env": env}]}
        if rng.random() < 0.2:
            spec["volumes"] = [{"name": "v", "configMap": {"name": "cm%d" % rng.randint(0, n_cm)}},
                               {"name": "s", "secret": {"secretName": "sec%d" % rng.randint(0, n_sec)}}]
        deployments.append({"metadata": md, "spec": {"replicas": rng.randint(1, 3), "template": {"spec": spec}}})
    pods = []
    for i in range(n_pod):
        md = {"name": "pod-%d" % i}
        if rng.random() < 0.9:
            md["labels"] = items(0, 5)
        pods.append({"metadata": md, "status": {"phase": "Running"}})
    ingresses = [{"metadata": {"name": "edge"}, "spec": {"rules": [{"http": {"paths": [
        {"backend": {"serviceName": rng.choice(svc_names)}}, {"backend": {"serviceName": "ghost"}}]}}]}}]
    return dict(services=services, deployments=deployments, pods=pods, ingresses=ingresses,
                configmaps=[{"metadata": {"name": "cm%d" % i}} for i in range(n_cm)],
                secrets=[{"metadata": {"name": "sec%d" % i}} for i in range(n_sec)])


def main():
    sys.dont_write_bytecode = True
    install_stubs()
    sys.path.insert(0, REF)
    os.chdir(tempfile.mkdtemp(prefix="krca_ref_"))
    from agents.resource_analyzer import ResourceAnalyzer  # noqa: E402
    from agents.topology_agent import TopologyAgent  # noqa: E402

    cases = {}
    for name, seed, shape in [("small", 1, (8, 10, 20)), ("medium", 2, (60, 200, 300)), ("wide", 3, (150, 120, 500))]:
        rng = random.Random(seed)
        sc = gen_cluster(rng, *shape)
        ag = TopologyAgent(DictClient(**sc))
        ag._build_service_graph(sc["deployments"], sc["services"], sc["pods"], sc["ingresses"], sc["configmaps"],
                                sc["secrets"])
        g = ag.service_graph
        nodes = [[n, {k: v for k, v in a.items()}] for n, a in g.nodes(data=True)]
        edges = [[u, v, a.get("type")] for u, v, a in g.edges(data=True)]
        ra = ResourceAnalyzer(DictClient(**sc))
        pod_idx = {p["metadata"]["name"]: i for i, p in enumerate(sc["pods"])}
        matches = [[pod_idx[p["metadata"]["name"]] for p in ra._find_matching_pods("shop", s["spec"]["selector"])]
                   for s in sc["services"]]
        cases[name] = {"inputs": sc, "nodes": nodes, "edges": edges, "service_pods": matches}
        print(name, len(nodes), "nodes", len(edges), "edges", sum(map(len, matches)), "pod matches")
    dump("topograph_cases.json", cases)


if __name__ == "__main__":
    main()
