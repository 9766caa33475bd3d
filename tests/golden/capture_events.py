#!/usr/bin/env python3
"""Golden capture for the f4 group-bys — TEST INFRASTRUCTURE.

Runs the REFERENCE's EventsAgent.analyze (ref:agents/events_agent.py:36-446) on seeded random
event lists (own generator below, with the hazards the columnar path must keep: missing keys,
timestamp and count ties, object keys that format to the same "kind/name" string, node names
shared with source hosts, substring reasons / components, non-ASCII text) and
Coordinator._correlate_findings / _identify_root_causes (ref:agents/coordinator.py:118-184) on
random finding lists, and records inputs and outputs as data.  Run by hand in the build
container only (`python tests/golden/capture_events.py`); writes tests/golden/events_random.json.
"""
import os
import random
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from capture_reference import REF, DictClient, dump, install_stubs, strip_ts  # noqa: E402

KINDS = ["Pod", "Pod", "Pod", "Node", "Deployment", "a/b", "a", "Pöd"]
NAMES = ["web-0", "web-1", "db-0", "node-1", "node-2", "c", "b/c", "ünï", "unknown"]
REASONS = ["BackOff", "Failed", "FailedScheduling", "FailedMount", "FailedMountX", "NodeNotReady", "XNodeNotReady",
           "Unhealthy", "Pulled", "MemoryPressure", "DiskPressure", "Evicted", "FailedAttachVolume",
           "FailedDetachVolume", "NetworkUnavailable", "KubeletNotReady", "CPUThrottling", "Error"]
MSGS = ["0/3 nodes are available: 3 Insufficient cpu.", "0/3 nodes: Insufficient memory", "node(s) had taint {x}",
        "node(s) didn't match node selector", "PersistentVolumeClaim data is PENDING", "MountVolume TIMEOUT expired",
        "no such file or directory", "Permission denied", "PVC claim Not Found", "kubelet stopped posting",
        "readiness probe failed", "ünïcode message ✓", ""]
COMPS = ["kubelet", "kube-scheduler", "kube-controller-manager", "etcd", "my-etcd-proxy", "kube-apiserver",
         "default-scheduler"]
HOSTS = ["node-1", "node-2", "node-3", "web-0"]
SEVS = ["info", "low", "medium", "high", "critical"]


def gen_events(rng, n, n_ts):
    evs = []
    for _ in range(n):
        e = {}
        io = {}
        if rng.random() < 0.95:
            io["kind"] = rng.choice(KINDS)
        if rng.random() < 0.95:
            io["name"] = rng.choice(NAMES)
        if rng.random() < 0.97:
            e["involvedObject"] = io
        if rng.random() < 0.95:
            e["type"] = rng.choice(["Warning", "Warning", "Normal", "Error"])
        if rng.random() < 0.95:
            e["reason"] = rng.choice(REASONS)
        if rng.random() < 0.95:
            e["message"] = rng.choice(MSGS)
        if rng.random() < 0.9:
            e["count"] = rng.choice([1, 5, 6, 6, 7, 20, 21, 30, rng.randint(1, 40)])
        if rng.random() < 0.93:
            e["lastTimestamp"] = "2024-01-01T00:%02d:00Z" % rng.randint(0, n_ts - 1)
        src = {}
        if rng.random() < 0.9:
            src["component"] = rng.choice(COMPS)
        if rng.random() < 0.9:
            src["host"] = rng.choice(HOSTS)
        if rng.random() < 0.95:
            e["source"] = src
        evs.append(e)
    return evs


def gen_findings(rng, n_lists, n, n_comp):
    comps = ["Pod/p%d" % i for i in range(n_comp)] + ["Node/n", "Service/ü"]
    return [[{"component": rng.choice(comps), "issue": "i%d" % rng.randint(0, 99), "severity": rng.choice(SEVS),
              "evidence": "e", "recommendation": "r"} for _ in range(rng.randint(0, n))] for _ in range(n_lists)]


def main():
    sys.dont_write_bytecode = True
    install_stubs()
    sys.path.insert(0, REF)
    os.chdir(tempfile.mkdtemp(prefix="krca_ref_"))
    from agents.coordinator import Coordinator  # noqa: E402
    from agents.events_agent import EventsAgent  # noqa: E402

    out = {"events": {}, "correlate": {}}
    for name, seed, n, n_ts in [("small", 1, 40, 5), ("ties", 2, 400, 3), ("medium", 3, 1500, 60)]:
        rng = random.Random(seed)
        evs = gen_events(rng, n, n_ts)
        res = strip_ts(EventsAgent(DictClient(events=evs)).analyze("x"))
        out["events"][name] = {"events": evs, "result": res}
        print(name, len(evs), "events", len(res["findings"]), "findings", "error" in res)
    coord = Coordinator(DictClient())
    for name, seed, shape in [("few", 4, (5, 6, 4)), ("many", 5, (5, 100, 30)), ("empty", 6, (5, 0, 1))]:
        rng = random.Random(seed)
        lists = gen_findings(rng, *shape)
        corr = coord._correlate_findings(*lists)
        roots = coord._identify_root_causes(corr)
        out["correlate"][name] = {"lists": lists, "correlated": corr, "root_causes": roots}
        print(name, sum(map(len, lists)), "findings", len(corr), "groups", len(roots), "roots")
    dump("events_random.json", out)


if __name__ == "__main__":
    main()
