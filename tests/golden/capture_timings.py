#!/usr/bin/env python3
"""The reference's own CPU path, timed in the build container (BASELINE.md §3 "Reference CPU
path"): its Python is never shipped to the GPU box, so its timings are recorded here as a fixture
(tests/golden/ref_cpu_timings.json) that bench.py reports next to the build's own CPU baseline.

Test / measurement infrastructure, run by hand (`python tests/golden/capture_timings.py`).
Protocol: 5 warm-up runs, then >= 20 timed runs; median and p95; one core
(the reference is single-threaded by construction); CPU model from lscpu.

  metrics_thresholds_100k  MetricsAgent.analyze on 100,000 dict pods (ref:agents/metrics_agent.py:19-67;
                           the per-pod loops :88-94, :135-141)
  logs_13_patterns_100k    LogsAgent._analyze_container_logs on one 100,000-line container
                           (ref:agents/logs_agent.py:124-181: splitlines + 13 re.search passes)
  betweenness_1k           nx.betweenness_centrality on a random 1,000-node / 2,000-edge digraph,
                           the SPOF call of ref:agents/topology_agent.py:329 (networkx 3.4.2)
  comprehensive_c1         Coordinator.run_analysis('comprehensive') on the shimmed mock cluster
                           (ref:agents/coordinator.py:39-116)
"""
import json
import os
import platform
import random
import statistics
import subprocess
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)


def timed(fn, warmup=5, runs=20):
    for _ in range(warmup):
        fn()
    ts = []
    for _ in range(runs):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return {"median_s": statistics.median(ts), "p95_s": ts[min(len(ts) - 1, int(round(0.95 * (len(ts) - 1))))],
            "min_s": ts[0], "runs": runs, "warmup": warmup}


def lscpu_model():
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, check=True).stdout
        for ln in out.splitlines():
            if ln.startswith("Model name:"):
                return ln.split(":", 1)[1].strip()
    except (OSError, subprocess.CalledProcessError):
        pass
    return platform.processor()


def main():
    from capture_reference import REF, DictClient, gen_container_text, install_stubs
    sys.dont_write_bytecode = True
    install_stubs()
    sys.path.insert(0, REF)
    os.chdir(tempfile.mkdtemp(prefix="krca_ref_"))  # the reference writes logs into the CWD
    import networkx as nx
    from agents.coordinator import Coordinator
    from agents.logs_agent import LogsAgent
    from agents.metrics_agent import MetricsAgent
    from utils.mock_k8s_client import MockK8sClient

    rng = random.Random(7)
    out = {}
    # 1. per-pod thresholds over 100k pods
    P = 100_000
    pm = {f"pod-{i:06d}": {"cpu": {"usage": "1m", "usage_percentage": rng.uniform(0, 100)},
                           "memory": {"usage": "1Mi", "usage_percentage": rng.uniform(0, 100)}} for i in range(P)}
    ma = MetricsAgent(DictClient(pod_metrics=pm))
    r = timed(lambda: ma.analyze("ns"))
    r.update(units=P, unit="pods", per_s=P / r["median_s"])
    out["metrics_thresholds_100k"] = r
    # 2. 13-pattern line histogram over one 100k-line container
    text = gen_container_text(random.Random(11), 100_000)
    L = len(text.splitlines())
    la = LogsAgent(DictClient())

    def logs():
        la.reset()
        la._analyze_container_logs("pod", "c", text)
    r = timed(logs, warmup=2, runs=20)
    r.update(units=L, unit="lines", per_s=L / r["median_s"])
    out["logs_13_patterns_100k"] = r
    # 3. betweenness (the SPOF check's networkx call)
    g = nx.gnm_random_graph(1000, 2000, seed=3, directed=True)
    r = timed(lambda: nx.betweenness_centrality(g), warmup=2, runs=20)
    r.update(units=1000, unit="nodes")
    out["betweenness_1k"] = r

    # 4. the whole comprehensive analysis on the C1 mock (shimmed: SURVEY.md §8c test double)
    class Shim(MockK8sClient):
        def get_recently_terminated_pods(self, namespace):
            return []

        def get_pod_logs(self, pod_name, namespace, container_name=None, tail_lines=100, previous=False):
            return MockK8sClient.get_pod_logs(self, namespace, pod_name, container_name, tail_lines, previous)
    co = Coordinator(Shim())
    r = timed(lambda: co.run_analysis("comprehensive", "test-microservices"))
    r.update(units=1, unit="analyses")
    out["comprehensive_c1"] = r
    res = {"host": {"cpu_model": lscpu_model(), "cores_used": 1, "python": platform.python_version(),
                    "networkx": nx.__version__, "nproc": os.cpu_count()},
           "protocol": "5 warm-up runs (2 for the >1 s probes), 20 timed; median and p95; single thread",
           "timings": out}
    path = os.path.join(HERE, "ref_cpu_timings.json")
    with open(path, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
