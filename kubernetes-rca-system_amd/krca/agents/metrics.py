"""MetricsAgent: per-pod usage thresholds (+ rolling z-score anomalies on the bulk path).

Reference: ref:agents/metrics_agent.py:4-365.  The per-pod threshold scans
(``_analyze_cpu_usage`` :69-114, ``_analyze_memory_usage`` :116-161) are the hot loops; here
they are one device pass (``krca_usage_flags`` / ``krca_rolling_score``) and the host only
formats the findings for the flagged pods, in pod order, with the reference's strings.

Node pressure (:163-209), resource configuration (:211-277) and HPA checks (:279-365) are
dict walks over a handful of objects and stay on the host.

Bulk path (additive): when the client exposes
``get_pod_metric_tensor(namespace) -> (pod_names, x)`` with ``x`` a float32 device tensor laid
out ``[T][P][M]`` (time-major; channel 0 = CPU %, channel 1 = memory %), the thresholds read the
last sample and the rolling z-score kernel adds the ``anomalies`` key (schema of
ref:agent_coordinator.py:113-115: resource / description / severity / deviation).
"""
import numpy as np

from .base import BaseAgent

CPU_CH, MEM_CH = 0, 1
# flag bits produced by the device kernels (include/krca.h)
F_CPU80, F_CPU90, F_MEM80, F_MEM90 = 1, 2, 4, 8


def to_f32_threshold_safe(values):
    """float64 -> float32 such that every ``> 80`` and ``> 90`` test keeps its float64 answer.

    Rounding to nearest is monotone and 80/90 are exact in float32, so the only flip is a
    value just above a threshold rounding down onto it; such values are nudged one ulp up.
    """
    v = np.asarray(values, dtype=np.float64)
    f = v.astype(np.float32)
    for t in (80.0, 90.0):
        bump = (v > t) & (f <= np.float32(t))
        f[bump] = np.nextafter(np.float32(t), np.float32(np.inf))
    return f


class MetricsAgent(BaseAgent):
    def __init__(self, k8s_client, engine=None, window=60, z_threshold=3.0, anomaly_topk=10):
        super().__init__(k8s_client, engine)
        self.window = window
        self.z_threshold = z_threshold
        self.anomaly_topk = anomaly_topk
        self.last_scores = None  # device outputs of the last bulk run (used by the Coordinator)

    # ------------------------------------------------------------------------------------
    def analyze(self, namespace, context=None, **kwargs):
        self.reset()
        self.last_scores = None
        try:
            self._maybe_set_context(context)
            bulk = getattr(self.k8s_client, "get_pod_metric_tensor", None)
            anomalies = None
            if bulk is not None:
                names, x = bulk(namespace)
                pods, flags, anomalies = self._score_tensor(names, x)
            else:
                pod_metrics = self.k8s_client.get_pod_metrics(namespace)
                pods, flags = self._score_dict(pod_metrics)
            node_metrics = self.k8s_client.get_node_metrics()
            self._report_usage(pods, flags, "CPU", "cpu", CPU_CH, F_CPU80, F_CPU90)
            self._report_usage(pods, flags, "memory", "memory", MEM_CH, F_MEM80, F_MEM90)
            self._analyze_node_resources(node_metrics)
            self._analyze_resource_configurations(namespace)
            self._analyze_hpa_configurations(namespace)
            res = self.get_results()
            if anomalies is not None:
                res["anomalies"] = anomalies
            return res
        except Exception as e:  # ref:agents/metrics_agent.py:58-67
            return self._error_result("metrics", e)

    # -- dict path (C1): usage_percentage per pod ----------------------------------------
    def _score_dict(self, pod_metrics):
        names = list(pod_metrics.keys())
        if not names:
            return [], None
        raw = np.zeros((len(names), 2), dtype=np.float64)
        for i, n in enumerate(names):
            m = pod_metrics[n]
            raw[i, 0] = m.get("cpu", {}).get("usage_percentage", 0)
            raw[i, 1] = m.get("memory", {}).get("usage_percentage", 0)
        usage = to_f32_threshold_safe(raw)
        flags = self.engine.usage_flags(usage)
        # evidence is printed from the caller's own values, exactly as the reference does
        pods = [(n,
                 pod_metrics[n].get("cpu", {}).get("usage_percentage", 0),
                 pod_metrics[n].get("memory", {}).get("usage_percentage", 0)) for n in names]
        return pods, flags

    # -- bulk path (C2-C5): [T][P][M] float32 device tensor ------------------------------
    def _score_tensor(self, names, x):
        T, P, M = x.shape
        if P == 0:
            return [], None, []
        out = self.engine.rolling_score(x, window=self.window, z_threshold=self.z_threshold)
        self.last_scores = out
        flags = out["flags"]
        flagged = np.nonzero(flags & (F_CPU80 | F_MEM80))[0]
        last = self.engine.gather_last(x, flagged)  # [n_flagged, M] float32 host copy
        lut = {int(p): last[i] for i, p in enumerate(flagged)}
        pods = _LazyPods(names, lut)
        anomalies = []
        k = min(self.anomaly_topk, P)
        idx, val = self.engine.topk(out["score"], k)
        for p, s in zip(idx.tolist(), val.tolist()):
            if not s > self.z_threshold:
                break
            anomalies.append({
                "resource": f"Pod/{names[p]}",
                "description": (f"Rolling z-score {s:.2f} over a {self.window}-step window; "
                                f"{int(out['n_exceed_host'][p])} samples beyond |z|>{self.z_threshold:g}"),
                "severity": "high" if s > 2 * self.z_threshold else "medium",
                "deviation": float(s),
            })
        return pods, flags, anomalies

    # -- shared reporting (ref:agents/metrics_agent.py:69-161) ---------------------------
    def _report_usage(self, pods, flags, label, key, ch, f80, f90):
        if not len(pods):
            self.add_reasoning_step(observation=f"No {label} metrics data available",
                                    conclusion=f"Unable to analyze {label} usage")
            return
        self.add_reasoning_step(observation=f"Analyzing {label} usage for {len(pods)} pods",
                                conclusion=f"Beginning {label} usage analysis")
        hit = np.nonzero(flags & f80)[0]
        if len(hit):
            sel = [pods[int(i)] for i in hit]
            vals = [(p[0], p[1 + ch]) for p in sel]
            pod_list = ", ".join(f"{name} ({usage:.1f}%)" for name, usage in vals)
            severe = bool(np.any(flags[hit] & f90))
            if ch == CPU_CH:
                self.add_finding(
                    component="Pods CPU Usage",
                    issue=f"High CPU usage detected in {len(vals)} pods",
                    severity="high" if severe else "medium",
                    evidence=f"Pods with high CPU usage: {pod_list}",
                    recommendation="Consider scaling these deployments or optimizing the application code")
                self.add_reasoning_step(
                    observation=f"Detected {len(vals)} pods with CPU usage above 80%",
                    conclusion="High CPU usage may indicate resource constraints or inefficient application code")
            else:
                self.add_finding(
                    component="Pods Memory Usage",
                    issue=f"High memory usage detected in {len(vals)} pods",
                    severity="high" if severe else "medium",
                    evidence=f"Pods with high memory usage: {pod_list}",
                    recommendation="Consider increasing memory limits, scaling horizontally, or investigating memory leaks")
                self.add_reasoning_step(
                    observation=f"Detected {len(vals)} pods with memory usage above 80%",
                    conclusion="High memory usage may indicate memory leaks or insufficient resource allocation")
        else:
            self.add_reasoning_step(observation=f"No pods with high {label} usage detected",
                                    conclusion=f"{label[0].upper() + label[1:]} usage appears to be within acceptable limits")

    # -- node pressure: 3 nodes in C1, host (ref:agents/metrics_agent.py:163-209) --------
    def _analyze_node_resources(self, node_metrics):
        if not node_metrics:
            self.add_reasoning_step(observation="No node metrics data available",
                                    conclusion="Unable to analyze node resource usage")
            return
        self.add_reasoning_step(observation=f"Analyzing resource usage for {len(node_metrics)} nodes",
                                conclusion="Beginning node resource analysis")
        pressured = []
        for node, m in node_metrics.items():
            c = m.get("cpu", {}).get("usage_percentage", 0)
            mem = m.get("memory", {}).get("usage_percentage", 0)
            if c > 80 or mem > 80:
                pressured.append((node, c, mem))
        if not pressured:
            self.add_reasoning_step(observation="No nodes with high resource pressure detected",
                                    conclusion="Node resource usage appears to be within acceptable limits")
            return
        listing = ", ".join(f"{n} (CPU: {c:.1f}%, Memory: {mem:.1f}%)" for n, c, mem in pressured)
        self.add_finding(
            component="Node Resources",
            issue=f"Resource pressure detected on {len(pressured)} nodes",
            severity="high" if any(c > 90 or mem > 90 for _, c, mem in pressured) else "medium",
            evidence=f"Nodes under resource pressure: {listing}",
            recommendation="Consider adding more nodes to the cluster or optimizing workload distribution")
        self.add_reasoning_step(
            observation=f"Detected {len(pressured)} nodes with high resource usage",
            conclusion="Node resource pressure may be affecting overall cluster performance and pod scheduling")

    # -- requests/limits (ref:agents/metrics_agent.py:211-277) ---------------------------
    def _analyze_resource_configurations(self, namespace):
        try:
            deployments = self.k8s_client.get_deployments(namespace)
            if not deployments:
                self.add_reasoning_step(observation=f"No deployments found in namespace {namespace}",
                                        conclusion="Unable to analyze resource configurations")
                return
            self.add_reasoning_step(
                observation=f"Analyzing resource configurations for {len(deployments)} deployments",
                conclusion="Beginning resource configuration analysis")
            missing = []
            for d in deployments:
                dname = d["metadata"]["name"]
                for c in d["spec"]["template"]["spec"]["containers"]:
                    res = c.get("resources", {})
                    req, lim = ("requests" in res), ("limits" in res)
                    complete = (req and "cpu" in res["requests"] and "memory" in res["requests"]
                                and lim and "cpu" in res["limits"] and "memory" in res["limits"])
                    if not complete:
                        missing.append(f"{dname}/{c['name']}")
            if missing:
                self.add_finding(
                    component="Resource Configuration",
                    issue=f"Missing resource requests or limits in {len(missing)} containers",
                    severity="medium",
                    evidence=f"Containers with missing resource configurations: {', '.join(missing)}",
                    recommendation="Add appropriate CPU and memory requests and limits to all containers")
                self.add_reasoning_step(
                    observation=f"Detected {len(missing)} containers with missing resource configurations",
                    conclusion="Missing resource configurations can lead to resource contention and unpredictable behavior")
            else:
                self.add_reasoning_step(observation="All containers have resource requests and limits configured",
                                        conclusion="Resource configurations appear to be properly defined")
        except Exception as e:
            self.add_reasoning_step(observation=f"Error analyzing resource configurations: {str(e)}",
                                    conclusion="Unable to complete resource configuration analysis")

    # -- HPA (ref:agents/metrics_agent.py:279-365) ---------------------------------------
    _HPA_FINDINGS = {
        "at_max_capacity": ("HPA is at maximum capacity ({cur}/{mx} replicas)", "high",
                            "HPA {name} is running at maximum capacity of {mx} replicas",
                            "Consider increasing the maximum replicas for this HPA"),
        "narrow_range": ("HPA has a narrow scaling range ({mn}-{mx} replicas)", "low",
                         "HPA {name} has min={mn}, max={mx} replicas",
                         "Consider widening the scaling range to allow more flexibility"),
        "scaling_delay": ("HPA desired replicas not matching current replicas", "medium",
                          "HPA {name} has desired replicas > current replicas",
                          "Investigate potential issues preventing scaling or configure less aggressive scaling"),
    }

    def _analyze_hpa_configurations(self, namespace):
        try:
            hpas = self.k8s_client.get_hpas(namespace)
            if not hpas:
                self.add_reasoning_step(observation=f"No HPAs found in namespace {namespace}",
                                        conclusion="No autoscaling configurations to analyze")
                return
            self.add_reasoning_step(observation=f"Analyzing {len(hpas)} Horizontal Pod Autoscalers",
                                    conclusion="Beginning HPA configuration analysis")
            problems = []
            for h in hpas:
                name = h["metadata"]["name"]
                mn = h["spec"].get("minReplicas", 1)
                mx = h["spec"].get("maxReplicas", 1)
                cur = h["status"].get("currentReplicas", 0)
                want = h["status"].get("desiredReplicas", 0)
                if cur == mx and cur > 0:
                    problems.append(("at_max_capacity", name, mn, mx, cur))
                if mx - mn < 2 and mn > 1:
                    problems.append(("narrow_range", name, mn, mx, cur))
                if want > cur:
                    problems.append(("scaling_delay", name, mn, mx, cur))
            if problems:
                for kind, name, mn, mx, cur in problems:
                    issue, sev, ev, rec = self._HPA_FINDINGS[kind]
                    fmt = dict(name=name, mn=mn, mx=mx, cur=cur)
                    self.add_finding(component=f"HPA/{name}", issue=issue.format(**fmt), severity=sev,
                                     evidence=ev.format(**fmt), recommendation=rec)
                self.add_reasoning_step(
                    observation=f"Detected {len(problems)} HPAs with potential configuration issues",
                    conclusion="HPA configuration issues may be affecting the ability to scale effectively")
            else:
                self.add_reasoning_step(observation="All HPAs appear to be properly configured",
                                        conclusion="HPA configurations look appropriate for the current workload")
        except Exception as e:
            self.add_reasoning_step(observation=f"Error analyzing HPA configurations: {str(e)}",
                                    conclusion="Unable to complete HPA configuration analysis")


class _LazyPods:
    """Sequence view over a million-pod tensor: only flagged rows are ever materialised."""

    def __init__(self, names, last_by_pod):
        self.names = names
        self.last = last_by_pod

    def __len__(self):
        return len(self.names)

    def __getitem__(self, p):
        row = self.last[p]
        return (self.names[p], float(row[CPU_CH]), float(row[MEM_CH]))
