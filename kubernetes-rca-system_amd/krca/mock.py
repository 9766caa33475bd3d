"""Offline fixture cluster (config C1).

``MockK8sClient`` serves the reference's demo cluster (ref:utils/mock_k8s_client.py:7-1311)
from ``data/mock_cluster.json`` — data captured from the reference by
``tests/golden/capture_reference.py``; no reference code lives here.  The reference's API
quirks are kept on purpose because parity depends on them:

* no ``get_recently_terminated_pods`` (so ``LogsAgent.analyze`` fails on the raw mock),
* ``get_pod_logs(namespace, pod_name, ...)`` argument order (the agents call it with
  ``(pod, namespace, container)``, so every call returns the "No logs" string),
* no ``get_services_by_label`` (``TracesAgent`` records three reasoning-step errors).
"""
import copy
import json
import os
from datetime import datetime

_DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "mock_cluster.json")


def load_cluster(path=_DATA):
    with open(path) as f:
        return json.load(f)


class MockK8sClient:
    def __init__(self, use_mock=True, data=None):
        self.use_mock = use_mock
        self.connected = True
        d = copy.deepcopy(data if data is not None else load_cluster())
        self._d = d
        self.current_context = d["current_context"]
        self.available_contexts = list(d["available_contexts"])
        self.namespaces = d["namespaces"]
        self.pods = d["pods"]
        self.services = d["services"]
        self.deployments = d["deployments"]
        self.pod_metrics = d["pod_metrics"]
        self.node_metrics = d["node_metrics"]
        self.events = d["events"]
        self.logs = d["logs"]
        self.network_policies = d["network_policies"]
        self.endpoints = d["endpoints"]
        self.hpas = d["hpas"]

    # -- context ----------------------------------------------------------------------
    def is_connected(self):
        return self.connected

    def get_available_contexts(self):
        return self.available_contexts

    def get_current_context(self):
        return self.current_context

    def set_context(self, context_name):
        if context_name not in self.available_contexts:
            return False
        self.current_context = context_name
        return True

    def get_current_time(self):
        return datetime.now().isoformat()

    # -- namespaced collections (ref:utils/mock_k8s_client.py:843-1134) ------------------
    def get_namespaces(self):
        return self.namespaces

    def get_pods(self, namespace):
        return self.pods.get(namespace, [])

    def get_services(self, namespace):
        return self.services.get(namespace, [])

    def get_deployments(self, namespace):
        return self.deployments.get(namespace, [])

    def get_node_metrics(self):
        return self.node_metrics

    def get_pod_metrics(self, namespace):
        return self.pod_metrics.get(namespace, {})

    def get_network_policies(self, namespace):
        return self.network_policies.get(namespace, [])

    def get_hpas(self, namespace):
        return self.hpas.get(namespace, [])

    def get_ingresses(self, namespace):
        return []

    def get_configmaps(self, namespace):
        return []

    def get_secrets(self, namespace):
        return []

    def get_statefulsets(self, namespace):
        return []

    def get_resource_quotas(self, namespace):
        return []

    def get_pod_logs(self, namespace, pod_name, container_name=None, tail_lines=100, previous=False):
        per_ns = self.logs.get(namespace)
        if per_ns is None or pod_name not in per_ns:
            return "No logs available for this pod"
        pod_logs = per_ns[pod_name]
        if container_name and container_name in pod_logs:
            return pod_logs[container_name]
        if container_name:
            return f"Container {container_name} not found in pod {pod_name}"
        return next(iter(pod_logs.values()), "No logs available for this pod")

    def get_events(self, namespace, field_selector=None, limit=None):
        events = self.events.get(namespace, [])
        if field_selector:
            kind = name = None
            has_kind = "involvedObject.kind" in field_selector
            has_name = "involvedObject.name" in field_selector
            if has_kind:
                kind = field_selector.split("involvedObject.kind=")[1]
                if has_name:
                    kind = kind.split(",")[0]
            if has_name:
                name = field_selector.split("involvedObject.name=")[1]
            events = [e for e in events
                      if (kind is None or e["involvedObject"]["kind"] == kind)
                      and (name is None or e["involvedObject"]["name"] == name)]
        if limit and limit < len(events):
            events = events[:limit]
        return events

    def get_endpoints(self, namespace, name):
        return self.endpoints.get(namespace, {}).get(name)

    def _find(self, table, namespace, name):
        for obj in table.get(namespace, []):
            if obj["metadata"]["name"] == name:
                return obj
        return None

    def get_pod_status(self, namespace, pod_name):
        return self._find(self.pods, namespace, pod_name)

    def get_service(self, namespace, service_name):
        return self._find(self.services, namespace, service_name)

    def get_deployment(self, namespace, deployment_name):
        return self._find(self.deployments, namespace, deployment_name)

    # -- trace-backend stubs (ref:utils/mock_k8s_client.py:1146-1309) ---------------------
    def get_trace_ids(self, service_name=None, error_only=False, limit=10):
        return self._d["trace_ids"][:limit]

    def get_trace_details(self, trace_id):
        d = copy.deepcopy(self._d["trace_details_template"])
        d["traceId"] = trace_id
        return d

    def get_service_latency_stats(self, service_name=None, time_range_minutes=30):
        stats = self._d["service_latency_stats"]
        if service_name and service_name in stats:
            return {service_name: stats[service_name]}
        return stats

    def get_error_rate_by_service(self, time_range_minutes=30):
        return dict(self._d["error_rate_by_service"])

    def get_service_dependencies(self, service_name=None):
        deps = self._d["service_dependencies"]
        if service_name and service_name in deps:
            return {service_name: deps[service_name]}
        return deps

    def find_slow_operations(self, threshold_ms=1000, time_range_minutes=30):
        return copy.deepcopy(self._d["slow_operations"])

    def are_traces_available(self):
        return True


class MeshClient(MockK8sClient):
    """The mock cluster with a synthetic pod mesh behind the bulk accessors:
    ``get_pod_metric_tensor`` serves the [T][P][M] metric tensor (device or host) and
    ``get_dependency_csr`` the pull-CSR of the mesh (krca.synth.Mesh), so the Coordinator's
    comprehensive run scores the mesh and ranks its pods; the dict methods keep serving the C1
    objects.  Used to check that ``ranked_root_causes`` equals the bench / RcaStep ranking."""

    def __init__(self, mesh, x, names=None, **kw):
        super().__init__(**kw)
        self.mesh, self.x = mesh, x
        self._mesh_names = names

    def get_pod_metric_tensor(self, namespace):
        return (self._mesh_names or self.mesh.names()), self.x

    def get_dependency_csr(self, namespace):
        m = self.mesh
        return (self._mesh_names or m.names()), m.row_ptr, m.col, m.outdeg
