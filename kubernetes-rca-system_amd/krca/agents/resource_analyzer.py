"""ResourceAnalyzer (host, first slice): namespace resource health.

Reference: ref:agents/resource_analyzer.py:15-959, called by the UI path through
``MCPCoordinator.run_resource_analysis`` (ref:agents/mcp_coordinator.py:590).  The per-pod
categorisation (``_analyze_pods`` :264-380 with ``_is_pod_healthy`` :856-895)
runs on the device: the pods are encoded once into columnar status (krca/podstate.py) and
krca_pod_classify returns each pod's group memberships; the group lists keep the reference's
order and its quirks (a pod can sit in both the ``failed`` and ``error`` groups and is then
reported twice; the non-standard phase ``CrashLoopBackOff`` is not categorised).  The per-group
findings stay on the host.  The reference's ``logging`` to a file in the CWD is not reproduced.
"""
import json
from datetime import datetime

from .. import podstate, topograph

_RELATION_KEYWORDS = {  # ref :774-781
    'crash': ['backoff', 'crash', 'exit', 'fail', 'error'],
    'scheduling': ['schedule', 'resource', 'affinity', 'taint', 'toleration'],
    'volume': ['volume', 'mount', 'pvc', 'storage'],
    'image': ['image', 'pull', 'registry', 'repo'],
    'network': ['network', 'connect', 'route', 'ingress', 'service'],
    'resource': ['cpu', 'memory', 'limit', 'request', 'oom'],
}


class ResourceAnalyzer:
    def __init__(self, k8s_client, engine=None):
        self.k8s_client = k8s_client
        self._engine = engine
        self.findings = []
        self.reasoning_steps = []

    def add_finding(self, component, issue, severity, evidence, recommendation):
        self.findings.append({'component': component, 'issue': issue, 'severity': severity, 'evidence': evidence,
                              'recommendation': recommendation, 'timestamp': datetime.now().isoformat()})

    def add_reasoning_step(self, observation, conclusion):
        self.reasoning_steps.append({'observation': observation, 'conclusion': conclusion,
                                     'timestamp': datetime.now().isoformat()})

    def _kubectl_items(self, kind, namespace):
        try:
            r = self.k8s_client._run_kubectl_command(["get", kind, "-n", namespace, "-o", "json"])
            return json.loads(r['output'])['items'] if r['success'] else []
        except Exception:
            return []

    def analyze_namespace_resources(self, namespace):  # ref :32-94
        c = self.k8s_client
        services = c.get_services(namespace)
        deployments = c.get_deployments(namespace)
        pods = c.get_pods(namespace)
        events = c.get_events(namespace)
        statefulsets = self._kubectl_items("statefulsets", namespace)
        daemonsets = self._kubectl_items("daemonsets", namespace)
        self._kubectl_items("cronjobs", namespace)
        self._analyze_services(services, namespace)
        self._analyze_deployments(deployments)
        self._analyze_statefulsets(statefulsets)
        self._analyze_daemonsets(daemonsets)
        self._analyze_pods(pods, namespace)
        self._correlate_with_events(events)
        return {'namespace': namespace,
                'resource_count': {'services': len(services), 'deployments': len(deployments),
                                   'statefulsets': len(statefulsets), 'daemonsets': len(daemonsets),
                                   'pods': len(pods)},
                'findings': self.findings, 'reasoning_steps': self.reasoning_steps}

    def _analyze_services(self, services, namespace):  # ref :96-148
        device = self._service_matches(services, namespace)
        for si, s in enumerate(services):
            name = s['metadata']['name']
            s['spec'].get('type', 'ClusterIP')
            sel = s['spec'].get('selector', {})
            comp = f"Service/{name}"
            if not sel:
                self.add_finding(comp, "Service has no selector", "medium",
                                 "No pod selector specified in service definition",
                                 "Add appropriate selectors to match target pods")
                continue
            matching = device[si] if device is not None else self._find_matching_pods(namespace, sel)
            if not matching:
                self.add_finding(comp, "Service selector matches no pods", "high",
                                 f"Selector {sel} does not match any pods in the namespace",
                                 "Verify selector labels or check if pods are running")
                continue
            bad = [p['metadata']['name'] for p in matching if not self._is_pod_healthy(p)]
            if bad:
                self.add_finding(comp, "Service targets unhealthy pods", "high",
                                 f"Pods {', '.join(bad)} matched by this service are unhealthy",
                                 "Investigate pod issues to restore service functionality")

    def _analyze_deployments(self, deployments):  # ref :150-196
        for d in deployments:
            name = d['metadata']['name']
            want = d['spec'].get('replicas', 0)
            avail = d['status'].get('availableReplicas', 0)
            ready = d['status'].get('readyReplicas', 0)
            unavail = d['status'].get('unavailableReplicas', 0)
            comp = f"Deployment/{name}"
            if ready < want:
                self.add_finding(comp, f"Deployment has {ready}/{want} ready replicas",
                                 "high" if ready == 0 else "medium",
                                 f"Status: {ready} ready, {avail} available, {unavail} unavailable of {want} desired",
                                 "Investigate pod creation issues or container problems")
            try:
                sel = d['spec'].get('selector', {}).get('matchLabels', {})
                tl = d['spec'].get('template', {}).get('metadata', {}).get('labels', {})
                if any(k not in tl or tl[k] != v for k, v in sel.items()):
                    self.add_finding(comp, "Deployment selector doesn't match template labels", "high",
                                     f"Selector {sel} doesn't match pod template labels {tl}",
                                     "Correct the selector to match pod template labels")
            except Exception:
                pass

    def _analyze_statefulsets(self, sts):  # ref :198-234
        for s in sts:
            name = s['metadata']['name']
            want = s['spec'].get('replicas', 0)
            ready = s['status'].get('readyReplicas', 0)
            if ready < want:
                self.add_finding(f"StatefulSet/{name}", f"StatefulSet has {ready}/{want} ready replicas",
                                 "high" if ready == 0 else "medium", f"Status: {ready} ready of {want} desired",
                                 "Check for persistent volume issues or pod scheduling problems")
            if not s['spec'].get('volumeClaimTemplates', []):
                self.add_finding(f"StatefulSet/{name}", "StatefulSet doesn't define persistent volume claim templates",
                                 "low", "No volumeClaimTemplates found in the StatefulSet definition",
                                 "Consider adding persistent storage for stateful applications")

    def _analyze_daemonsets(self, dss):  # ref :236-262
        for d in dss:
            name = d['metadata']['name']
            want = d['status'].get('desiredNumberScheduled', 0)
            cur = d['status'].get('currentNumberScheduled', 0)
            ready = d['status'].get('numberReady', 0)
            if ready < want:
                self.add_finding(f"DaemonSet/{name}", f"DaemonSet has {ready}/{want} ready pods",
                                 "high" if ready == 0 else "medium",
                                 f"Status: {ready} ready, {cur} scheduled of {want} desired",
                                 "Check for node taints or affinity issues")

    # -- pod categorisation (ref :264-380) -------------------------------------------------
    def _eng(self):
        if self._engine is None:
            from ..native import default_engine
            self._engine = default_engine()
        return self._engine

    def categorize_pods(self, pods):
        """status_groups of ref :274-343, from the device's per-pod group masks."""
        mask, _ = self._eng().pod_classify(*podstate.encode_pods(pods))
        return podstate.groups_from_masks(pods, mask)

    def _analyze_pods(self, pods, namespace):
        g = self.categorize_pods(pods)
        self._pending(g['pending'])
        self._failing(g['failed'] + g['error'])
        self._crashloop(g['crashloopbackoff'], namespace, "Container in CrashLoopBackOff with {n} restarts",
                        "Check container logs for application errors and fix the root cause", 'containerStatuses')
        self._imagepull(g['imagepullbackoff'])
        self._creating(g['containercreating'])
        self._crashloop(g['init_crashloopbackoff'], namespace, "Init container in CrashLoopBackOff with {n} restarts",
                        "Check init container logs and fix initialization errors", 'initContainerStatuses')
        self._not_ready(g['not_ready'])
        self._evicted(g['evicted'])
        bad = sum(len(v) for k, v in g.items() if k not in ('running', 'succeeded'))
        if bad > 0:
            self.add_finding(f"Namespace/{namespace}", f"Found {bad} pods with issues", "high" if bad > 5 else "medium",
                             self._format_pod_status_evidence(g),
                             "Investigate pod issues based on their specific error states")

    def _pending(self, pods):
        for pod in pods:
            for cond in pod['status'].get('conditions', []):
                if (cond.get('type') == 'PodScheduled' and cond.get('status') == 'False'
                        and cond.get('reason', '') == 'Unschedulable'):
                    self.add_finding(f"Pod/{pod['metadata']['name']}", "Pod cannot be scheduled", "high",
                                     f"Message: {cond.get('message', '')}",
                                     "Check node resources, taints, tolerations, and node selectors")

    def _failing(self, pods):
        for pod in pods:
            for cs in pod['status'].get('containerStatuses', []):
                state = cs.get('state', {})
                if 'terminated' in state:
                    t = state['terminated']
                    self.add_finding(f"Pod/{pod['metadata']['name']}/{cs.get('name', '')}",
                                     f"Container terminated with exit code {t.get('exitCode', 0)}", "high",
                                     f"Reason: {t.get('reason', '')}, Message: {t.get('message', '')}",
                                     "Check container logs and fix application errors")

    def _crashloop(self, pods, namespace, issue, rec, key):
        for pod in pods:
            pname = pod['metadata']['name']
            for cs in pod['status'].get(key, []):
                cname = cs.get('name', '')
                n = cs.get('restartCount', 0)
                if n <= 0:
                    continue
                term = cs.get('lastState', {}).get('terminated', {})
                self.add_finding(f"Pod/{pname}/{cname}", issue.format(n=n), "high",
                                 f"Last exit code: {term.get('exitCode', 'unknown')}, reason: {term.get('reason', 'unknown')}",
                                 rec)
                try:  # the reference only logs these (ref :498-504)
                    self.k8s_client.get_pod_logs(pname, namespace, cname, tail_lines=50)
                except Exception:
                    pass

    def _imagepull(self, pods):
        for pod in pods:
            for cs in pod['status'].get('containerStatuses', []):
                w = cs.get('state', {}).get('waiting', {})
                if w.get('reason', '') in ('ImagePullBackOff', 'ErrImagePull'):
                    self.add_finding(f"Pod/{pod['metadata']['name']}/{cs.get('name', '')}",
                                     f"Cannot pull image: {cs.get('image', '')}", "high",
                                     f"Message: {w.get('message', '')}",
                                     "Verify image name, tag, and registry credentials")

    def _creating(self, pods):
        for pod in pods:
            pvcs = [v for v in pod['spec'].get('volumes', []) if 'persistentVolumeClaim' in v]
            if pvcs:
                names = ', '.join(v.get('persistentVolumeClaim', {}).get('claimName', '') for v in pvcs)
                ev, rec = f"Pod uses PVCs: {names} which may be pending", "Check PVC status and storage provisioner"
            else:
                ev = "Pod has been in ContainerCreating state for an extended period"
                rec = "Check for resource constraints or image pull issues"
            self.add_finding(f"Pod/{pod['metadata']['name']}", "Pod stuck in ContainerCreating state", "medium", ev, rec)

    def _not_ready(self, pods):
        for pod in pods:
            pname = pod['metadata']['name']
            for ctr in pod['spec'].get('containers', []):
                cname = ctr.get('name', '')
                if not ctr.get('readinessProbe'):
                    self.add_finding(f"Pod/{pname}/{cname}", "Container has no readiness probe", "low",
                                     "No readiness probe specified in container definition",
                                     "Add appropriate readiness probe to container")
                    continue
                cs = next((s for s in pod['status'].get('containerStatuses', []) if s.get('name') == cname), None)
                if cs and not cs.get('ready', False):
                    self.add_finding(f"Pod/{pname}/{cname}", "Container not passing readiness probe", "medium",
                                     "Container is running but failing readiness checks",
                                     "Check application logs and fix readiness issues")

    def _evicted(self, pods):
        for pod in pods:
            self.add_finding(f"Pod/{pod['metadata']['name']}", "Pod has been evicted", "medium",
                             f"Eviction message: {pod['status'].get('message', 'Unknown reason')}",
                             "Check for resource constraints, particularly node disk pressure")

    # -- events (ref :714-833) -----------------------------------------------------------
    def _correlate_with_events(self, events):
        if not events:
            return
        by_obj = {}
        for e in events:
            o = e.get('involvedObject', {})
            kind, name = o.get('kind', ''), o.get('name', '')
            if kind and name:
                by_obj.setdefault(f"{kind}/{name}", []).append(e)
        for comp, evs in by_obj.items():
            existing = [f for f in self.findings if f['component'] == comp]
            if not existing:
                self._create_findings_from_events(comp, evs)
                continue
            for f in existing:
                rel = [e for e in evs if self._is_event_related_to_finding(e, f)]
                if rel:
                    msgs = [f"{e.get('reason', '')}: {e.get('message', '')}" for e in rel[:3]]
                    f['evidence'] += f"\nRelated events: {' | '.join(msgs)}"

    @staticmethod
    def _is_event_related_to_finding(event, finding):
        reason = event.get('reason', '').lower()
        msg = event.get('message', '').lower()
        issue = finding.get('issue', '').lower()
        kind = next((t for t, kws in _RELATION_KEYWORDS.items() if any(k in issue for k in kws)), None)
        return bool(kind) and any(k in reason or k in msg for k in _RELATION_KEYWORDS[kind])

    def _create_findings_from_events(self, comp, evs):
        groups = {}
        for e in evs:
            if e.get('type', '') != 'Normal':
                groups.setdefault(e.get('reason', 'Unknown'), []).append(e)
        for reason, lst in groups.items():
            last = max(lst, key=lambda e: e.get('lastTimestamp', ''))
            self.add_finding(comp, f"Event warning: {reason}",
                             "high" if reason in ('Failed', 'FailedCreate', 'FailedMount') else "medium",
                             f"Message: {last.get('message', '')} (event count: {len(lst)})",
                             "Investigate the reported issue and take appropriate action")

    def _service_matches(self, services, namespace):
        """Every service's matching pods (the O(S*P) loop of _find_matching_pods, ref :835-854)
        from one krca_selector_match launch over (pod, service) pairs; the pod list is fetched
        once instead of once per service.  None -> the per-service host loop (inputs that are not
        plain dicts keep the reference's own errors)."""
        try:
            sels = [s['spec'].get('selector', {}) for s in services]
            if not any(sels) or not all(isinstance(x, dict) for x in sels):
                return None
            pods = self.k8s_client.get_pods(namespace)
            labels = [p['metadata'].get('labels', {}) for p in pods]
        except Exception:
            return None
        if not pods or not all(isinstance(x, dict) for x in labels):
            return None
        bits = topograph.selector_bits(self._eng(), [x.items() for x in labels], [x.items() for x in sels],
                                       identity=False)
        cols = topograph.match_cols(bits, len(services))
        return [[pods[i] for i in c] for c in cols]

    def _find_matching_pods(self, namespace, selector):
        return [p for p in self.k8s_client.get_pods(namespace)
                if all(k in p['metadata'].get('labels', {}) and p['metadata']['labels'][k] == v
                       for k, v in selector.items())]

    @staticmethod
    def _is_pod_healthy(pod):  # ref :856-895
        st = pod['status']
        if st.get('phase', '') != 'Running':
            return False
        ready = next((c for c in st.get('conditions', []) if c.get('type') == 'Ready'), None)
        if not ready or ready.get('status') != 'True':
            return False
        css = st.get('containerStatuses', [])
        if not css:
            return False
        for cs in css:
            if not cs.get('ready', False):
                return False
            state = cs.get('state', {})
            if 'waiting' in state:
                return False
            if 'terminated' in state and state['terminated'].get('reason', '') != 'Completed':
                return False
        return True

    @staticmethod
    def _format_pod_status_evidence(groups):
        out = []
        for status, pods in groups.items():
            if status in ('running', 'succeeded') or not pods:
                continue
            names = ", ".join(p['metadata']['name'] for p in pods[:5])
            if len(pods) > 5:
                names += f" and {len(pods) - 5} more"
            out.append(f"{status.replace('_', ' ').title()}: {names}")
        return "\n".join(out)
