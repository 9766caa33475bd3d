"""EventsAgent (host): group-bys over a namespace's events.

Reference: ref:agents/events_agent.py:4-446.  Out of the hot-path scope (SURVEY.md §2 row 9;
§8f f4 lists a device group-by as a later step); kept on the host with identical findings so
``Coordinator.run_analysis('comprehensive')`` correlates the same five finding lists.
"""
from .base import BaseAgent

CRITICAL_REASONS = ('Failed', 'FailedCreate', 'FailedScheduling', 'FailedMount', 'NodeNotReady',
                    'KubeletNotReady', 'FailedAttachVolume', 'FailedDetachVolume', 'FreeDiskSpaceFailed',
                    'OutOfDisk', 'MemoryPressure', 'DiskPressure', 'NetworkUnavailable', 'Unhealthy',
                    'FailedSync', 'Evicted', 'BackOff', 'Error')  # ref:agents/events_agent.py:28-34

# (predicate on message, cause, recommendation) in priority order (ref :201-215, :266-277)
_SCHED_CAUSES = (
    (lambda m: "Insufficient cpu" in m, "insufficient CPU", "Increase CPU capacity in your cluster or reduce CPU requests"),
    (lambda m: "Insufficient memory" in m, "insufficient memory", "Increase memory capacity in your cluster or reduce memory requests"),
    (lambda m: "node(s) had taint" in m, "node taints", "Add appropriate tolerations to the pod or remove taints from nodes"),
    (lambda m: "node(s) didn't match node selector" in m, "node selector mismatch", "Update the pod's node selector or label your nodes correctly"),
    (lambda m: "persistentvolumeclaim" in m.lower() and "pending" in m.lower(), "pending PVC", "Check the PVC status and ensure storage is available"),
)
_VOLUME_CAUSES = (
    (lambda m: "timeout" in m, "mounting timeout", "Check if storage system is responsive and resources are available"),
    (lambda m: "no such file" in m, "path doesn't exist", "Verify the volume path exists in the source"),
    (lambda m: "permission denied" in m, "permission issue", "Check volume permissions and pod security context"),
    (lambda m: "not found" in m and "pvc" in m, "PVC not found", "Ensure the PVC exists and is in the correct namespace"),
)
_NODE_ISSUES = (("NotReady", "node not ready", "Check kubelet status, node connectivity, and system logs on the node"),
                ("MemoryPressure", "memory pressure", "Free up memory on the node or add more memory resources"),
                ("DiskPressure", "disk pressure", "Free up disk space on the node or expand storage"),
                ("NetworkUnavailable", "network unavailable", "Check network configuration, CNI plugins, and network connectivity"))
_CONTROL_PLANE = ('kube-apiserver', 'kube-controller-manager', 'kube-scheduler', 'etcd')
_NODE_REASONS = ('NodeNotReady', 'KubeletNotReady', 'MemoryPressure', 'DiskPressure', 'NetworkUnavailable')


def _group(items, key):
    out = {}
    for it in items:
        out.setdefault(key(it), []).append(it)
    return out


def _latest(evs):
    return max(evs, key=lambda e: e.get('lastTimestamp', ''))


def _obj_key(e):
    o = e.get('involvedObject', {})
    return f"{o.get('kind', 'Unknown')}/{o.get('name', 'unknown')}"


class EventsAgent(BaseAgent):
    def __init__(self, k8s_client, engine=None):
        super().__init__(k8s_client, engine)
        self.event_severity = {'Normal': 'info', 'Warning': 'medium', 'Error': 'high', 'Critical': 'critical'}
        self.critical_event_reasons = list(CRITICAL_REASONS)

    def analyze(self, namespace, context=None, **kwargs):
        self.reset()
        try:
            self._maybe_set_context(context)
            events = self.k8s_client.get_events(namespace)
            if not events:
                self.add_reasoning_step(observation=f"No events found in namespace {namespace}",
                                        conclusion="No event data to analyze")
                return self.get_results()
            self.add_reasoning_step(observation=f"Found {len(events)} events in namespace {namespace}",
                                    conclusion="Beginning events analysis")
            by_obj = _group(events, _obj_key)
            self.add_reasoning_step(observation=f"Grouped events into {len(by_obj)} unique objects",
                                    conclusion="Will analyze events by object type and name")
            self._object_warnings(by_obj)
            self._scheduling(events)
            self._volumes(events)
            self._frequent(events)
            self._control_plane(events)
            self._nodes(events)
            return self.get_results()
        except Exception as e:
            return self._error_result("events", e)

    def _object_warnings(self, by_obj):  # ref :136-167
        for key, evs in by_obj.items():
            warn = [e for e in evs if e.get('type', '') == 'Warning']
            if len(warn) < 3:
                continue
            recent = sorted(warn, key=lambda e: e.get('lastTimestamp', ''), reverse=True)[:3]
            reasons = [e.get('reason', 'Unknown') for e in recent]
            msgs = "\n".join(f"- {e.get('message', '')}" for e in recent)
            self.add_finding(component=key, issue=f"Multiple warning events detected for {key}",
                             severity="high" if any(r in self.critical_event_reasons for r in reasons) else "medium",
                             evidence=f"Recent warnings ({', '.join(reasons)}):\n{msgs}",
                             recommendation=f"Investigate the {key} resource for configuration or operational issues")
            self.add_reasoning_step(observation=f"Detected {len(warn)} warning events for {key}",
                                    conclusion=f"{key} is experiencing recurring issues")

    def _scheduling(self, events):  # ref :169-228
        sched = [e for e in events if e.get('reason', '') == 'FailedScheduling']
        for pod, evs in _group(sched, lambda e: e.get('involvedObject', {}).get('name', 'unknown')).items():
            msg = _latest(evs).get('message', '')
            cause, rec = "unknown", "Check node resources and pod resource requirements"
            for pred, c, r in _SCHED_CAUSES:
                if pred(msg):
                    cause, rec = c, r
                    break
            self.add_finding(component=f"Pod/{pod}", issue=f"Pod scheduling failed due to {cause}", severity="high",
                             evidence=f"Message: {msg}", recommendation=rec)
            self.add_reasoning_step(observation=f"Detected {len(evs)} scheduling failures for pod {pod}",
                                    conclusion=f"Pod {pod} cannot be scheduled due to {cause}")

    def _volumes(self, events):  # ref :230-290
        vol = [e for e in events if any(r in e.get('reason', '') for r in
                                        ('FailedMount', 'FailedAttachVolume', 'FailedDetachVolume'))]
        for key, evs in _group(vol, _obj_key).items():
            last = _latest(evs)
            reason, msg = last.get('reason', ''), last.get('message', '')
            cause, rec = "unknown issue", "Check the volume configuration and storage system"
            for pred, c, r in _VOLUME_CAUSES:
                if pred(msg.lower()):
                    cause, rec = c, r
                    break
            self.add_finding(component=key, issue=f"Volume operation failed due to {cause}", severity="high",
                             evidence=f"Reason: {reason}, Message: {msg}", recommendation=rec)
            self.add_reasoning_step(observation=f"Detected {len(evs)} volume issues for {key}",
                                    conclusion=f"{key} is experiencing volume issues: {cause}")

    def _frequent(self, events):  # ref :292-328
        hot = [e for e in events if e.get('count', 1) > 5]
        hot.sort(key=lambda e: e.get('count', 1), reverse=True)
        for e in hot[:5]:
            if e.get('type', 'Normal') != 'Warning':
                continue
            count = e.get('count', 0)
            o = e.get('involvedObject', {})
            kind, name = o.get('kind', 'Unknown'), o.get('name', 'unknown')
            reason = e.get('reason', 'Unknown')
            self.add_finding(component=f"{kind}/{name}",
                             issue=f"Frequent {reason} events detected ({count} occurrences)",
                             severity="high" if count > 20 else "medium",
                             evidence=f"Message: {e.get('message', '')}",
                             recommendation=f"Investigate the root cause of these recurring events on {kind} {name}")
            self.add_reasoning_step(observation=f"Detected {count} occurrences of {reason} events for {kind}/{name}",
                                    conclusion="Recurring events indicate a persistent issue that needs attention")

    def _control_plane(self, events):  # ref :330-375
        cp = [e for e in events if any(c in e.get('source', {}).get('component', '') for c in _CONTROL_PLANE)]
        for comp, evs in _group(cp, lambda e: e.get('source', {}).get('component', 'unknown')).items():
            warn = [e for e in evs if e.get('type', '') == 'Warning']
            if not warn:
                continue
            last = _latest(warn)
            self.add_finding(component=f"Control Plane/{comp}",
                             issue=f"Control plane component {comp} reporting warnings", severity="critical",
                             evidence=f"Reason: {last.get('reason', 'Unknown')}, Message: {last.get('message', '')}",
                             recommendation=f"Investigate health of {comp} in your Kubernetes control plane")
            self.add_reasoning_step(observation=f"Detected {len(warn)} warning events from {comp}",
                                    conclusion=f"Control plane component {comp} may be experiencing issues")

    def _nodes(self, events):  # ref :377-446
        def is_node(e):
            return (e.get('involvedObject', {}).get('kind', '') == 'Node'
                    or any(c in e.get('reason', '') for c in _NODE_REASONS))

        def node_of(e):
            o = e.get('involvedObject', {})
            if o.get('kind', '') == 'Node':
                return o.get('name', 'unknown')
            return e.get('source', {}).get('host', 'unknown')

        for node, evs in _group([e for e in events if is_node(e)], node_of).items():
            warn = [e for e in evs if e.get('type', '') == 'Warning']
            if not warn:
                continue
            last = _latest(warn)
            reason = last.get('reason', 'Unknown')
            issue, rec = "unknown issue", "Investigate the node's status and logs"
            for needle, i, r in _NODE_ISSUES:
                if needle in reason:
                    issue, rec = i, r
                    break
            self.add_finding(component=f"Node/{node}", issue=f"Node experiencing {issue}", severity="critical",
                             evidence=f"Reason: {reason}, Message: {last.get('message', '')}", recommendation=rec)
            self.add_reasoning_step(observation=f"Detected {len(warn)} warning events for node {node}",
                                    conclusion=f"Node {node} is experiencing {issue}")
