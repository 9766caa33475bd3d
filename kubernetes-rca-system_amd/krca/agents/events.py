"""EventsAgent: group-bys over a namespace's events, on the device.

Reference: ref:agents/events_agent.py:4-446.  The events are encoded into columns once
(krca/eventcols.py) and the five group-bys run as one ``krca_group_reduce`` launch plus one
``krca_topk_i64`` for the frequent events; findings and reasoning steps are replayed in the
reference's order.  A client with a bulk accessor ``get_event_columns(namespace)`` hands the
columns over directly.  Event lists that are not plain dicts of str / int fields take the
reference's own loops below (``_host_analyze``), which also raise the reference's errors.
"""
from .. import eventcols
from .base import BaseAgent

from ..eventcols import (CONTROL_PLANE as _CONTROL_PLANE, CRITICAL_REASONS, NODE_ISSUES as _NODE_ISSUES,  # noqa: E402
                         NODE_REASONS as _NODE_REASONS, SCHED_CAUSES as _SCHED_CAUSES,
                         VOLUME_CAUSES as _VOLUME_CAUSES)


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
            bulk = getattr(self.k8s_client, 'get_event_columns', None)
            cols = bulk(namespace) if bulk is not None else None
            events = cols if cols is not None else self.k8s_client.get_events(namespace)
            if (len(cols) == 0) if cols is not None else not events:
                self.add_reasoning_step(observation=f"No events found in namespace {namespace}",
                                        conclusion="No event data to analyze")
                return self.get_results()
            self.add_reasoning_step(observation=f"Found {len(events)} events in namespace {namespace}",
                                    conclusion="Beginning events analysis")
            if cols is None:
                cols = eventcols.encode_events(events)
            if cols is not None:
                for kind, kw in eventcols.analyze(self.engine, cols):
                    (self.add_finding if kind == 'finding' else self.add_reasoning_step)(**kw)
                return self.get_results()
            self._host_analyze(events)
            return self.get_results()
        except Exception as e:
            return self._error_result("events", e)

    def _host_analyze(self, events):
        """The reference's loops (ref :105-446) for events the columnar encoding cannot hold."""
        by_obj = _group(events, _obj_key)
        self.add_reasoning_step(observation=f"Grouped events into {len(by_obj)} unique objects",
                                conclusion="Will analyze events by object type and name")
        self._object_warnings(by_obj)
        self._scheduling(events)
        self._volumes(events)
        self._frequent(events)
        self._control_plane(events)
        self._nodes(events)

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
