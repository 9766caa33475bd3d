"""Columnar events and the EventsAgent group-bys on the device.

The reference (ref:agents/events_agent.py:105-446) walks event dicts six times and builds a dict
per analysis: events by object key (``f"{kind}/{name}"``, :105-133), FailedScheduling events by
pod name (:169-228), volume events by object key (:230-290), control-plane events by source
component (:330-375) and node events by node name (:377-446); frequent events are the top 5 by
count (:292-328).  Here the string keys are interned once into dense ids, every analysis becomes
membership records (slot, key) of ONE ``krca_group_reduce`` launch (csrc/groupby.hip), and the
frequent events one ``krca_topk_i64``.  The host then replays the findings in the reference's
order from the per-group first position, sizes and latest members.

Sort keys: ``(rank(lastTimestamp) << 32) | (2^31 - 1 - event index)``.  Python's ``max`` returns
the first maximal event and ``sorted(..., reverse=True)`` is stable, so among equal timestamps
the earlier event wins in both; the packed key orders exactly that way and is unique per event.

Columns (``EventColumns``), one entry per event, ids into per-column string tables:
  kind, name (involvedObject; missing -> 'Unknown' / 'unknown'), reason (-1 = missing: filters
  see '', findings show 'Unknown'), message (missing -> ''), comp (source.component, -1 =
  missing), host (source.host, missing -> 'unknown'), warn u8 (type == 'Warning'), ts int32
  (rank of lastTimestamp among the distinct values, missing -> ''), count int64 (missing -> 1).
Events that are not plain dicts of strings / ints take the reference's host loop instead
(:func:`encode_events` returns None), which raises the reference's own errors.
"""
import numpy as np

CRITICAL_REASONS = ('Failed', 'FailedCreate', 'FailedScheduling', 'FailedMount', 'NodeNotReady',
                    'KubeletNotReady', 'FailedAttachVolume', 'FailedDetachVolume', 'FreeDiskSpaceFailed',
                    'OutOfDisk', 'MemoryPressure', 'DiskPressure', 'NetworkUnavailable', 'Unhealthy',
                    'FailedSync', 'Evicted', 'BackOff', 'Error')  # ref:agents/events_agent.py:28-34
VOLUME_REASONS = ('FailedMount', 'FailedAttachVolume', 'FailedDetachVolume')  # ref :238
CONTROL_PLANE = ('kube-apiserver', 'kube-controller-manager', 'kube-scheduler', 'etcd')  # ref :339
NODE_REASONS = ('NodeNotReady', 'KubeletNotReady', 'MemoryPressure', 'DiskPressure', 'NetworkUnavailable')  # :389

# (predicate on message, cause, recommendation) in priority order (ref :201-215, :266-277)
SCHED_CAUSES = (
    (lambda m: "Insufficient cpu" in m, "insufficient CPU", "Increase CPU capacity in your cluster or reduce CPU requests"),
    (lambda m: "Insufficient memory" in m, "insufficient memory", "Increase memory capacity in your cluster or reduce memory requests"),
    (lambda m: "node(s) had taint" in m, "node taints", "Add appropriate tolerations to the pod or remove taints from nodes"),
    (lambda m: "node(s) didn't match node selector" in m, "node selector mismatch", "Update the pod's node selector or label your nodes correctly"),
    (lambda m: "persistentvolumeclaim" in m.lower() and "pending" in m.lower(), "pending PVC", "Check the PVC status and ensure storage is available"),
)
VOLUME_CAUSES = (  # predicates take message.lower()
    (lambda m: "timeout" in m, "mounting timeout", "Check if storage system is responsive and resources are available"),
    (lambda m: "no such file" in m, "path doesn't exist", "Verify the volume path exists in the source"),
    (lambda m: "permission denied" in m, "permission issue", "Check volume permissions and pod security context"),
    (lambda m: "not found" in m and "pvc" in m, "PVC not found", "Ensure the PVC exists and is in the correct namespace"),
)
NODE_ISSUES = (("NotReady", "node not ready", "Check kubelet status, node connectivity, and system logs on the node"),
               ("MemoryPressure", "memory pressure", "Free up memory on the node or add more memory resources"),
               ("DiskPressure", "disk pressure", "Free up disk space on the node or expand storage"),
               ("NetworkUnavailable", "network unavailable", "Check network configuration, CNI plugins, and network connectivity"))

_IDX_MASK = 0x7FFFFFFF
_MISSING = object()
TOP_R = 3  # the object analysis keeps the 3 latest warnings (ref :148)


class EventColumns:
    """Columnar events (see module docstring).  Tables are lists of str."""

    def __init__(self, kind, name, reason, message, comp, host, warn, ts, count, kinds, names, reasons, messages,
                 comps, hosts):
        self.kind, self.name = np.asarray(kind, np.int32), np.asarray(name, np.int32)
        self.reason, self.message = np.asarray(reason, np.int32), np.asarray(message, np.int32)
        self.comp, self.host = np.asarray(comp, np.int32), np.asarray(host, np.int32)
        self.warn, self.ts = np.asarray(warn, np.uint8), np.asarray(ts, np.int32)
        self.count = np.asarray(count, np.int64)
        self.kinds, self.names, self.reasons, self.messages = kinds, names, reasons, messages
        self.comps, self.hosts = comps, hosts

    def __len__(self):
        return len(self.kind)

    def reason_str(self, e, missing=''):
        r = int(self.reason[e])
        return missing if r < 0 else self.reasons[r]


def _is_str(x):
    return type(x) is str


def encode_events(events):
    """event dicts -> EventColumns, or None when an event is not a plain dict of str / int fields
    (the agent then runs the reference's host loop, which raises the reference's errors)."""
    tabs = [{} for _ in range(6)]  # kind, name, reason, message, comp, host
    E = len(events)
    cols = np.empty((6, E), np.int32)
    warn = np.zeros(E, np.uint8)
    count = np.ones(E, np.int64)
    ts_raw = []
    for e, ev in enumerate(events):
        if type(ev) is not dict:
            return None
        io = ev.get('involvedObject', {})
        src = ev.get('source', {})
        if type(io) is not dict or type(src) is not dict:
            return None
        vals = (io.get('kind', 'Unknown'), io.get('name', 'unknown'), ev.get('reason', _MISSING),
                ev.get('message', ''), src.get('component', _MISSING), src.get('host', 'unknown'))
        for c, v in enumerate(vals):
            if v is _MISSING:
                cols[c, e] = -1
                continue
            if not _is_str(v):
                return None
            t = tabs[c]
            cols[c, e] = t.setdefault(v, len(t))
        ty = ev.get('type', '')
        ts = ev.get('lastTimestamp', '')
        cnt = ev.get('count', 1)
        if not _is_str(ty) or not _is_str(ts) or type(cnt) not in (int, bool) or not -2**62 < cnt < 2**62:
            return None
        warn[e] = ty == 'Warning'
        count[e] = cnt
        ts_raw.append(ts)
    uniq = sorted(set(ts_raw))
    rank = {t: i for i, t in enumerate(uniq)}
    ts = np.fromiter((rank[t] for t in ts_raw), np.int32, E)
    tables = [list(t) for t in tabs]  # dicts keep insertion order = id order
    return EventColumns(cols[0], cols[1], cols[2], cols[3], cols[4], cols[5], warn, ts, count, *tables)


def _intern(strings):
    ids, table = np.empty(len(strings), np.int32), {}
    for i, s in enumerate(strings):
        ids[i] = table.setdefault(s, len(table))
    return ids, list(table)


def group_records(cols):
    """Membership records of the five group-bys -> (slot, key, layout).  layout[a] = (offset,
    size, key strings of the slots) for a in objects, scheduling, volume, control_plane, nodes."""
    E = len(cols)
    ev = np.arange(E, dtype=np.int64)
    pack = (cols.ts.astype(np.int64) << 32) | (_IDX_MASK - ev)
    warn = cols.warn.astype(bool)
    wkey = np.where(warn, pack, -1)
    # object keys f"{kind}/{name}" (distinct (kind, name) pairs may format to the same string)
    pair = (cols.kind.astype(np.int64) << 32) | cols.name.astype(np.int64)
    upair, inv = np.unique(pair, return_inverse=True)
    ostr = [f"{cols.kinds[p >> 32]}/{cols.names[p & 0xFFFFFFFF]}" for p in upair.tolist()]
    oid_of_pair, okeys = _intern(ostr)
    objid = oid_of_pair[inv.reshape(-1)]
    rs = cols.reasons
    r_sched = np.array([r == 'FailedScheduling' for r in rs] + [False], bool)  # index -1 = missing
    r_vol = np.array([any(x in r for x in VOLUME_REASONS) for r in rs] + [False], bool)
    r_node = np.array([any(x in r for x in NODE_REASONS) for r in rs] + [False], bool)
    c_cp = np.array([any(x in c for x in CONTROL_PLANE) for c in cols.comps] + [False], bool)
    k_node = np.array([k == 'Node' for k in cols.kinds], bool)
    # node name: the involved object's name for Node events, else source.host (ref :398-403)
    node_ids, nkeys = _intern(list(cols.names) + list(cols.hosts))
    nn = len(cols.names)
    is_node_obj = k_node[cols.kind]
    nodeval = np.where(is_node_obj, node_ids[cols.name], node_ids[nn + cols.host])
    m_sched = r_sched[cols.reason]
    m_vol = r_vol[cols.reason]
    m_cp = c_cp[cols.comp]
    m_node = is_node_obj | r_node[cols.reason]
    segs = [(objid, wkey, okeys),
            (cols.name[m_sched], pack[m_sched], cols.names),
            (objid[m_vol], pack[m_vol], okeys),
            (cols.comp[m_cp], wkey[m_cp], cols.comps),
            (nodeval[m_node], wkey[m_node], nkeys)]
    slots, keys, layout, off = [], [], [], 0
    for s, k, names in segs:
        slots.append(s.astype(np.int32) + off)
        keys.append(k)
        layout.append((off, len(names), names))
        off += len(names)
    return np.concatenate(slots), np.concatenate(keys), layout


def _event(key):
    return _IDX_MASK - (int(key) & 0xFFFFFFFF)


def analyze(engine, cols):
    """Findings and reasoning steps of EventsAgent for E >= 1 events, in the reference's order:
    a list of ('finding' | 'step', kwargs)."""
    out = []
    slot, key, layout = group_records(cols)
    S = layout[-1][0] + layout[-1][1]
    first, count, n_key, top = engine.group_reduce(slot, key, S, TOP_R, n_ranked=len(cols))  # ranks 2-3: objects

    def step(obs, concl):
        out.append(('step', dict(observation=obs, conclusion=concl)))

    def finding(**kw):
        out.append(('finding', kw))

    def groups(a):
        off, n, names = layout[a]
        s = np.arange(off, off + n)
        s = s[count[off:off + n] > 0]
        for g in s[np.argsort(first[s], kind='stable')].tolist():
            yield g, names[g - off]

    msg = lambda e: cols.messages[cols.message[e]]  # noqa: E731
    step(f"Grouped events into {layout[0][1]} unique objects", "Will analyze events by object type and name")
    for g, k in groups(0):  # ref :136-167
        if n_key[g] < 3:
            continue
        recent = [_event(top[r, g]) for r in range(3)]
        reasons = [cols.reason_str(e, 'Unknown') for e in recent]
        msgs = "\n".join(f"- {msg(e)}" for e in recent)
        finding(component=k, issue=f"Multiple warning events detected for {k}",
                severity="high" if any(r in CRITICAL_REASONS for r in reasons) else "medium",
                evidence=f"Recent warnings ({', '.join(reasons)}):\n{msgs}",
                recommendation=f"Investigate the {k} resource for configuration or operational issues")
        step(f"Detected {n_key[g]} warning events for {k}", f"{k} is experiencing recurring issues")
    for g, pod in groups(1):  # ref :169-228
        m = msg(_event(top[0, g]))
        cause, rec = "unknown", "Check node resources and pod resource requirements"
        for pred, c, r in SCHED_CAUSES:
            if pred(m):
                cause, rec = c, r
                break
        finding(component=f"Pod/{pod}", issue=f"Pod scheduling failed due to {cause}", severity="high",
                evidence=f"Message: {m}", recommendation=rec)
        step(f"Detected {count[g]} scheduling failures for pod {pod}", f"Pod {pod} cannot be scheduled due to {cause}")
    for g, k in groups(2):  # ref :230-290
        e = _event(top[0, g])
        reason, m = cols.reason_str(e), msg(e)
        cause, rec = "unknown issue", "Check the volume configuration and storage system"
        for pred, c, r in VOLUME_CAUSES:
            if pred(m.lower()):
                cause, rec = c, r
                break
        finding(component=k, issue=f"Volume operation failed due to {cause}", severity="high",
                evidence=f"Reason: {reason}, Message: {m}", recommendation=rec)
        step(f"Detected {count[g]} volume issues for {k}", f"{k} is experiencing volume issues: {cause}")
    idx, val = engine.topk(cols.count, min(5, len(cols)))  # ref :292-328
    for e, c in zip(np.asarray(idx).tolist(), np.asarray(val).tolist()):
        if c <= 5 or not cols.warn[e]:
            continue
        kind, name = cols.kinds[cols.kind[e]], cols.names[cols.name[e]]
        reason = cols.reason_str(e, 'Unknown')
        finding(component=f"{kind}/{name}", issue=f"Frequent {reason} events detected ({c} occurrences)",
                severity="high" if c > 20 else "medium", evidence=f"Message: {msg(e)}",
                recommendation=f"Investigate the root cause of these recurring events on {kind} {name}")
        step(f"Detected {c} occurrences of {reason} events for {kind}/{name}",
             "Recurring events indicate a persistent issue that needs attention")
    for g, comp in groups(3):  # ref :330-375
        if n_key[g] == 0:
            continue
        e = _event(top[0, g])
        finding(component=f"Control Plane/{comp}", issue=f"Control plane component {comp} reporting warnings",
                severity="critical", evidence=f"Reason: {cols.reason_str(e, 'Unknown')}, Message: {msg(e)}",
                recommendation=f"Investigate health of {comp} in your Kubernetes control plane")
        step(f"Detected {n_key[g]} warning events from {comp}", f"Control plane component {comp} may be experiencing issues")
    for g, node in groups(4):  # ref :377-446
        if n_key[g] == 0:
            continue
        e = _event(top[0, g])
        reason = cols.reason_str(e, 'Unknown')
        issue, rec = "unknown issue", "Investigate the node's status and logs"
        for needle, i, r in NODE_ISSUES:
            if needle in reason:
                issue, rec = i, r
                break
        finding(component=f"Node/{node}", issue=f"Node experiencing {issue}", severity="critical",
                evidence=f"Reason: {reason}, Message: {msg(e)}", recommendation=rec)
        step(f"Detected {n_key[g]} warning events for node {node}", f"Node {node} is experiencing {issue}")
    return out


def make_events(E, seed=0, n_obj=None, n_hosts=64):
    """Synthetic columnar events (scale tests / timing): every analysis represented, hot control-
    plane slots, many small object groups, timestamp ties."""
    rng = np.random.default_rng(seed)
    n_obj = n_obj or max(E // 8, 1)
    kinds = ['Pod', 'Node', 'Deployment', 'ReplicaSet']
    reasons = ['BackOff', 'Failed', 'FailedScheduling', 'FailedMount', 'NodeNotReady', 'Unhealthy', 'Pulled',
               'MemoryPressure', 'DiskPressure', 'Evicted', 'FailedAttachVolume', 'CPUThrottling', 'Started']
    messages = ['0/3 nodes are available: 3 Insufficient cpu.', 'Insufficient memory', 'node(s) had taint {x}',
                "node(s) didn't match node selector", 'persistentvolumeclaim data is Pending', 'MountVolume timeout',
                'no such file or directory', 'permission denied', 'pvc claim not found', 'readiness probe failed',
                'Back-off restarting failed container']
    comps = ['kubelet', 'kube-scheduler', 'kube-controller-manager', 'etcd', 'default-scheduler', 'kube-apiserver-x']
    names = [f"obj-{i}" for i in range(n_obj)]
    hosts = [f"node-{i}" for i in range(n_hosts)]
    kind = rng.choice(len(kinds), E, p=[0.7, 0.05, 0.15, 0.1]).astype(np.int32)
    name = rng.integers(0, n_obj, E, dtype=np.int32)
    reason = rng.integers(-1, len(reasons), E).astype(np.int32)
    comp = rng.integers(-1, len(comps), E).astype(np.int32)
    return EventColumns(kind, name, reason, rng.integers(0, len(messages), E), comp,
                        rng.integers(0, n_hosts, E), rng.random(E) < 0.6, rng.integers(0, max(E // 4, 1), E),
                        rng.integers(1, 40, E), kinds, names, reasons, messages, comps, hosts)
