"""Columnar pod status for the f1 categorisation kernel (krca_pod_classify, csrc/podstate.hip).

The reference walks pod dicts (ref:agents/resource_analyzer.py:264-380, _is_pod_healthy :856-895).
This module defines the columnar format those checks need and encodes pod dicts into it once:

  pod_code  u8[P]     bits 0-2 phase, bit 3 first Ready condition "True", bit 4 some Ready condition
                      not "True", bit 5 status.reason == "Evicted"
  cont_off  i64[P+1]  container records of pod p, containerStatuses first, then initContainerStatuses
  cont_code u16[C]    bit 0 init list, bit 1 ready, bit 2 waiting, bit 3 terminated, bits 4-6 waiting
                      reason, bits 7-8 terminated reason, bit 9 name starts with "init-"

Group bits follow the reference's status_groups dict order (GROUPS).  A container status with no
"name" encodes as a non-"init-" name (the reference would raise KeyError there, and only for a
CrashLoopBackOff container).  For namespaces too large for dicts, a cluster client can hand the
columns over directly (``get_pod_status_columns``); :func:`make_pod_states` synthesises them.
"""
import numpy as np

GROUPS = ('pending', 'running', 'succeeded', 'failed', 'unknown', 'crashloopbackoff', 'imagepullbackoff',
          'containercreating', 'error', 'evicted', 'init_crashloopbackoff', 'not_ready')
_PHASE = {'Pending': 0, 'Running': 1, 'Succeeded': 2, 'Failed': 3, 'Unknown': 4}
_WAIT = {'CrashLoopBackOff': 1, 'ImagePullBackOff': 2, 'ErrImagePull': 3, 'ContainerCreating': 4}
_TERM = {'Completed': 1, 'Error': 2}


def _cont_code(cs, is_init):
    state = cs.get('state', {}) or {}
    c = (1 if is_init else 0) | (2 if cs.get('ready', False) else 0)
    if 'waiting' in state:
        c |= 4 | (_WAIT.get((state['waiting'] or {}).get('reason', ''), 0) << 4)
    if 'terminated' in state:
        c |= 8 | (_TERM.get((state['terminated'] or {}).get('reason', ''), 0) << 7)
    if str(cs.get('name', '')).startswith('init-'):
        c |= 512
    return c


def encode_pods(pods):
    """pod dicts -> (pod_code u8[P], cont_off i64[P+1], cont_code u16[C])."""
    P = len(pods)
    pod_code = np.zeros(P, np.uint8)
    cont_off = np.zeros(P + 1, np.int64)
    codes = []
    for p, pod in enumerate(pods):
        st = pod.get('status', {}) or {}
        c = _PHASE.get(st.get('phase', 'Unknown'), 5)
        conds = st.get('conditions', []) or []
        first = next((x for x in conds if x.get('type') == 'Ready'), None)
        if first is not None and first.get('status') == 'True':
            c |= 8
        if any(x.get('type') == 'Ready' and x.get('status') != 'True' for x in conds):
            c |= 16
        if st.get('reason', '') == 'Evicted':
            c |= 32
        pod_code[p] = c
        for cs in st.get('containerStatuses', []) or []:
            codes.append(_cont_code(cs, False))
        for cs in st.get('initContainerStatuses', []) or []:
            codes.append(_cont_code(cs, True))
        cont_off[p + 1] = len(codes)
    return pod_code, cont_off, np.asarray(codes, np.uint16)


def groups_from_masks(items, mask):
    """status_groups dict (reference order and membership) from the kernel's per-pod masks."""
    mask = np.asarray(mask, np.uint16)
    return {g: [items[i] for i in np.nonzero(mask & (1 << b))[0]] for b, g in enumerate(GROUPS)}


def make_pod_states(P, seed=0, containers=(1, 4)):
    """Synthetic columnar pod status with every category represented (for scale tests / bench)."""
    rng = np.random.default_rng(seed)
    phase = rng.choice(6, P, p=[0.05, 0.8, 0.05, 0.04, 0.03, 0.03]).astype(np.uint8)
    flags = (rng.random(P) < 0.85).astype(np.uint8) << 3
    flags |= (rng.random(P) < 0.15).astype(np.uint8) << 4
    flags |= (rng.random(P) < 0.02).astype(np.uint8) << 5
    pod_code = phase | flags
    n = rng.integers(containers[0], containers[1] + 1, P)
    cont_off = np.zeros(P + 1, np.int64)
    np.cumsum(n, out=cont_off[1:])
    C = int(cont_off[-1])
    pos = np.arange(C) - np.repeat(cont_off[:-1], n)
    is_init = (pos >= np.repeat(np.maximum(n - 1, 1), n)) & (rng.random(C) < 0.3)
    code = is_init.astype(np.uint16)
    code |= (rng.random(C) < 0.85).astype(np.uint16) << 1
    waiting = rng.random(C) < 0.12
    code |= waiting.astype(np.uint16) << 2
    code |= (waiting * rng.integers(0, 5, C)).astype(np.uint16) << 4
    term = rng.random(C) < 0.1
    code |= term.astype(np.uint16) << 3
    code |= (term * rng.integers(0, 3, C)).astype(np.uint16) << 7
    code |= (rng.random(C) < 0.2).astype(np.uint16) << 9
    return pod_code.astype(np.uint8), cont_off, code.astype(np.uint16)
