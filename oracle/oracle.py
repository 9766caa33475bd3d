"""CPU oracle for the krca numeric core.  TEST INFRASTRUCTURE ONLY.

Only tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg import this module.
It is the checker, never the thing measured or shipped.

Parity anchors:
  * log histograms: :func:`log_hist` restates ref:agents/logs_agent.py:140-151 literally
    (``str.splitlines`` + ``re.search(p, line, re.IGNORECASE)`` with the reference's 13
    patterns) and is pinned by tests/golden/logs_corpus.json, captured from the reference;
  * thresholds: pinned by tests/golden/metrics_scaled.json and the C1 goldens;
  * PageRank: :func:`ppr_f64` is the networkx 3.4.2 ``_pagerank_scipy`` iteration in float64,
    pinned by tests/golden/ppr_known.json (networkx on the reference's mock dependency map);
  * pod status groups: :func:`categorize_pods_ref` restates ref:agents/resource_analyzer.py:
    264-380 + :856-895 on pod dicts (pinned by the C1 ResourceAnalyzer golden), and
    :func:`pod_classify_ref` the same rules on the columnar encoding of krca/podstate.py;
  * service-graph construction: :func:`selector_match_ref` / :func:`substr_match_ref` are the
    pair tests of ref:agents/topology_agent.py:133,257 and ref:agents/resource_analyzer.py:851,
    pinned through the agents by tests/golden/topograph_cases.json (reference graphs);
  * event / finding group-bys: :func:`group_reduce_ref` is the dict-insertion-order group-by
    with Python ``max`` / stable ``sorted(reverse=True)`` of ref:agents/events_agent.py:105-446
    and ref:agents/coordinator.py:118-155, pinned through EventsAgent / Coordinator by
    tests/golden/events_cases.json and tests/golden/events_random.json (reference outputs);
  * rolling z-score / correlation / template hashing have no reference counterpart (new
    primitives named by the north star): their float64 restatements here are
    "parity unpinned" by the reference and define the semantics.
The bit-exact twins of the device arithmetic live in oracle/krca_oracle.c (:func:`c_lib`).
"""
import ctypes
import os
import re
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ERROR_PATTERNS = (  # ref:agents/logs_agent.py:20-34 (data)
    ("oom_kill", r"(Out of memory|OOMKilled|Killed|signal: killed)"),
    ("connection_refused", r"(Connection refused|connect: connection refused)"),
    ("permission_denied", r"(Permission denied|Forbidden|Access denied)"),
    ("timeout", r"(timeout|Timeout|timed out|ETIMEDOUT)"),
    ("crash_loop", r"(CrashLoopBackOff|Back-off restarting)"),
    ("api_error", r"(API server error|StatusCode=5\d\d)"),
    ("volume_mount", r"(Unable to mount volumes|MountVolume.SetUp failed)"),
    ("image_pull", r"(ErrImagePull|ImagePullBackOff)"),
    ("dns_resolution", r"(DNS resolution failed|could not resolve)"),
    ("authentication", r"(Unauthorized|Authentication failed)"),
    ("config_error", r"(Invalid configuration|ConfigMap not found|Secret not found)"),
    ("internal_server_error", r"(internal server error|InternalServerError|500 Internal Server Error)"),
    ("exception", r"(Exception|Error|Traceback|FATAL|CRITICAL|Panic|panic:)"),
)
_COMPILED = [re.compile(p, re.IGNORECASE) for _, p in ERROR_PATTERNS]


# ------------------------------------------------------------------------------------------
# logs (a12)
# ------------------------------------------------------------------------------------------
def line_mask(line):
    m = 0
    for b, rx in enumerate(_COMPILED):
        if rx.search(line):
            m |= 1 << b
    return m


def log_hist(text):
    """-> (n_lines, hist[13], first3[13] list of line strings) for one container's log text."""
    lines = text.splitlines()
    hist = [0] * 13
    ex = [[] for _ in range(13)]
    for ln in lines:
        m = line_mask(ln)
        for c in range(13):
            if m >> c & 1:
                hist[c] += 1
                if len(ex[c]) < 3:
                    ex[c].append(ln)
    return len(lines), hist, ex


# ------------------------------------------------------------------------------------------
# error templates (a13): new primitive, semantics of csrc/template.hip restated
# ------------------------------------------------------------------------------------------
_WORD = re.compile(rb"[A-Za-z0-9_]+")
_HEX = re.compile(rb"[0-9a-fA-F]{8,}")
# a UUID: five words of 8, 4, 4, 4 and 12 hex characters joined by single '-' (SURVEY.md §8a a13:
# "UUIDs masked"); tried first at every word start, so the leftmost UUID wins
_UUID = rb"(?<![A-Za-z0-9_])[0-9a-fA-F]{8}(?:-[0-9a-fA-F]{4}){3}-[0-9a-fA-F]{12}(?![A-Za-z0-9_])"
_TOKEN = re.compile(rb"(" + _UUID + rb")|[A-Za-z0-9_]+")


TEMPLATE_MASK = b"\xff"  # the one byte a masked word or UUID becomes (never in UTF-8 text; shown as "<*>")


def template_of(line_bytes):
    """csrc/template.hip's template (csrc/tmpl_dfa.h): every UUID, and every other maximal
    [A-Za-z0-9_] run holding a digit or of >= 8 hex digits, replaced by TEMPLATE_MASK."""
    def sub(m):
        if m.group(1) is not None:
            return TEMPLATE_MASK
        w = m.group(0)
        if any(48 <= c <= 57 for c in w) or _HEX.fullmatch(w):
            return TEMPLATE_MASK
        return w
    return _TOKEN.sub(sub, line_bytes)


def fnv1a64(b):
    h = 0xcbf29ce484222325
    for c in b:
        h = ((h ^ c) * 0x100000001b3) & 0xFFFFFFFFFFFFFFFF
    return h


def template_hist(text):
    """-> [(hash, count)] ascending for one container's log text (lines as str.splitlines)."""
    from collections import Counter
    cnt = Counter(fnv1a64(template_of(ln.encode("utf-8", "surrogatepass"))) for ln in text.splitlines())
    return sorted(cnt.items())


# ------------------------------------------------------------------------------------------
# rolling z-score (a5), float64 independent formulation (prefix sums)
# ------------------------------------------------------------------------------------------
def rolling_score_f64(x, W, z_thr=3.0):
    """x [T, P, M] -> (z_last [P, M], score [P], n_exceed [P]) in float64 / int."""
    x = np.asarray(x, dtype=np.float64)
    T, P, M = x.shape
    if T <= W:
        return np.zeros((P, M)), np.zeros(P), np.zeros(P, np.int64)
    c1 = np.concatenate([np.zeros((1, P, M)), np.cumsum(x, axis=0)])
    c2 = np.concatenate([np.zeros((1, P, M)), np.cumsum(x * x, axis=0)])
    t = np.arange(W, T)
    s1 = c1[t] - c1[t - W]
    s2 = c2[t] - c2[t - W]
    mean = s1 / W
    var = np.maximum(s2 / W - mean * mean, 0.0)
    d = x[W:] - mean
    ok = var > 1e-12
    z = np.where(ok, d / np.sqrt(np.where(ok, var, 1.0)), 0.0)
    n = (np.abs(z) > z_thr).sum(axis=(0, 2))
    zl = z[-1]
    return zl, np.abs(zl).max(axis=1), n


# ------------------------------------------------------------------------------------------
# personalized PageRank (a10): networkx 3.4.2 iteration in float64
# ------------------------------------------------------------------------------------------
def ppr_f64(row_ptr, col, outdeg, seed, alpha=0.85, max_iter=100, tol=1e-6):
    row_ptr = np.asarray(row_ptr, np.int64)
    col = np.asarray(col, np.int64)
    outdeg = np.asarray(outdeg, np.float64)
    N = len(outdeg)
    p = np.maximum(np.asarray(seed, np.float64), 0.0)
    p = p / p.sum() if p.sum() > 0 else np.full(len(p), 1.0 / len(p))
    inv = np.where(outdeg > 0, 1.0 / np.where(outdeg > 0, outdeg, 1.0), 0.0)
    dangling = outdeg == 0
    rows = np.repeat(np.arange(N), np.diff(row_ptr))
    x = np.full(N, 1.0 / N)
    for it in range(max_iter):
        xl = x
        contrib = (xl * inv)[col]
        y = np.bincount(rows, weights=contrib, minlength=N)
        x = alpha * (y + xl[dangling].sum() * p) + (1 - alpha) * p
        if tol > 0 and np.abs(x - xl).sum() < N * tol:
            return x, it + 1
    return x, max_iter


def topk_ref(v, k):
    """Descending, ties -> lower index (the device contract)."""
    v = np.asarray(v)
    order = np.lexsort((np.arange(len(v)), -v.astype(np.float64) if v.dtype.kind == "f" else -v))
    idx = order[:k]
    return idx.astype(np.int32), v[idx]


def corr_standardize(x, channel=0):
    """x [T, P, M] -> z [P, T] float64 with z·zᵀ = Pearson r (population std; flat -> 0).
    New primitive a9: no reference counterpart, semantics defined here."""
    s = np.asarray(x[:, :, channel], dtype=np.float64).T
    T = s.shape[1]
    mu = s.mean(axis=1, keepdims=True)
    d = s - mu
    var = (d * d).mean(axis=1, keepdims=True)
    sc = np.where(var > 1e-20, 1.0 / np.sqrt(np.maximum(var, 1e-300) * T), 0.0)
    return d * sc


def corr_rows(z, rows, k, tau):
    """For pods `rows`: (idx [n,k], r [n,k], count [n], gap [n]) by |r| desc, index asc, self
    excluded; gap = |r|_(k) - |r|_(k+1) (how far the k-th is from being tied)."""
    rows = np.asarray(rows)
    P = z.shape[0]
    R = z[rows] @ z.T
    R[np.arange(len(rows)), rows] = np.nan
    a = np.abs(R)
    count = (a > tau).sum(axis=1)
    a = np.where(np.isnan(a), -1.0, a)
    idx = np.empty((len(rows), k), np.int64)
    gap = np.empty(len(rows))
    kk = min(k + 1, P - 1)
    for n in range(len(rows)):
        thr = np.partition(-a[n], kk - 1)[kk - 1]
        part = np.nonzero(-a[n] <= thr)[0]  # every pod at least as good as the kk-th (ties kept)
        o = part[np.lexsort((part, -a[n][part]))]
        idx[n] = o[:k]
        gap[n] = a[n][o[k - 1]] - (a[n][o[k]] if len(o) > k else -1.0)
    r = np.take_along_axis(R, idx, axis=1)
    return idx.astype(np.int32), r, count, gap


# ------------------------------------------------------------------------------------------
# f1: pod status groups (ref:agents/resource_analyzer.py:264-380, _is_pod_healthy :856-895)
# ------------------------------------------------------------------------------------------
POD_GROUPS = ('pending', 'running', 'succeeded', 'failed', 'unknown', 'crashloopbackoff', 'imagepullbackoff',
              'containercreating', 'error', 'evicted', 'init_crashloopbackoff', 'not_ready')


def _pod_healthy_ref(pod):  # ref :856-895
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


def categorize_pods_ref(pods):
    """ref :289-343 on pod dicts -> {group: [pod index, ...]} in the reference's order."""
    g = {k: [] for k in POD_GROUPS}
    for i, pod in enumerate(pods):
        st = pod['status']
        phase = st.get('phase', 'Unknown')
        if phase == 'Pending':
            g['pending'].append(i)
        elif phase == 'Running':
            if not _pod_healthy_ref(pod):
                for cs in st.get('containerStatuses', []) + st.get('initContainerStatuses', []):
                    state = cs.get('state', {})
                    if 'waiting' in state:
                        reason = state['waiting'].get('reason', '')
                        if reason == 'CrashLoopBackOff':
                            g['init_crashloopbackoff' if cs['name'].startswith('init-') else 'crashloopbackoff'].append(i)
                            break
                        elif reason == 'ImagePullBackOff' or reason == 'ErrImagePull':
                            g['imagepullbackoff'].append(i)
                            break
                        elif reason == 'ContainerCreating':
                            g['containercreating'].append(i)
                            break
                ready = True
                for cond in st.get('conditions', []):
                    if cond.get('type') == 'Ready' and cond.get('status') != 'True':
                        ready = False
                        break
                if not ready:
                    g['not_ready'].append(i)
            else:
                g['running'].append(i)
        elif phase == 'Succeeded':
            g['succeeded'].append(i)
        elif phase == 'Failed':
            g['failed'].append(i)
        elif phase == 'Unknown':
            g['unknown'].append(i)
        if st.get('reason', '') == 'Evicted':
            g['evicted'].append(i)
        for cs in st.get('containerStatuses', []):
            if cs.get('state', {}).get('terminated', {}).get('reason', '') == 'Error':
                g['error'].append(i)
                break
    return g


def pod_classify_ref(pod_code, cont_off, cont_code):
    """The same rules on the columnar encoding -> (mask u16[P], hist i32[12])."""
    P = len(pod_code)
    mask = np.zeros(P, np.uint16)
    for p in range(P):
        pc = int(pod_code[p])
        cc = [int(x) for x in cont_code[cont_off[p]:cont_off[p + 1]]]
        main = [x for x in cc if not x & 1]
        phase, m = pc & 7, 0
        if phase == 0:
            m |= 1
        elif phase == 1:
            healthy = bool(pc & 8) and len(main) > 0 and all(
                (x & 2) and not (x & 4) and not ((x & 8) and ((x >> 7) & 3) != 1) for x in main)
            if healthy:
                m |= 2
            else:
                for x in cc:
                    if not x & 4:
                        continue
                    wr = (x >> 4) & 7
                    if wr == 1:
                        m |= 1 << (10 if x & 512 else 5)
                        break
                    if wr in (2, 3):
                        m |= 1 << 6
                        break
                    if wr == 4:
                        m |= 1 << 7
                        break
                if pc & 16:
                    m |= 1 << 11
        elif phase in (2, 3, 4):
            m |= 1 << phase
        if pc & 32:
            m |= 1 << 9
        if any((x & 8) and ((x >> 7) & 3) == 2 for x in main):
            m |= 1 << 8
        mask[p] = m
    hist = np.array([int(((mask >> b) & 1).sum()) for b in range(12)], np.int32)
    return mask, hist



# ------------------------------------------------------------------------------------------
# f2: service-graph construction (ref:agents/topology_agent.py:94-260,
#     ref:agents/resource_analyzer.py:835-854) — semantics of csrc/topograph.hip
# ------------------------------------------------------------------------------------------
def selector_match_ref(lab, lab_off, sel, sel_off):
    """Interned item-id sets -> uint64 bits [D][ceil(S/64)]: bit s of row d iff every id of
    selector s occurs among the ids of object d (the ``all(item in labels.items() ...)`` test
    of ref:agents/topology_agent.py:133 once the host has interned the items)."""
    D, S = len(lab_off) - 1, len(sel_off) - 1
    SW = (S + 63) // 64
    bits = np.zeros((D, SW), np.uint64)
    sels = [set(int(x) for x in sel[sel_off[s]:sel_off[s + 1]]) for s in range(S)]
    for d in range(D):
        have = set(int(x) for x in lab[lab_off[d]:lab_off[d + 1]])
        for s in range(S):
            if sels[s] <= have:
                bits[d, s // 64] |= np.uint64(1 << (s % 64))
    return bits


def substr_match_ref(text, val_off, pat, pat_off):
    """Byte blobs -> sorted int64 v*K + k for every key k contained in value v (``key in value``
    of ref:agents/topology_agent.py:257; the empty key is in every value)."""
    text, pat = bytes(text), bytes(pat)
    V, K = len(val_off) - 1, len(pat_off) - 1
    out = []
    for v in range(V):
        val = text[val_off[v]:val_off[v + 1]]
        for k in range(K):
            if pat[pat_off[k]:pat_off[k + 1]] in val:
                out.append(v * K + k)
    return np.asarray(out, np.int64)

# ------------------------------------------------------------------------------------------
# C restatement (bit-exact twin of the device arithmetic)
# ------------------------------------------------------------------------------------------
_c = None


def group_reduce_ref(slot, key, S, R, n_ranked=None):
    """Group-by of krca_group_reduce, written as the reference's dict loops
    (ref:agents/events_agent.py:122-127 ``object_events.setdefault(key, []).append(event)``,
    ``max(..., key=lastTimestamp)`` :193, ``sorted(..., reverse=True)[:3]`` :148;
    ref:agents/coordinator.py:134-139,150): groups in first-seen order, then per group the
    member count, the selected count (key >= 0) and the R largest selected keys.
    Ranks r >= 1 only over records i < n_ranked.  Returns (first, count, n_key, top[R, S])."""
    n_ranked = len(slot) if n_ranked is None else n_ranked
    groups = {}
    for i, (s, k) in enumerate(zip(np.asarray(slot).tolist(), np.asarray(key).tolist())):
        if 0 <= s < S:
            groups.setdefault(s, []).append((i, k))
    first = np.full(S, 2**31 - 1, np.int32)
    count = np.zeros(S, np.int32)
    n_key = np.zeros(S, np.int32)
    top = np.full((R, S), -1, np.int64)
    for s, mem in groups.items():
        first[s] = mem[0][0]
        count[s] = len(mem)
        sel = sorted((k for _, k in mem if k >= 0), reverse=True)
        n_key[s] = len(sel)
        uniq = sorted(set(sel), reverse=True)
        if uniq:
            top[0, s] = uniq[0]
        ranked = sorted({k for i, k in mem if k >= 0 and i < n_ranked and k < uniq[0]}, reverse=True) if uniq else []
        for r, k in enumerate(ranked[:R - 1]):
            top[r + 1, s] = k
    return first, count, n_key, top


def c_lib():
    global _c
    if _c is not None:
        return _c
    # KRCA_ORACLE_LIB: the AddressSanitizer build of the same source (tests/test_host_asan_cpu.py)
    path = os.environ.get("KRCA_ORACLE_LIB") or os.path.join(HERE, "_build", "libkrca_oracle.so")
    if not os.path.exists(path):
        subprocess.run(["make", "-C", HERE], check=True, capture_output=True)
    lib = ctypes.CDLL(path)
    vp, i64, i32, f32, f64 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_float, ctypes.c_double
    lib.krco_usage_flags.argtypes = [vp, i64, vp]
    lib.krco_rolling_score.argtypes = [vp, i64, i32, i32, i32, f32, vp, vp, vp, vp]
    lib.krco_ppr.argtypes = [vp, vp, vp, i64, vp, f32, f64, i32, f64, vp, vp, vp]
    lib.krco_ppr.restype = i32
    lib.krco_ppr_start.argtypes = [vp, vp, vp, i64, vp, f32, f64, i32, f64, vp, vp, vp, ctypes.c_int]
    lib.krco_ppr_start.restype = i32
    lib.krco_rca_key.argtypes = [vp, vp, i64, vp]
    lib.krco_ppr_ex.argtypes = [vp, vp, vp, i64, vp, f32, f64, i32, f64, vp, vp, vp, ctypes.c_int, vp]
    lib.krco_ppr_ex.restype = i32
    lib.krco_rca_explain.argtypes = [vp, i64, f32, vp, vp, i64, i64, vp]
    lib.krco_rca_key_explained.argtypes = [vp, vp, vp, vp, i64, vp]
    lib.krco_corr_z32.argtypes = [vp, i64, i32, i32, i32, vp, vp, vp]
    lib.krco_corr_counts.argtypes = [vp, i64, i32, vp, i64, f64, f64, vp, vp]
    _c = lib
    return lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def c_usage_flags(usage):
    u = np.ascontiguousarray(usage, np.float32).reshape(-1, 2)
    out = np.zeros(len(u), np.uint8)
    c_lib().krco_usage_flags(_p(u), len(u), _p(out))
    return out


def c_rolling_score(x, W, z_thr=3.0):
    x = np.ascontiguousarray(x, np.float32)
    T, P, M = x.shape
    z = np.zeros((P, M), np.float32)
    s = np.zeros(P, np.float32)
    n = np.zeros(P, np.int32)
    f = np.zeros(P, np.uint8)
    c_lib().krco_rolling_score(_p(x), P, M, T, W, z_thr, _p(z), _p(s), _p(n), _p(f))
    return dict(z_last=z, score=s, n_exceed=n, flags=f)


def c_ppr(row_ptr, col, outdeg, seed, alpha=0.85, max_iter=100, tol=1e-6, seed_floor=0.0, return_q=False):
    rp = np.ascontiguousarray(row_ptr, np.int64)
    cl = np.ascontiguousarray(col, np.int32)
    od = np.ascontiguousarray(outdeg, np.int32)
    sd = np.ascontiguousarray(seed, np.float32)
    N = len(od)
    r = np.zeros(N, np.int64)
    q = np.zeros(N, np.int64)
    rf = np.zeros(N, np.float32)
    it = c_lib().krco_ppr(_p(rp), _p(cl), _p(od), N, _p(sd), seed_floor, alpha, max_iter, tol, _p(r), _p(rf), _p(q))
    return (rf, r, it, q) if return_q else (rf, r, it)


def c_ppr_warm(row_ptr, col, outdeg, seed, r_start, alpha, max_iter, tol, seed_floor):
    """krco_ppr started from the fixed-point vector r_start (streaming re-ranking) -> (r, iters, q)."""
    rp = np.ascontiguousarray(row_ptr, np.int64)
    cl = np.ascontiguousarray(col, np.int32)
    od = np.ascontiguousarray(outdeg, np.int32)
    sd = np.ascontiguousarray(seed, np.float32)
    N = len(od)
    r = np.array(r_start, np.int64, copy=True)
    q = np.zeros(N, np.int64)
    rf = np.zeros(N, np.float32)
    it = c_lib().krco_ppr_start(_p(rp), _p(cl), _p(od), N, _p(sd), seed_floor, alpha, max_iter, tol, _p(r), _p(rf),
                                _p(q), 1)
    return r, it, q


def c_corr_z32(x, channel=0):
    """Bit-exact twin of krca_corr_prepare (csrc/corr.hip corr_stats + corr_transpose): x [T, P, M]
    float32 -> (z32 [P, T] float32, mean [P], scale [P]).  The |r| > tau counts are defined on these
    rows (float64 dot products), so they can be checked exactly (new primitive a9)."""
    x = np.ascontiguousarray(x, np.float32)
    T, P, M = x.shape
    z = np.empty((P, T), np.float32)
    mean = np.empty(P, np.float32)
    scale = np.empty(P, np.float32)
    c_lib().krco_corr_z32(_p(x), P, M, T, int(channel), _p(mean), _p(scale), _p(z))
    return z, mean, scale


def c_corr_counts(z32, rows, tau, band_eps=1e-12):
    """-> (count [n], band [n]): exact |r| > tau counts of `rows` over the fp32 rows z32 (float64
    sums), and the number of partners within band_eps of tau (float64 summation-order ties)."""
    z = np.ascontiguousarray(z32, np.float32)
    rows = np.ascontiguousarray(rows, np.int64)
    cnt = np.zeros(len(rows), np.int32)
    band = np.zeros(len(rows), np.int32)
    c_lib().krco_corr_counts(_p(z), z.shape[0], z.shape[1], _p(rows), len(rows), float(tau), float(band_eps),
                             _p(cnt), _p(band))
    return cnt, band


def c_ppr_ex(row_ptr, col, outdeg, seed, alpha, max_iter, tol, seed_floor, r_start=None):
    """krco_ppr_ex -> dict(r, rf, it, q, recv): recv = the mass each node received from its callers in
    the last iteration (r = recv + teleport share); r_start: warm start (krca_ppr_shard_init_warm)."""
    rp = np.ascontiguousarray(row_ptr, np.int64)
    cl = np.ascontiguousarray(col, np.int32)
    od = np.ascontiguousarray(outdeg, np.int32)
    sd = np.ascontiguousarray(seed, np.float32)
    N = len(od)
    r = np.zeros(N, np.int64) if r_start is None else np.array(r_start, np.int64, copy=True)
    q = np.zeros(N, np.int64)
    recv = np.zeros(N, np.int64)
    rf = np.zeros(N, np.float32)
    it = c_lib().krco_ppr_ex(_p(rp), _p(cl), _p(od), N, _p(sd), seed_floor, alpha, max_iter, tol, _p(r), _p(rf), _p(q),
                             0 if r_start is None else 1, _p(recv))
    return dict(r=r, rf=rf, it=it, q=q, recv=recv)


def c_rca_explain(score, seed_floor, row_ptr, col, lo=0, hi=None):
    """krco_rca_explain: d[hi - lo] = the largest quantised anomaly of a dependency that explains
    each pod of [lo, hi), over the whole pull-CSR and the scores of every pod."""
    sc = np.ascontiguousarray(score, np.float32)
    rp = np.ascontiguousarray(row_ptr, np.int64)
    cl = np.ascontiguousarray(col, np.int32)
    N = len(sc)
    hi = N if hi is None else int(hi)
    d = np.zeros(max(hi - lo, 0), np.int64)
    c_lib().krco_rca_explain(_p(sc), N, seed_floor, _p(rp), _p(cl), int(lo), hi, _p(d))
    return d


def c_rca_key_explained(r, recv, q, d):
    r = np.ascontiguousarray(r, np.int64)
    recv = np.ascontiguousarray(recv, np.int64)
    q = np.ascontiguousarray(q, np.int64)
    d = np.ascontiguousarray(d, np.int64)
    key = np.zeros(len(q), np.int64)
    c_lib().krco_rca_key_explained(_p(r), _p(recv), _p(q), _p(d), len(q), _p(key))
    return key


def c_rca_key(r, q):
    r = np.ascontiguousarray(r, np.int64)
    q = np.ascontiguousarray(q, np.int64)
    key = np.zeros(len(r), np.int64)
    c_lib().krco_rca_key(_p(r), _p(q), len(r), _p(key))
    return key


def rca_keys(row_ptr, col, outdeg, score, alpha, iters, seed_floor, key="explained", tol=0.0, r_start=None):
    """The pipeline's root-cause keys (krca.rca.Config.key) of every pod -> (key, ppr dict).
    "explained": bits(recv_i * u_i), u = the anomaly no explaining dependency accounts for
    (krco_rca_explain); "rq": bits(r_i * q_i)."""
    o = c_ppr_ex(row_ptr, col, outdeg, score, alpha, iters, tol, seed_floor, r_start)
    return rca_keys_from(o, score, seed_floor, row_ptr, col, key), o


def rca_keys_from(o, score, seed_floor, row_ptr, col, key="explained"):
    """The keys of a finished c_ppr_ex solve `o` (dict r, q, recv)."""
    if key == "rq":
        return c_rca_key(o["r"], o["q"])
    if key != "explained":
        raise ValueError(f"unknown ranking key {key!r}")
    o["d"] = c_rca_explain(score, seed_floor, row_ptr, col)
    return c_rca_key_explained(o["r"], o["recv"], o["q"], o["d"])


def rca_rank(row_ptr, col, outdeg, score, alpha, iters, seed_floor, k=10, key="explained", tol=0.0):
    """Reference root-cause ranking of the pipeline: top-k of the Config key (ties -> lower index);
    iters = the cap, tol = the L1 stop rule (krca.rca.Config)."""
    kv, o = rca_keys(row_ptr, col, outdeg, score, alpha, iters, seed_floor, key, tol=tol)
    idx, _ = topk_ref(kv, k)
    return idx, o["rf"], o["r"]
