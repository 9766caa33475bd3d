"""Seeded synthetic meshes: pod metric tensors, dependency CSR, log corpora.

Shapes follow the reference's mock cluster (ref:utils/mock_k8s_client.py:468-495: per-pod CPU /
memory usage percentages; :909-934 per-container log text; :1251-1272 a caller -> dependency
map) scaled to the BASELINE configs (C2: 10k pods / 200k edges, C4: 1M pods / 20M edges,
M = 8 metrics x T = 1440 steps).  Metrics are generated with torch on any device (the 46 GB C4
tensor is generated in place on the GPU); graphs with NumPy on the host.

Metric model:  x[t,p,m] = clip(b + a*sin(2*pi*t/1440 + phi_p) + N(0, sigma^2), 0, 100),
b ~ U(25,55), a ~ U(0,12), sigma ~ U(0.5,3) (SURVEY.md §8d proposes U(10,60)/U(0,15); the narrower
ranges keep the noise off the 0/100 clamps, where flat windows give meaningless z-scores); R root pods get a +12 sigma spike on the last
`spike_steps` samples and their callers (hop h = 1..3) a +5*0.8^(h-1) sigma spike, so the
current-step z-scores the scorer reports (|z| at t = T-1 against the trailing window) single
them out.  Channel 0 = CPU %, 1 = memory %.
Graph model: pods grouped into services of 20; services wired by preferential attachment
(caller -> callee); each pod calls ~deg pods of its service's callees; no self loops, no
duplicate edges; edge direction symptom(caller) -> dependency.
"""
import math

import numpy as np


class Mesh:
    def __init__(self, n_pods, row_ptr, col, outdeg, roots, names=None):
        self.n_pods = n_pods
        self.row_ptr = row_ptr  # pull-CSR: row i = callers j of i (edges j -> i), int64[N+1]
        self.col = col          # int32[E]
        self.outdeg = outdeg    # int32[N]
        self.roots = roots      # int64[R] planted root causes
        self._names = names

    @property
    def n_edges(self):
        return int(self.row_ptr[-1])

    def names(self):
        if self._names is None:
            self._names = [f"pod-{i:07d}" for i in range(self.n_pods)]
        return self._names


def _services_ba(n_services, m, rng):
    """Preferential attachment over services; returns (caller, callee) arrays."""
    m = max(1, min(m, n_services - 1)) if n_services > 1 else 0
    src, dst = [], []
    targets = list(range(m))
    repeated = []
    for s in range(m, n_services):
        chosen = set()
        while len(chosen) < m:
            if repeated and rng.random() < 0.8:
                chosen.add(repeated[int(rng.integers(len(repeated)))])
            else:
                chosen.add(int(rng.integers(s)))
        for c in chosen:
            src.append(s)
            dst.append(c)
        repeated.extend(chosen)
        repeated.extend([s] * m)
    del targets
    return np.asarray(src, np.int64), np.asarray(dst, np.int64)


def make_graph(n_pods, avg_degree=20, service_size=20, seed=0, n_roots=10, m_services=4, n_edges=None):
    """Pull-CSR mesh with exactly `n_edges` distinct caller -> callee edges (default
    avg_degree * n_pods; the BASELINE shapes: C2 10k pods / 200k edges, C4 1M / 20M).  Edges are
    drawn per pod (Poisson out-degree) from its service's callee services, deduplicated, topped up
    in further seeded rounds until the target is reached, then a seeded random subset of the
    surplus is dropped.  Pods of callee-less services (the first m_services) call nobody."""
    rng = np.random.default_rng(seed)
    n_srv = max(1, math.ceil(n_pods / service_size))
    s_src, s_dst = _services_ba(n_srv, m_services, rng)
    # callee lists per service (CSR over services)
    order = np.argsort(s_src, kind="stable")
    callee = s_dst[order]
    cptr = np.zeros(n_srv + 1, np.int64)
    np.cumsum(np.bincount(s_src, minlength=n_srv), out=cptr[1:])
    pod_srv = np.arange(n_pods, dtype=np.int64) // service_size
    ncallee = (cptr[1:] - cptr[:-1])[pod_srv]
    callers = np.flatnonzero(ncallee > 0)
    target = int(round(avg_degree * n_pods)) if n_edges is None else int(n_edges)
    # capacity: a pod can call every pod of its callee services except itself
    srv_pods = np.minimum((np.arange(n_srv) + 1) * service_size, n_pods) - np.arange(n_srv) * service_size
    cap_srv = np.zeros(n_srv, np.int64)
    np.add.at(cap_srv, s_src, srv_pods[s_dst])
    target = min(target, int(cap_srv[pod_srv[callers]].sum()))
    key = np.zeros(0, np.int64)
    eff = 0.85  # new distinct edges per drawn edge (re-estimated every round)
    for _ in range(64):
        need = target - len(key)
        if need <= 0:
            break
        draw = need / max(eff, 0.05) * 1.05 + 16
        deg = rng.poisson(draw / max(len(callers), 1), len(callers)).astype(np.int64)
        src = np.repeat(callers, deg)
        k = rng.integers(0, np.iinfo(np.int64).max, len(src)) % np.repeat(ncallee[callers], deg)
        tsrv = callee[cptr[pod_srv[src]] + k]
        lo = tsrv * service_size
        hi = np.minimum(lo + service_size, n_pods)
        dst = lo + rng.integers(0, np.iinfo(np.int64).max, len(src)) % (hi - lo)
        keep = src != dst
        n0 = len(key)
        key = np.union1d(key, src[keep] * n_pods + dst[keep])
        eff = (len(key) - n0) / max(len(src), 1)
    if len(key) > target:  # drop a seeded random subset of the surplus
        key = np.delete(key, rng.choice(len(key), size=len(key) - target, replace=False))
    src, dst = key // n_pods, key % n_pods
    pull = np.sort(dst * n_pods + src)  # rows by destination, callers ascending inside a row
    col = (pull % n_pods).astype(np.int32)
    del pull
    row_ptr = np.zeros(n_pods + 1, np.int64)
    np.cumsum(np.bincount(dst, minlength=n_pods), out=row_ptr[1:])
    outdeg = np.bincount(src, minlength=n_pods).astype(np.int32)
    # roots: pods of distinct, well-called services
    indeg = np.diff(row_ptr)
    cand = np.argsort(-indeg, kind="stable")[: max(n_roots * 50, n_roots)]
    roots = np.sort(rng.choice(cand, size=min(n_roots, len(cand)), replace=False)).astype(np.int64)
    return Mesh(n_pods, row_ptr, col, outdeg, roots)


def chain_roots(mesh, n_chains=5, seed=0):
    """The held-out failure model (nothing in the ranking was tuned on it): two
    faults in one call chain.  For each of `n_chains` downstream roots B (well-called pods of
    distinct services, as make_graph picks its roots), one of B's callers A that has callers of its
    own is a root too: A calls B, both carry a root's spike, and their callers carry the default
    model's symptoms (caller_hops over all 2 * n_chains roots).  -> int64 roots, sorted."""
    rng = np.random.default_rng(int(seed) + 4242)
    indeg = np.diff(mesh.row_ptr)
    cand = np.argsort(-indeg, kind="stable")[: max(n_chains * 50, n_chains)]
    roots, used_srv = [], set()
    for b in rng.permutation(cand):
        b = int(b)
        if b // 20 in used_srv:
            continue
        callers = mesh.col[mesh.row_ptr[b]:mesh.row_ptr[b + 1]].astype(np.int64)
        callers = [int(c) for c in callers if indeg[c] > 0 and c // 20 not in used_srv and c // 20 != b // 20]
        if not callers:
            continue
        a = callers[int(rng.integers(len(callers)))]
        roots += [a, b]
        used_srv.update((a // 20, b // 20))
        if len(roots) == 2 * n_chains:
            break
    return np.sort(np.asarray(roots, np.int64))


def caller_hops(mesh, roots, hops=3, cap=2000):
    """Pods that (transitively) call the roots: list of int64 arrays per hop (capped)."""
    seen = set(int(r) for r in roots)
    frontier = np.asarray(roots, np.int64)
    out = []
    for _ in range(hops):
        nxt = []
        for r in frontier:
            nxt.extend(mesh.col[mesh.row_ptr[r]:mesh.row_ptr[r + 1]].tolist())
        nxt = [c for c in dict.fromkeys(nxt) if c not in seen][:cap]
        seen.update(nxt)
        frontier = np.asarray(nxt, np.int64)
        out.append(frontier)
    return out


def make_metrics(n_pods, n_metrics=8, n_steps=1440, window=60, seed=0, roots=(), hop_sets=(), device="cpu",
                 spike_steps=1, root_sigma=12.0, hop_sigma=5.0, hop_decay=0.8, chunk_steps=None, group_size=0,
                 group_sigma=12.0):
    """-> torch.float32 tensor [T, P, M] (time-major) on `device`.

    group_size > 0 adds a shared load signal per block of `group_size` consecutive pods (a
    service's replicas): a per-group random walk scaled by a per-pod loading in [0.2, 1) *
    group_sigma, which gives the cross-pod correlation structure a9 ranks."""
    import torch
    g = torch.Generator(device=device)
    g.manual_seed(int(seed))
    P, M, T = n_pods, n_metrics, n_steps
    b = torch.rand((P, M), generator=g, device=device) * 30 + 25
    a = torch.rand((P, M), generator=g, device=device) * 12
    sig = torch.rand((P, M), generator=g, device=device) * 2.5 + 0.5
    phi = torch.rand((P, 1), generator=g, device=device) * (2 * math.pi)
    x = torch.empty((T, P, M), dtype=torch.float32, device=device)
    cs = chunk_steps or max(1, min(T, (1 << 28) // max(P * M, 1)))
    for t0 in range(0, T, cs):
        t1 = min(T, t0 + cs)
        tt = torch.arange(t0, t1, device=device, dtype=torch.float32).view(-1, 1, 1)
        blk = b + a * torch.sin(2 * math.pi * tt / 1440.0 + phi) + sig * torch.randn(
            (t1 - t0, P, M), generator=g, device=device)
        x[t0:t1] = blk
    if group_size > 0:
        G = (P + group_size - 1) // group_size
        walk = torch.randn((T, G), generator=g, device=device).cumsum_(0)
        walk = (walk - walk.mean(0)) / walk.std(0).clamp_min(1e-6)
        load = (torch.rand((P, 1), generator=g, device=device) * 0.8 + 0.2) * group_sigma
        gid = torch.arange(P, device=device) // group_size
        for t0 in range(0, T, cs):
            t1 = min(T, t0 + cs)
            x[t0:t1] += walk[t0:t1][:, gid].unsqueeze(2) * load.view(1, P, 1)
    x.clamp_(0.0, 100.0)
    w0 = max(0, T - spike_steps)
    if len(roots):
        r = torch.as_tensor(np.asarray(roots), device=device)
        x[w0:, r, :] = (x[w0:, r, :] + root_sigma * sig[r]).clamp_(0.0, 100.0)
    for h, pods in enumerate(hop_sets):
        if len(pods):
            pr = torch.as_tensor(np.asarray(pods), device=device)
            x[w0:, pr, :] = (x[w0:, pr, :] + (hop_sigma * hop_decay ** h) * sig[pr]).clamp_(0.0, 100.0)
    return x


def make_metrics_range(lo, hi, n_metrics=8, n_steps=1440, window=60, seed=0, roots=(), hop_sets=(), device="cpu",
                       block=62_500, **kw):
    """Pods [lo, hi) of a mesh-wide metric tensor, independent of how the pods are sharded: the
    mesh is generated in fixed blocks of `block` pods (block b seeded seed * 1000 + b), so a rank
    owning [lo, hi) holds exactly the rows a single GPU would hold for those pods."""
    import torch
    x = torch.empty((n_steps, hi - lo, n_metrics), dtype=torch.float32, device=device)
    roots = np.asarray(roots, np.int64)
    hop_sets = [np.asarray(h, np.int64) for h in hop_sets]
    for b in range(lo // block, (hi + block - 1) // block):
        b0, b1 = b * block, (b + 1) * block
        sel = lambda a: a[(a >= b0) & (a < b1)] - b0  # noqa: E731
        xb = make_metrics(block, n_metrics, n_steps, window=window, seed=seed * 1000 + b, roots=sel(roots),
                          hop_sets=[sel(h) for h in hop_sets], device=device, **kw)
        s0, s1 = max(lo, b0), min(hi, b1)
        x[:, s0 - lo:s1 - lo] = xb[:, s0 - b0:s1 - b0]
        del xb
    return x


# ------------------------------------------------------------------------------------------
# log corpora (C5 shape): ASCII templates per category plus benign ones, 60-200 B lines
# ------------------------------------------------------------------------------------------
ERROR_LINES = (
    "Out of memory: Kill process {n} ({w}) score {m}", "container {w} OOMKilled", "signal: killed",
    "dial tcp 10.0.{m}.{n}:5432: connect: connection refused", "Connection refused by {w}",
    "open /var/lib/{w}: permission denied", "403 Forbidden: {w}", "Access denied for {w}",
    "request to {w} timed out after {n}ms", "Timeout waiting for {w}", "read tcp: ETIMEDOUT",
    "Back-off restarting failed container {w}", "pod {w} CrashLoopBackOff",
    "API server error: {w}", "upstream StatusCode=50{d}", "Unable to mount volumes for pod {w}",
    "MountVolume.SetUp failed for volume {w}", "ErrImagePull {w}:{n}", "ImagePullBackOff {w}",
    "DNS resolution failed for {w}", "could not resolve host {w}", "Unauthorized {w}",
    "Authentication failed for {w}", "Invalid configuration {w}", "ConfigMap not found {w}",
    "Secret not found {w}", "500 Internal Server Error {w}", "InternalServerError {w}",
    "Exception in {w}", "ERROR processing batch {n}", "Traceback (most recent call last)",
    "FATAL {w}", "CRITICAL {w}", "panic: {w}",
)
BENIGN_LINES = (
    "INFO GET /api/v1/{w} 200 {n}ms", "DEBUG cache ratio 0.{n}", "Starting worker {n} queue {w}",
    "healthcheck ok {n}", "INFO request id={h} user={w} latency={n}ms", "Reconciling {w} gen {n}",
    "listening on 0.0.0.0:{n}", "WARN slow query {n}ms on {w}", "connected to {w}:{n}",
)
_WORDS = ("frontend", "backend", "db", "cache", "payments", "auth", "queue", "search", "gateway")


def make_log_corpus(n_docs, lines_per_doc=2.5, error_rate=0.3, seed=0, hazard_rate=0.0):
    """-> list[str] of container log texts (Poisson line counts, '\\n' separated)."""
    rng = np.random.default_rng(seed)
    counts = rng.poisson(lines_per_doc, n_docs)
    total = int(counts.sum())
    is_err = rng.random(total) < error_rate
    e_idx = rng.integers(0, len(ERROR_LINES), total)
    b_idx = rng.integers(0, len(BENIGN_LINES), total)
    ns = rng.integers(0, 100000, total)
    ms = rng.integers(0, 256, total)
    ws = rng.integers(0, len(_WORDS), total)
    pad = rng.integers(20, 120, total)
    hz = rng.random(total) < hazard_rate
    # 5 % of the lines carry a trace UUID whose hex groups are mostly letters (a13 masks a UUID as one
    # token, also when a group holds no digit); a generator of its own keeps every other draw as before
    rng_u = np.random.default_rng(int(seed) + 7777)
    has_u = rng_u.random(total) < 0.05
    hexch = np.frombuffer(b"abcdefabcdefabcdef0123456789", np.uint8)
    uu = hexch[rng_u.integers(0, len(hexch), (total, 32))]
    lines = []
    for i in range(total):
        t = ERROR_LINES[e_idx[i]] if is_err[i] else BENIGN_LINES[b_idx[i]]
        s = t.format(n=int(ns[i]), m=int(ms[i]), w=_WORDS[ws[i]], d=int(ns[i]) % 10, h="%08x" % int(ns[i]))
        s = "2024-05-01T00:00:%02d.%03dZ " % (int(ms[i]) % 60, int(ns[i]) % 1000) + s + " " + "k" * int(pad[i] // 4)
        if has_u[i]:
            u = uu[i].tobytes().decode()
            s += " trace=%s-%s-%s-%s-%s" % (u[:8], u[8:12], u[12:16], u[16:20], u[20:])
        if hz[i]:
            s += " café Kelvin ſ"
        lines.append(s)
    docs, k = [], 0
    for c in counts:
        docs.append("\n".join(lines[k:k + c]) + ("\n" if c and rng.random() < 0.5 else ""))
        k += c
    return docs


def spread_hops(mesh, roots, hops=2, per_root=20, seed=0):
    """Callers of each root that carry the fault's symptoms, for the 'spread' ranking scenario
    (DESIGN.md §3.2): per root and hop, up to `per_root` not-yet-chosen callers of that root's
    previous hop, sampled (seeded).  Unlike caller_hops (every caller up to a global cap), the
    anomalous callers stay a small set per root, so the root is what they have in common."""
    rng = np.random.default_rng(int(seed) + 99)
    seen = set(int(r) for r in roots)
    frontier = {int(r): [int(r)] for r in roots}
    out = []
    for _ in range(hops):
        nxt, newf = [], {}
        for r, fr in frontier.items():
            cand = []
            for v in fr:
                cand.extend(mesh.col[mesh.row_ptr[v]:mesh.row_ptr[v + 1]].tolist())
            cand = [c for c in dict.fromkeys(cand) if c not in seen]
            if len(cand) > per_root:
                cand = rng.choice(cand, per_root, replace=False).tolist()
            seen.update(cand)
            nxt.extend(cand)
            newf[r] = cand
        frontier = newf
        out.append(np.asarray(nxt, np.int64))
    return out


# the spread scenario's spikes: callers one hop up carry a LARGER spike than the root itself
SPREAD_SIGMAS = dict(root_sigma=8.0, hop_sigma=9.0, hop_decay=0.9)
