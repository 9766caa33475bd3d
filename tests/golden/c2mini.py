"""Inputs of the C2-mini golden (SURVEY.md §8c golden #7): P = 256 pods, M = 8 metrics,
T = 1440 steps, a 256-node / 5120-edge dependency graph, 256 container logs; seed 0.

Self-contained numpy (PCG64) generator so the fixture does not depend on the product's synthetic
generator; tests/golden/c2mini.npz stores the sha256 of the generated arrays and the test fails
loudly if a numpy release ever changes the streams.  Used by tests/golden/capture_scale.py (which
writes the expected outputs) and by the tests.
"""
import hashlib

import numpy as np

P, M, T, W = 256, 8, 1440, 60
N_EDGES = 5120
SERVICE = 16
ROOTS = (5, 77, 130, 201)

_TEMPLATES = (
    "Out of memory: Kill process {n} ({w})", "dial tcp 10.0.{m}.{n}:5432: connect: connection refused",
    "open /var/lib/{w}: permission denied", "request to {w} timed out after {n}ms",
    "Back-off restarting failed container {w}", "upstream StatusCode=50{d}", "MountVolume.SetUp failed for {w}",
    "ImagePullBackOff {w}:{n}", "could not resolve host {w}", "Unauthorized {w}", "ConfigMap not found {w}",
    "500 Internal Server Error {w}", "Exception in {w} id={h}", "INFO GET /api/v1/{w} 200 {n}ms",
    "DEBUG cache ratio 0.{n}", "healthcheck ok {n}", "connected to {w}:{n}", "WARN slow query {n}ms on {w}",
)
_WORDS = ("frontend", "backend", "db", "cache", "payments", "auth", "queue")


def graph():
    """Edges caller -> callee (int64 [E, 2]), services of 16 pods, callers of a service's pods
    drawn from lower-numbered services; exactly N_EDGES distinct edges, no self loops."""
    rng = np.random.default_rng(0)
    edges = set()
    while len(edges) < N_EDGES:
        u = int(rng.integers(SERVICE, P))
        v = int(rng.integers(0, (u // SERVICE) * SERVICE))
        edges.add((u, v))
    return np.array(sorted(edges), np.int64)


def metrics(edges):
    """float32 [T, P, M] time-major; roots spike 12 sigma at the last step, their callers 5 sigma."""
    rng = np.random.default_rng(1)
    b = rng.uniform(25, 55, (P, M))
    a = rng.uniform(0, 12, (P, M))
    sig = rng.uniform(0.5, 3.0, (P, M))
    phi = rng.uniform(0, 2 * np.pi, (P, 1))
    t = np.arange(T, dtype=np.float64)[:, None, None]
    x = b + a * np.sin(2 * np.pi * t / 1440.0 + phi) + sig * rng.standard_normal((T, P, M))
    grp = rng.standard_normal((T, P // SERVICE)).cumsum(0)
    grp = (grp - grp.mean(0)) / grp.std(0)
    x += grp[:, np.arange(P) // SERVICE, None] * rng.uniform(2, 10, (1, P, 1))
    x = np.clip(x, 0, 100)
    roots = np.array(ROOTS)
    x[-1, roots, :] = np.clip(x[-1, roots, :] + 12 * sig[roots], 0, 100)
    callers = np.unique(edges[np.isin(edges[:, 1], roots), 0])
    callers = callers[~np.isin(callers, roots)]
    x[-1, callers, :] = np.clip(x[-1, callers, :] + 5 * sig[callers], 0, 100)
    return x.astype(np.float32)


def logs():
    """256 container texts ('\\n' separated, Poisson line counts, a few non-ASCII hazards)."""
    rng = np.random.default_rng(2)
    docs = []
    for _ in range(P):
        lines = []
        for _ in range(int(rng.poisson(6))):
            tpl = _TEMPLATES[int(rng.integers(len(_TEMPLATES)))]
            n = int(rng.integers(0, 100000))
            s = tpl.format(n=n, m=n % 256, d=n % 10, w=_WORDS[n % len(_WORDS)], h="%08x" % n)
            if rng.random() < 0.03:
                s += " café Kelvin"
            lines.append(s)
        docs.append("\n".join(lines) + ("\n" if lines and rng.random() < 0.5 else ""))
    return docs


def pack(docs):
    enc = [d.encode("utf-8", "surrogatepass") for d in docs]
    off = np.zeros(len(enc) + 1, np.int64)
    np.cumsum([len(e) for e in enc], out=off[1:])
    return b"".join(enc), off


def sha(*arrays):
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def inputs():
    e = graph()
    x = metrics(e)
    blob, off = pack(logs())
    return e, x, blob, off
