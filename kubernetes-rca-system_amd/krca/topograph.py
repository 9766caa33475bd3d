"""Host side of the service-graph construction kernels.

TopologyAgent._build_service_graph (ref:agents/topology_agent.py:94-160) tests every
(deployment, service) pair with ``all(item in labels.items() for item in selector.items())``,
_infer_dependencies_from_env (:228-260) every (env value, DNS key) pair with ``key in value``,
and ResourceAnalyzer._find_matching_pods (ref:agents/resource_analyzer.py:835-854) every
(service, pod) pair with ``all(k in labels and labels[k] == v ...)``.  The all-pairs tests run on
the device (csrc/topograph.hip: krca_selector_match, krca_substr_match); this module interns the
label items to dense ids, packs the strings and turns the device output back into per-row match
lists in the order the reference visits them.
"""
import numpy as np


class ItemIds:
    """Dense ids of (key, value) label items under the equality the reference's test uses.

    ``identity=True`` is ItemsView membership (``mapping[k] is v or mapping[k] == v``), which is
    also what a tuple-keyed dict does; ``identity=False`` is the plain ``labels[k] == v`` of
    _find_matching_pods, under which a value that is not equal to itself (NaN) matches nothing.
    Unhashable values (a list as a label value) get ids by equality search."""

    def __init__(self, identity=True):
        self.identity = identity
        self._ids = {}
        self._odd = []  # (key, value, id) for unhashable values
        self.n = 0

    def _new(self):
        self.n += 1
        return self.n - 1

    def get(self, k, v, add):
        try:
            hash(v)
        except TypeError:
            for kk, vv, i in self._odd:
                if kk == k and ((self.identity and vv is v) or vv == v):
                    return i
            if not add:
                return None
            i = self._new()
            self._odd.append((k, v, i))
            return i
        if not self.identity and v != v:  # never equal to anything, itself included
            return self._new() if add else None
        i = self._ids.get((k, v))
        if i is None and add:
            i = self._ids[(k, v)] = self._new()
        return i


def pack_item_sets(item_lists, ids, add):
    """[[(k, v), ...], ...] -> (int32 ids, int64 offsets); with add=False items no selector
    mentions are dropped (they cannot decide a match)."""
    out, off = [], [0]
    for items in item_lists:
        for k, v in items:
            i = ids.get(k, v, add)
            if i is not None:
                out.append(i)
        off.append(len(out))
    return np.asarray(out, np.int32), np.asarray(off, np.int64)


def selector_bits(engine, object_items, selector_items, identity=True):
    """Device all-pairs selector test -> uint64 bits [n_objects][ceil(n_selectors/64)]."""
    ids = ItemIds(identity)
    sel, sel_off = pack_item_sets(selector_items, ids, True)
    lab, lab_off = pack_item_sets(object_items, ids, False)
    return engine.selector_match(lab, lab_off, sel, sel_off)


def match_rows(bits, S, chunk=4096):
    """Yield, per object row, the ascending selector indices whose bit is set."""
    for r0 in range(0, bits.shape[0], chunk):
        m = np.unpackbits(np.ascontiguousarray(bits[r0:r0 + chunk]).view(np.uint8), axis=1, bitorder="little")[:, :S]
        for row in m:
            yield np.flatnonzero(row)


def match_cols(bits, S, chunk=4096):
    """Per selector, the ascending object indices whose bit is set."""
    rows, cols = [], []
    for r0 in range(0, bits.shape[0], chunk):
        m = np.unpackbits(np.ascontiguousarray(bits[r0:r0 + chunk]).view(np.uint8), axis=1, bitorder="little")[:, :S]
        r, c = np.nonzero(m)
        rows.append(r + r0)
        cols.append(c)
    rows = np.concatenate(rows) if rows else np.zeros(0, np.int64)
    cols = np.concatenate(cols) if cols else np.zeros(0, np.int64)
    order = np.argsort(cols, kind="stable")  # rows ascend within each column
    rows, cols = rows[order], cols[order]
    cuts = np.searchsorted(cols, np.arange(S + 1))
    return [rows[cuts[s]:cuts[s + 1]].tolist() for s in range(S)]


def pack_strings(strs):
    """list[str] -> (UTF-8 blob, int64 offsets).  Lone surrogates pass through."""
    enc = [s.encode("utf-8", "surrogatepass") for s in strs]
    off = np.zeros(len(enc) + 1, np.int64)
    if enc:
        off[1:] = np.cumsum([len(e) for e in enc])
    return b"".join(enc), off


def substring_matches(engine, values, keys):
    """For str values and keys: per value, the ascending key indices k with keys[k] in value."""
    V, K = len(values), len(keys)
    out = [[] for _ in range(V)]
    if not V or not K:
        return out
    text, voff = pack_strings(values)
    pat, poff = pack_strings(keys)
    pairs = engine.substr_match(text, voff, pat, poff)
    for v, k in zip((pairs // K).tolist(), (pairs % K).tolist()):
        out[v].append(k)
    return out
