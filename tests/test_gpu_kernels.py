"""Parity of the HIP kernels (through the C-ABI) against the oracle, on an MI355X.

Integer outputs bit-exact; float outputs within the tolerance stated per test; top-k identical.
"""
import numpy as np
import pytest
import torch

import oracle
from krca import native, synth
from krca.agents.logs import pack_documents

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    return native.NativeEngine()


# ---- a1/a2 thresholds ------------------------------------------------------------------------
def test_usage_flags_bit_exact(eng):
    rng = np.random.default_rng(0)
    u = rng.uniform(0, 100, (100003, 2)).astype(np.float32)
    edge = np.array([80, 90, np.nextafter(np.float32(80), 100), np.nextafter(np.float32(90), 0), 0, 100,
                     np.nan, -np.inf, np.inf], np.float32)
    u[:len(edge), 0] = edge
    u[:len(edge), 1] = edge[::-1]
    assert np.array_equal(eng.usage_flags(u), oracle.c_usage_flags(u))


# ---- a5 rolling z-score ------------------------------------------------------------------------
ROLL_CASES = [  # (P, M, T, W)
    (1000, 8, 1440, 60), (513, 8, 300, 60), (700, 8, 200, 30), (300, 4, 97, 20), (300, 2, 64, 15),
    (200, 8, 50, 10), (128, 8, 60, 60), (128, 8, 61, 60), (64, 8, 20, 60), (100, 8, 300, 45), (77, 1, 90, 7),
    (64, 16, 150, 60), (32, 64, 130, 60),
]


@pytest.mark.parametrize("P,M,T,W", ROLL_CASES)
def test_rolling_score_vs_oracle(eng, P, M, T, W):
    mesh_roots = np.arange(0, P, max(1, P // 7))
    x = synth.make_metrics(P, M, T, window=W, seed=P + T, roots=mesh_roots)
    got = eng.rolling_score(x.cuda(), window=W, z_threshold=3.0)
    ref = oracle.c_rolling_score(x.numpy(), W, 3.0)
    assert np.array_equal(got["n_exceed_host"], ref["n_exceed"])        # bit-exact
    assert np.array_equal(got["flags"], ref["flags"])                    # bit-exact
    z = got["z_last"].cpu().numpy()
    assert np.allclose(z, ref["z_last"], rtol=1e-5, atol=1e-6)           # 1e-5 relative
    assert np.allclose(got["score"].cpu().numpy(), ref["score"], rtol=1e-5, atol=1e-6)
    zl, sc, _ = oracle.rolling_score_f64(x.numpy(), W)                   # independent f64 formulation
    assert np.allclose(z, zl, rtol=1e-5, atol=1e-5)


def test_rolling_score_non_finite_samples_as_oracle(eng):
    """Non-finite samples are outside the reference's inputs (missing metrics are absent, not NaN);
    the contract is only that a NaN / +-Inf in a series never faults and gives what the C twin
    gives: counts and flags bit-exact, z / score equal (NaN where the twin has NaN)."""
    P, M, T, W = 300, 8, 200, 30
    x = synth.make_metrics(P, M, T, window=W, seed=41, roots=np.arange(0, P, 11)).numpy().copy()
    rng = np.random.default_rng(41)
    for val in (np.nan, np.inf, -np.inf):
        idx = rng.integers(0, x.size, 40)
        x.reshape(-1)[idx] = val
    got = eng.rolling_score(torch.from_numpy(x).cuda(), window=W, z_threshold=3.0)
    ref = oracle.c_rolling_score(x, W, 3.0)
    assert np.array_equal(got["n_exceed_host"], ref["n_exceed"])
    assert np.array_equal(got["flags"], ref["flags"])
    assert np.allclose(got["z_last"].cpu().numpy(), ref["z_last"], rtol=1e-5, atol=1e-6, equal_nan=True)
    assert np.allclose(got["score"].cpu().numpy(), ref["score"], rtol=1e-5, atol=1e-6, equal_nan=True)


SCORE_VARIANTS = [("2", "20"), ("1", "20"), ("4", "20"), ("4", "15"), ("5", "20")] + [("0", c) for c in ("10", "12", "15", "20", "30")]


@pytest.mark.parametrize("P,M,T,W", [(1000, 8, 1440, 60), (128, 8, 61, 60), (129, 8, 139, 60), (700, 8, 200, 30)])
def test_rolling_score_kernel_variants_bit_exact(eng, monkeypatch, P, M, T, W):
    """Every kernel form (W-block buffer loads, plain loads, pipelined chunks, LDS-DMA rows) = the C oracle."""
    x = synth.make_metrics(P, M, T, window=W, seed=P + T + 1, roots=np.arange(0, P, 9))
    ref = oracle.c_rolling_score(x.numpy(), W, 3.0)
    xd = x.cuda()
    z0 = None
    for impl, chunk in SCORE_VARIANTS:
        with native.tune(eng.lib, KRCA_SCORE_IMPL=int(impl), KRCA_SCORE_CHUNK=int(chunk)):
            got = eng.rolling_score(xd, window=W, z_threshold=3.0)
        assert np.array_equal(got["n_exceed_host"], ref["n_exceed"]), (impl, chunk)
        assert np.array_equal(got["flags"], ref["flags"]), (impl, chunk)
        z = got["z_last"].cpu().numpy()
        assert np.allclose(z, ref["z_last"], rtol=1e-5, atol=1e-6), (impl, chunk)
        z0 = z if z0 is None else z0
        assert np.array_equal(z, z0), (impl, chunk)                       # same arithmetic -> same bits


def test_rolling_score_deterministic_and_planted_roots(eng):
    m = synth.make_graph(2000, avg_degree=10, seed=1)
    hops = synth.caller_hops(m, m.roots)
    x = synth.make_metrics(2000, 8, 1440, roots=m.roots, hop_sets=hops, seed=2).cuda()
    a = eng.rolling_score(x)
    b = eng.rolling_score(x)
    assert torch.equal(a["score"], b["score"]) and np.array_equal(a["n_exceed_host"], b["n_exceed_host"])
    idx, _ = eng.topk(a["score"], len(m.roots))
    assert set(idx.tolist()) == set(m.roots.tolist())


# ---- top-k -----------------------------------------------------------------------------------
@pytest.mark.parametrize("N,k", [(1, 1), (10, 10), (1000, 10), (1 << 20, 10), (3_000_001, 16), (777, 5)])
def test_topk_float_and_int(eng, N, k):
    rng = np.random.default_rng(N)
    v = rng.integers(0, 50, N).astype(np.float32)  # many ties -> index tie-break
    idx, val = eng.topk(torch.from_numpy(v), k)
    ridx, rval = oracle.topk_ref(v, k)
    assert np.array_equal(idx, ridx) and np.array_equal(val, rval)
    vi = rng.integers(-(1 << 62), 1 << 62, N).astype(np.int64)
    vi[::7] = 12345
    idx, val = eng.topk(torch.from_numpy(vi), k)
    ridx, rval = oracle.topk_ref(vi, k)
    assert np.array_equal(idx, ridx) and np.array_equal(val, rval)


def test_topk_nan_never_selected(eng):
    v = np.full(5000, np.nan, np.float32)
    v[[3, 4000]] = [1.0, 2.0]
    idx, val = eng.topk(torch.from_numpy(v), 2)
    assert idx.tolist() == [4000, 3]
    # fewer than k non-NaN keys: the rest are the sentinel, never a NaN entry
    idx, val = eng.topk(torch.from_numpy(v), 5)
    assert idx.tolist() == [4000, 3, -1, -1, -1]
    assert val[:2].tolist() == [2.0, 1.0] and np.all(np.isneginf(val[2:]))
    w = np.full(300, np.nan, np.float32)
    w[7] = -np.inf  # a real -inf key still beats the sentinel
    idx, val = eng.topk(torch.from_numpy(w), 3)
    assert idx.tolist() == [7, -1, -1]


# ---- a12 log histograms ----------------------------------------------------------------------
def _check_docs(eng, docs):
    blob, off = pack_documents(docs)
    scan = eng.log_scan(blob, off)
    for d, text in enumerate(docs):
        n, h, ex = oracle.log_hist(text)
        assert scan.n_lines[d] == n, (d, repr(text[:80]))
        assert scan.hist[d].tolist() == h, (d, repr(text[:80]))
        for c in range(13):
            assert scan.examples(d, c) == ex[c], (d, c)


@pytest.mark.parametrize("knobs", [dict(KRCA_LOG_FUSED=0), dict(KRCA_LOG_FUSED=1), dict(KRCA_LOG_FUSED=2),
                                   dict(KRCA_LOG_FUSED=0, KRCA_LOG_IMPL=1), dict(KRCA_LOG_FUSED=0, KRCA_LOG_IMPL=2)])
def test_log_scan_no_match_across_container_end(eng, knobs):
    """A container without a trailing separator ends its last line: the next container's first
    bytes must not complete a pattern ("Erro" | "r", "StatusCode=50" | "0", "OOMKille" | "d"),
    nor may the bytes after the text's end; at every offset of the 16-byte block, every walk."""
    docs = []
    for pad in range(16):
        docs += ["p" * pad + " state Erro", "r happened", "x StatusCode=50", "0 y", "OOMKille", "d z",
                 "q" * pad + "Kille", "d", "Tracebac", "k", "panic", ": x", "time", "out"]
    docs.append("tail StatusCode=50")  # the text's last bytes
    with native.tune(eng.lib, **knobs):
        _check_docs(eng, docs)


@pytest.mark.parametrize("knobs", [dict(KRCA_LOG_FUSED=0), dict(KRCA_LOG_FUSED=1), dict(KRCA_LOG_FUSED=2),
                                   dict(KRCA_LOG_FUSED=0, KRCA_LOG_IMPL=1), dict(KRCA_LOG_FUSED=0, KRCA_LOG_IMPL=2)])
def test_log_scan_fragment_fuzz(eng, knobs):
    """Every literal alternative of the 13 patterns cut at a random point, its halves scattered
    over lines and containers with separators, multi-byte characters and fillers of random length
    (so pattern halves meet at container ends without a trailing separator, at 16-byte block edges,
    at line ends and across separators): histograms and examples equal the oracle's, every walk."""
    import re as _re
    from krca.patterns import ERROR_PATTERNS
    lits = [a for _, p in ERROR_PATTERNS for a in p.strip("()").split("|")]
    lits = [_re.sub(r"\\d", "7", a).replace("\\", "") for a in lits]  # StatusCode=5\d\d -> digits
    rng = np.random.default_rng(21)
    seps = ["\n", "\r", "\r\n", "\x0b", "\x0c", "\x1c", "\x1d", "\x1e", "\x85", "\u2028", "\u2029", ""]
    other = ["é", "İ", "\u212a", "ſ", "x", " ", "0", "a" * 13, "q" * 40]
    docs = []
    for _ in range(1500):
        parts = []
        for _ in range(int(rng.integers(0, 12))):
            r = rng.random()
            if r < 0.45:
                a = lits[int(rng.integers(0, len(lits)))]
                cut = int(rng.integers(0, len(a) + 1))
                parts.append(a[:cut] if rng.random() < 0.5 else a[cut:])
            elif r < 0.6:
                parts.append(lits[int(rng.integers(0, len(lits)))])
            elif r < 0.8:
                parts.append(seps[int(rng.integers(0, len(seps)))])
            else:
                parts.append(other[int(rng.integers(0, len(other)))] * int(rng.integers(1, 4)))
        docs.append("".join(parts))
    with native.tune(eng.lib, **knobs):
        _check_docs(eng, docs)


@pytest.mark.parametrize("fused", [0, 1, 2])
def test_log_scan_degenerate_texts(eng, fused):
    """An all-empty window (one and several empty containers: no text at all), a text of exactly one
    16-byte piece / one 32 KiB / one 64 KiB tile, a single separator, a text of separators only;
    histograms, line counts and the template histograms against the oracle."""
    cases = [[""], ["", "", ""], ["x" * 15 + "\n"], ["\n"], ["\r\n" * 7 + "\x85"],
             ["a" * 32767 + "\n"], ["Error " * 5461 + "ab"], ["b" * 65535 + "\n", ""], ["", "Killed", ""]]
    with native.tune(eng.lib, KRCA_LOG_FUSED=fused):
        for docs in cases:
            _check_docs(eng, docs)
            got = eng.template_hist(*pack_documents(docs))
            assert got == [oracle.template_hist(d) for d in docs], [len(d) for d in docs]


def test_log_scan_reference_corpus(eng):
    import json
    import os
    from conftest import GOLDEN
    g = json.load(open(os.path.join(GOLDEN, "logs_corpus.json")))
    docs = [c["text"] for c in g["containers"]]
    _check_docs(eng, docs)
    # per-line masks against the masks the reference produced
    blob, off = pack_documents(docs)
    r = eng.log_scan_device(eng.upload_blob(blob), torch.from_numpy(off).cuda())
    masks = (r["line_mask"].cpu().numpy() & 0x1FFF).tolist()  # bits 16-28: the example marks
    assert masks == [m for c in g["containers"] for m in c["masks"]]


def test_log_scan_boundaries(eng):
    """Separators, multi-byte characters and lines straddling 256-byte chunks / 64 KiB tiles."""
    rng = np.random.default_rng(7)
    docs = ["", "\n", "\r\n", "\r", "a", "x\r\ny", "\n\n\n", "Killed\r", " ", "timeout Killed\x85panic:",
            "", "e" * 255 + "\r\n" + "Error", "f" * 254 + "é" + "Timeout", "g" * 253 + " " + "ERROR",
            "h" * 300000 + " Traceback " + "i" * 70000, "StatusCode=5" + "٣٤" + "\n" + "K" + "illed"]
    for L in (250, 255, 256, 257, 511, 512, 65535, 65536, 65537):
        docs.append("x" * (L - 8) + "timeout\r" + "\nERROR")
    pieces = ["Error", "\r", "\n", "\r\n", "é", "KILLED", "\u0085", "ſecret not found", "a" * 37, "panic:",
              "Back-off restarting", "\x1c", "\x0b", " ", "\u2028", "\u2029", "\x1d", "\x1e", "\x0c", "\u00e2\u0080"]
    for _ in range(200):
        docs.append("".join(pieces[i] for i in rng.integers(0, len(pieces), rng.integers(0, 60))))
    # containers ending in a separator followed by containers starting with one (the line-start
    # test at a container's first byte must not see the previous container's bytes)
    docs += ["a\r", "\nb", "x\u2028", "\u2029y", "\r", "\n", "q\x85", "\x85", "", "\u2028", "z\r", "\r\n"]
    _check_docs(eng, docs)


def test_log_scan_container_starts_at_tile_boundaries(eng):
    """Container starts placed exactly at 64 KiB tile boundaries (k*65536) and one byte before
    (k*65536-1), with \r / \n / CRLF pairs split across the container edge and empty containers
    there: log_count / log_lines read the container starts of a tile (and the byte at tile0-1)
    from a per-tile LDS bitmap."""
    TILE = 65536
    tails = ["\r", "x\r", "Error\n", "", "timeout"]
    heads = ["\nKilled", "\n", "\r\npanic:", "ERROR", "", "\x85z"]
    docs, pos, k = [], 0, 1
    for i in range(24):
        target = k * TILE - (i % 2)  # even i: start at the boundary, odd: one byte before it
        tail = tails[i % len(tails)]
        fill = target - pos - len(tail.encode())
        if fill < 0:
            k += 1
            continue
        docs.append("a" * max(fill - 1, 0) + (" " if fill else "") + tail)
        pos += len(docs[-1].encode())
        assert pos == target
        if i % 3 == 0:
            docs += ["", ""]  # empty containers at the boundary
        docs.append(heads[i % len(heads)] + " Error timeout")
        pos += len(docs[-1].encode())
        k += 1
    _check_docs(eng, docs)


def test_log_scan_impls_identical(eng, monkeypatch):
    """The line-index + DFA-lane path (default) and the chunk-lane path (KRCA_LOG_IMPL=1) give the
    same line offsets, masks, histograms and examples, long lines (> 1 KiB, a wave each) included."""
    rng = np.random.default_rng(11)
    docs = synth.make_log_corpus(3000, lines_per_doc=4, seed=5, hazard_rate=0.02)
    docs += ["x" * 5000 + " Killed " + "y" * 3000 + "\n" + "z" * 1025 + "timeout", "é" * 2000 + "panic:",
             "a\r", "\nb", "ſ" * 700 + "Error" + "\u2028" + "k" * 1100, ""]
    docs += ["".join(rng.choice(["Error ", "\r\n", "é", "\x85", "OOMKilled", "w" * 300]) for _ in range(40))
             for _ in range(50)]
    blob, off = pack_documents(docs)
    tb, toff = eng.upload_blob(blob), torch.from_numpy(off).cuda()
    out = {}
    for impl in ("0", "1", "2"):
        with native.tune(eng.lib, KRCA_LOG_IMPL=int(impl)):
            r = eng.log_scan_device(tb, toff)
            out[impl] = {k: v.cpu().numpy() for k, v in r.items() if hasattr(v, "cpu")}
    for other in ("1", "2"):
        assert out["0"].keys() == out[other].keys()
        for k in out["0"]:
            assert np.array_equal(out["0"][k], out[other][k]), (other, k)
    _check_docs(eng, docs)


def test_log_scan_block_edges(eng):
    """log_dfa walks 16-byte blocks from each line's 4-byte-aligned start: lines starting at every
    offset mod 16, multi-byte code points (2, 3 and 4 bytes, case folds) straddling block and word
    edges, matches ending on the last byte of a block, and texts ending at every offset mod 16
    (the buffer load straddling the text's end)."""
    docs = []
    for k in range(20):
        for cp in ("é", "€", "\U0001d400", "\u212a", "ſ"):
            docs.append("a" * k + cp + "Error" + "\n" + "b" * (k % 7) + "Killed" + cp * 3)
        docs.append("c" * k + "timeout")  # a match ending at every offset
        docs.append(" " * (k % 5) + "\u212aILLED " + "x" * k + "secret not found")
    _check_docs(eng, docs)
    for tail in range(17):
        _check_docs(eng, ["z" * 11 + "\n" + "Error" * 3 + "q" * tail])
        _check_docs(eng, ["y" * (37 + tail) + "é" + "panic:"])


@pytest.mark.parametrize("fused", [1, 2])
def test_log_scan_fused_multibyte_lines(eng, fused):
    """The fused walk keeps bytes >= 0x80 as they are among the ASCII symbol offsets and decodes a
    block's code points when one is there: a text where nearly every line holds 2-, 3- and 4-byte
    characters (case folds among them: K, ſ, İ) equals the oracle, short lines and split long ones."""
    rng = np.random.default_rng(23)
    words = ["é", "Error", "\u212aILLED", "ſecret not found", "panic:", "x", "Tim\u0130eout", "€", " ", "\U0001d400"]
    docs = ["\n".join("".join(rng.choice(words, 4)) for _ in range(400)) for _ in range(10)]
    # lines over 88 bytes are walked by two lanes, the second warmed up over the 23 bytes before the
    # split point, or 95 when one of them is >= 0x80: matches and multi-byte characters across it
    docs += ["\n".join("".join(rng.choice(words, int(rng.integers(10, 90)))) for _ in range(60)) for _ in range(10)]
    with native.tune(eng.lib, KRCA_LOG_FUSED=fused):
        _check_docs(eng, docs)


def test_log_scan_synthetic_large(eng):
    docs = synth.make_log_corpus(20000, lines_per_doc=6, seed=3, hazard_rate=0.01)
    _check_docs(eng, docs)


def test_log_scan_one_call_and_fallback_identical(eng):
    """krca_log_scan (line index in one pass with a decoupled look-back over > 64 tiles, every later
    kernel on the device line count) equals the two-call protocol (krca_log_index, then
    krca_log_match), both when its line arrays are too small (it leaves the index in the workspace
    and krca_log_match takes over) and when they hold every line."""
    docs = synth.make_log_corpus(40000, lines_per_doc=5, seed=8, hazard_rate=0.02)
    docs += ["a\r", "\nb", "x ", " y", "q\x85", "", "z\r", "\r\n", "é" * 3000 + "Killed"]
    blob, off = pack_documents(docs)
    assert len(blob) > 65 * 65536  # look-back windows of 64 tiles
    tb, toff = eng.upload_blob(blob), torch.from_numpy(off).cuda()
    fresh = native.NativeEngine()
    out = []
    for e, impl in ((fresh, 0), (fresh, 0), (eng, 1)):  # fallback (cap 1024), one call, two calls
        with native.tune(e.lib, KRCA_LOG_IMPL=impl):
            r = e.log_scan_device(tb, toff)
            out.append({k: v.cpu().numpy() for k, v in r.items() if hasattr(v, "cpu")})
    assert fresh._log_cap >= out[0]["line_start"].shape[0]
    for o in out[1:]:
        for k in out[0]:
            assert np.array_equal(out[0][k], o[k]), k
    # the dense example table (A/B form) equals the example bits of the masks, in both protocols
    for e in (fresh, eng):
        r = e.log_scan_device(tb, toff, dense_examples=True)
        bits = native.example_ids(r["line_mask"].cpu().numpy(), r["doc_line0"].cpu().numpy(),
                                  r["doc_lines"].cpu().numpy())
        assert np.array_equal(r["examples"].cpu().numpy(), bits)
        assert np.array_equal(r["line_mask"].cpu().numpy(), out[0]["line_mask"])


def test_log_scan_fused_walk_identical(eng):
    """krca_log_scan's fused pass (log_index_match: the DFA walks each tile's lines from LDS in the
    line-index pass, a tile's last line over the 1 KiB loaded after the tile; lines over 1 KiB and
    lines holding a byte >= 0x80 go to log_dfa_long),
    in both shapes (KRCA_LOG_FUSED=1: 32 KiB tiles, 16-bit table; 2: 64 KiB tiles, 32-bit table), equals
    the round-3 path (KRCA_LOG_FUSED=0: the index, then log_dfa re-reading the text) on every
    output, and the oracle: tiles of more than 4,096 lines (several list windows per tile: 2-byte
    and empty lines), lines straddling one and several tiles (a 300 KiB line leaves whole tiles
    without a line start), CRLF and U+2028 split across a tile edge, lines of exactly 1,024 and
    1,025 bytes, a text ending mid-piece."""
    rng = np.random.default_rng(13)
    docs = synth.make_log_corpus(5000, lines_per_doc=4, seed=12, hazard_rate=0.02)
    docs.append("e\n" * 40000)                         # 2-byte lines: ~32k lines per tile
    docs.append("\n" * 70000 + "Error")                # empty lines
    docs.append("k" * 300_000 + " OOMKilled " + "m" * 1000)  # tiles with no line start
    docs.append("x" * 1024 + "\n" + "y" * 1020 + "Error\n" + "z" * 1023)  # 1024 / 1025 bytes

    def to_tile_end(extra):  # filler so that the next byte sits `extra` bytes before a tile edge
        pos = sum(len(d.encode()) for d in docs) + 1
        return (-pos - extra) % 65536 + 1
    docs.append("p" * to_tile_end(1) + "\r\nKilled timeout")  # CRLF split across a tile edge
    docs.append("w" * to_tile_end(1) + "\u2028 Traceback")    # U+2028 split across a tile edge
    # a tile's last line ending in the 1,024 bytes loaded after the tile: its next line starting at
    # the last of them (+1023) and just past them (+1024: log_dfa_long), lengths 1,024 and 1,025,
    # a match across the tile edge
    for m in (1017, 1018):
        docs.append("r" * to_tile_end(2) + "\n" + "Erro" + "r" + "t" * m + "\nnext")
    for m in (1018, 1019, 1020):
        docs.append("s" * to_tile_end(3) + "\n" + "Tim" + "eout" + "u" * (m - 2))
    docs.append("c" * to_tile_end(4) + "\nKil" + "led é" + "d" * 900 + "\nend")  # a multi-byte character in it
    docs.append("g" * to_tile_end(2) + "\né" + "\u212a" + "illed")  # one split across the tile edge
    docs += ["".join(rng.choice(["Error ", "\r\n", "é", "\x85", "panic:", "v" * 200, " "]) for _ in range(30))
             for _ in range(300)]
    docs.append("tail Error é")                        # the text ends mid-piece
    nb = sum(len(d.encode()) for d in docs)
    if (nb + 32767) // 32768 % 2 == 0:  # an odd number of 32 KiB tiles: the last 64 KiB tile is half-covered
        docs.append("f" * 32768 + " ERROR")
    blob, off = pack_documents(docs)
    assert (len(blob) + 32767) // 32768 % 2 == 1
    tb, toff = eng.upload_blob(blob), torch.from_numpy(off).cuda()
    nws = 8 * int(eng.lib.krca_log_index_size(len(blob)))
    out = {}
    # the fused pass with line arrays that hold every line, the fallback (krca_log_match after a
    # krca_log_scan into too small arrays: a fresh engine), and the round-3 path; the workspace is
    # filled with garbage before each call (what the scan leaves unwritten must not be read)
    for name, fused, fresh in (("fused", 1, False), ("fallback", 1, True), ("fused64", 2, False),
                               ("fallback64", 2, True), ("unfused", 0, False)):
        e = native.NativeEngine() if fresh else eng
        e._workspace("logidx", nws).fill_(0x5B)
        with native.tune(e.lib, KRCA_LOG_FUSED=fused):
            if not fresh:
                e.log_scan_device(tb, toff)  # sizes the engine's line arrays
                e._workspace("logidx", nws).fill_(0x5B)
            r = e.log_scan_device(tb, toff)
            out[name] = {k: v.cpu().numpy() for k, v in r.items() if hasattr(v, "cpu")}
    for name in ("fallback", "fused64", "fallback64", "unfused"):
        assert out["fused"].keys() == out[name].keys()
        for k in out["fused"]:
            assert np.array_equal(out["fused"][k], out[name][k]), (name, k)
    _check_docs(eng, docs)


# ---- a10 personalized PageRank ---------------------------------------------------------------
def test_ppr_known_answer(eng):
    import json
    import os
    from conftest import GOLDEN
    from krca.agents.topology import csr_from_edges
    g = json.load(open(os.path.join(GOLDEN, "ppr_known.json")))
    names = g["nodes"]
    pos = {n: i for i, n in enumerate(names)}
    rp, col, od = csr_from_edges(len(names), [pos[s] for s, _ in g["edges"]], [pos[d] for _, d in g["edges"]])
    seed = np.array([g["personalization"][n] for n in names], np.float32)
    r, rf, it = eng.ppr(rp, col, od, seed, g["alpha"])
    ref = np.array([g["pagerank"][n] for n in names])
    assert np.allclose(r.cpu().numpy(), ref, rtol=1e-5, atol=0)
    rfo, ro, ito = oracle.c_ppr(rp, col, od, seed, g["alpha"])
    assert np.array_equal(rf.cpu().numpy(), ro) and it == ito


@pytest.mark.parametrize("n,deg,tol,iters", [(5000, 8, 1e-6, 100), (20000, 20, 0.0, 30), (3000, 3, 1e-9, 300)])
def test_ppr_bit_exact_vs_oracle(eng, n, deg, tol, iters):
    m = synth.make_graph(n, avg_degree=deg, seed=n)
    rng = np.random.default_rng(n)
    seed = (rng.random(n) ** 8).astype(np.float32)
    r, rf, it = eng.ppr(m.row_ptr, m.col, m.outdeg, seed, 0.85, iters, tol)
    rfo, ro, ito = oracle.c_ppr(m.row_ptr, m.col, m.outdeg, seed, 0.85, iters, tol)
    assert it == abs(ito)
    assert np.array_equal(rf.cpu().numpy(), ro)  # bit-identical fixed point
    # float64 restatement fed the same 2^-32-quantised seeds: 1e-5 relative on every rank that
    # carries at least 1e-9 of the mass (below that the 2^-60 fixed point is the tolerance)
    qs = np.floor(seed.astype(np.float64) * 2.0 ** 32) / 2.0 ** 32
    x, _ = oracle.ppr_f64(m.row_ptr, m.col, m.outdeg, qs, 0.85, it, 0.0)
    rr = r.cpu().numpy().astype(np.float64)
    big = x >= 1e-9
    assert np.max(np.abs(rr[big] - x[big]) / x[big]) < 1e-5
    assert np.max(np.abs(rr[~big] - x[~big])) < 1e-13
    idx, _ = eng.topk(rf, 10)
    assert np.array_equal(idx, oracle.topk_ref(ro, 10)[0])


@pytest.mark.parametrize("grid", [16, 40, 0])
def test_ppr_xcd_entry_map_bit_identical(eng, grid):
    """KRCA_PPR_XCD: workgroups g, g + 8, ... take one contiguous eighth of the plan entries (small
    grids force nblk >= grid at 40k pods; grid 0 = the occupancy grid, where the map stays off below
    that many blocks); tolerance runs included (the converged early exit)."""
    m = synth.make_graph(40000, avg_degree=12, seed=5)
    rng = np.random.default_rng(5)
    seed = (rng.random(40000) ** 8).astype(np.float32)
    rfo, ro, ito = oracle.c_ppr(m.row_ptr, m.col, m.outdeg, seed, 0.85, 40, 1e-9)
    with native.tune(eng.lib, KRCA_PPR_XCD=1, KRCA_PPR_GRID=grid):
        r, rf, it = eng.ppr(m.row_ptr, m.col, m.outdeg, seed, 0.85, 40, 1e-9)
        assert it == abs(ito) and np.array_equal(rf.cpu().numpy(), ro)
        r, rf, it = eng.ppr(m.row_ptr, m.col, m.outdeg, seed, 0.85, 25, 0.0)
    rfo, ro, _ = oracle.c_ppr(m.row_ptr, m.col, m.outdeg, seed, 0.85, 25, 0.0)
    assert np.array_equal(rf.cpu().numpy(), ro)


@pytest.mark.parametrize("case", ["self_loops", "no_edges", "single", "two_cycle", "star_in", "star_out",
                                  "zero_seed", "one_seed"])
def test_ppr_small_graph_edge_cases(eng, case):
    """Self-loops (the topology agent's deployment merged into its service), a graph without edges,
    one node, a 2-cycle, stars into / out of a hub, all-zero and single-pod personalization: the
    fixed point bit-identical to the C oracle (iteration count included) and within 1e-5 of the
    float64 restatement."""
    from krca.agents.topology import csr_from_edges
    rng = np.random.default_rng(3)
    n = {"single": 1, "two_cycle": 2}.get(case, 50)
    src, dst = [], []
    if case == "self_loops":
        src, dst = list(range(0, 50, 2)) + list(range(50)), list(range(0, 50, 2)) + list((np.arange(50) + 1) % 50)
    elif case == "two_cycle":
        src, dst = [0, 1], [1, 0]
    elif case == "star_in":
        src, dst = list(range(1, n)), [0] * (n - 1)
    elif case == "star_out":
        src, dst = [0] * (n - 1), list(range(1, n))
    elif case in ("zero_seed", "one_seed"):
        src, dst = list(rng.integers(0, n, 200)), list(rng.integers(0, n, 200))
    pairs = sorted(set(zip(src, dst)))  # a DiGraph: each (caller, callee) once
    rp, col, od = csr_from_edges(n, [a for a, _ in pairs], [b for _, b in pairs])
    seed = (rng.random(n) ** 4).astype(np.float32)
    if case == "zero_seed":
        seed[:] = 0
    if case == "one_seed":
        seed[:] = 0
        seed[7] = 1
    if case == "two_cycle":
        # below the weight codes' resolution (26 significant bits: ~2^-26 of the mass per sweep) a
        # tolerance of N * 1e-9 is not reachable on two nodes: the oracle reports no convergence
        # (negative count) and the device call raises, as networkx's PowerIterationFailedConvergence
        _, _, ito = oracle.c_ppr(rp, col, od, seed, 0.85, 200, 1e-9)
        assert ito == -200
        with pytest.raises(native.KrcaError):
            eng.ppr(rp, col, od, seed, 0.85, 200, 1e-9)
    for iters, tol in ((60, 0.0), (200, 1e-6 if case == "two_cycle" else 1e-9)):
        r, rf, it = eng.ppr(rp, col, od, seed, 0.85, iters, tol)
        rfo, ro, ito = oracle.c_ppr(rp, col, od, seed, 0.85, iters, tol)
        assert np.array_equal(rf.cpu().numpy(), ro) and it == abs(ito), (case, iters)
        qs = np.floor(seed.astype(np.float64) * 2.0 ** 32) / 2.0 ** 32
        x, _ = oracle.ppr_f64(rp, col, od, qs, 0.85, it, 0.0)
        rr = r.cpu().numpy().astype(np.float64)
        big = x >= 1e-9
        assert np.max(np.abs(rr[big] - x[big]) / x[big]) < 1e-5, case


def test_ppr_long_rows_and_dangling(eng):
    # a hub with 10k callers (long-row chunks + int64 atomics), isolated and dangling nodes
    n = 12000
    src = np.concatenate([np.arange(1, 10001), np.arange(10001, 11999)])
    dst = np.concatenate([np.zeros(10000, np.int64), np.arange(10002, 12000)])
    from krca.agents.topology import csr_from_edges
    rp, col, od = csr_from_edges(n, src, dst)
    seed = np.ones(n, np.float32)
    r, rf, it = eng.ppr(rp, col, od, seed, 0.85, 50, 0.0)
    rfo, ro, _ = oracle.c_ppr(rp, col, od, seed, 0.85, 50, 0.0)
    assert np.array_equal(rf.cpu().numpy(), ro)


# ---- the full RCA step (krca/rca.py) on one device ------------------------------------------
@pytest.mark.parametrize("n,iters", [(5000, 30), (40000, 12)])
def test_rca_step_single_gpu_vs_oracle(eng, n, iters):
    from krca.rca import Comm, Config, DeviceShard, RcaStep, shard_graph, shard_range
    m = synth.make_graph(n, avg_degree=20, seed=n)
    hops = synth.caller_hops(m, m.roots)
    x = synth.make_metrics(n, 8, 400, window=60, seed=1, roots=m.roots, hop_sets=hops).cuda()
    cfg = Config(iters=iters)
    lo, hi, n_max = shard_range(n, 1, 0)
    rp, col, od = shard_graph(m.row_ptr, m.col, m.outdeg, lo, hi)
    step = RcaStep(DeviceShard(eng, x, rp, col, od, n, n_max, 1, cfg), Comm(), cfg, 0)
    idx, key = step.run()
    score = step.s.score_out["score"].cpu().numpy()
    ridx, rf, r = oracle.rca_rank(m.row_ptr, m.col, m.outdeg, score, cfg.alpha, cfg.iters, cfg.floor(n, 8), cfg.k,
                                  tol=cfg.tol)
    assert np.array_equal(step.s.r[:n].cpu().numpy(), r)
    assert list(idx) == list(ridx)
    idx2, _ = step.run()  # re-run on the same buffers: identical
    assert list(idx2) == list(idx)
    assert len(set(idx.tolist()) & set(m.roots.tolist())) >= 8


@pytest.mark.parametrize("tol", [0.0, 1e-10])
def test_rca_step_graph_replay_equals_eager(eng, tol):
    """RcaStep's HIP-graph solve (captured once per step count, replayed per step) equals the eager
    launch sequence bit for bit, also after the scores change under the captured buffers; under
    the stop rule (tol > 0) the first solve's graph has the cap's 30 steps and the later ones the
    converged count + 1, and the iteration counts match too."""
    from krca.rca import Comm, Config, DeviceShard, RcaStep, shard_graph, shard_range
    n = 20000
    m = synth.make_graph(n, avg_degree=20, seed=5)
    hops = synth.caller_hops(m, m.roots)
    cfg = Config(iters=30, tol=tol)
    lo, hi, n_max = shard_range(n, 1, 0)
    rp, col, od = shard_graph(m.row_ptr, m.col, m.outdeg, lo, hi)
    xs = [synth.make_metrics(n, 8, 300, window=60, seed=s, roots=m.roots, hop_sets=hops).cuda() for s in (1, 2)]
    res = {}
    for graph in (False, True):
        x = xs[0].clone()
        step = RcaStep(DeviceShard(eng, x, rp, col, od, n, n_max, 1, cfg), Comm(), cfg, 0, graph=graph)
        assert step.graph == graph
        out = []
        for xi in xs + xs[:1]:
            x.copy_(xi)  # new metrics under the same buffers (the graph's inputs)
            idx, key = step.run()
            out.append((list(idx), list(key), step.s.r[:n].cpu().numpy().copy(), step.last_iters))
        res[graph] = out
        if graph and tol > 0:
            assert len(step._graphs) >= 2, sorted(step._graphs)  # the cap's, then count + 1
    for (ia, ka, ra, na), (ib, kb, rb, nb) in zip(res[False], res[True]):
        assert ia == ib and ka == kb and np.array_equal(ra, rb) and na == nb
    assert np.array_equal(res[True][0][2], res[True][2][2]) and not np.array_equal(res[True][0][2], res[True][1][2])


@pytest.mark.parametrize("launches", [0, 300, 5000])
def test_rca_graph_replay_after_eager_launches(eng, launches):
    """The captured solve replayed after `launches` unrelated eager kernel launches (tiny torch adds)
    between its first and second replay still equals the eager solve.  Failed at 300 and 5000 with
    the runtime's graph packet capture on (R5n); tests/conftest.py turns it off, as RcaStep requires."""
    from krca.rca import Comm, Config, DeviceShard, RcaStep, shard_graph
    n = 20000
    m = synth.make_graph(n, avg_degree=20, seed=5)
    cfg = Config(iters=30, tol=0.0)
    rp, col, od = shard_graph(m.row_ptr, m.col, m.outdeg, 0, n)
    x0 = synth.make_metrics(n, 8, 300, window=60, seed=1, roots=m.roots, hop_sets=synth.caller_hops(m, m.roots)).cuda()
    refs = []
    xe = x0.clone()
    st_e = RcaStep(DeviceShard(eng, xe, rp, col, od, n, n, 1, cfg), Comm(), cfg, 0)
    for shift in (0.0, 3.0):
        xe[-1, :50] += shift * 10.0
        refs.append(([int(i) for i in st_e.run()[0]], st_e.s.r[:n].cpu().numpy().copy()))
    xg = x0.clone()
    st_g = RcaStep(DeviceShard(eng, xg, rp, col, od, n, n, 1, cfg), Comm(), cfg, 0, graph=True)
    junk = torch.zeros(64, device="cuda")
    got = []
    for shift in (0.0, 3.0):
        xg[-1, :50] += shift * 10.0
        if shift:
            for _ in range(launches):
                junk.add_(1.0)
        got.append(([int(i) for i in st_g.run()[0]], st_g.s.r[:n].cpu().numpy().copy()))
    for (ie, re), (ig, rg) in zip(refs, got):
        assert ie == ig and np.array_equal(re, rg), (launches, int((re != rg).sum()))


@pytest.mark.parametrize("G", [2, 3])
@pytest.mark.parametrize("folded", [False, True])
def test_rca_sharded_path_emulated_on_one_gpu(eng, G, folded):
    """G pod shards on one device with the all-gather done by copies: the remapped-column /
    slot-payload path of the multi-GPU step, unfolded and folded, bit-identical to the
    single-process oracle."""
    from krca.rca import Config, DeviceShard, shard_graph, shard_range
    n = 30000
    m = synth.make_graph(n, avg_degree=20, seed=11)
    hops = synth.caller_hops(m, m.roots)
    x = synth.make_metrics(n, 8, 300, window=60, seed=3, roots=m.roots, hop_sets=hops).cuda()
    cfg = Config(iters=15, tol=0.0)  # the emulation runs exactly cfg.iters folded steps
    shards = []
    for g in range(G):
        lo, hi, n_max = shard_range(n, G, g)
        rp, col, od = shard_graph(m.row_ptr, m.col, m.outdeg, lo, hi)
        shards.append(DeviceShard(eng, x[:, lo:hi, :].contiguous(), rp, col, od, n, n_max, G, cfg))

    def exchange():
        wall = torch.cat([s.send for s in shards])
        for s in shards:
            s.w_all.copy_(wall)

    for s in shards:
        s.score()
        s.init(cfg.alpha, cfg.floor(n, 8))
    exchange()
    if folded:  # krca_ppr_shard_step_folded: each step reduces the previous one's slot set
        for it in range(1, cfg.iters + 1):
            for s in shards:
                s.step_folded(cfg.alpha, cfg.tol, it, 3)
            exchange()
        for s in shards:
            s.finish(cfg.alpha, cfg.tol, cfg.iters)
            assert s.ctl_read() == (cfg.iters, False)
    else:
        for s in shards:
            s.reduce(cfg.alpha, cfg.tol, 1)
        for _ in range(cfg.iters):
            for s in shards:
                s.step(cfg.alpha)
            exchange()
            for s in shards:
                s.reduce(cfg.alpha, cfg.tol, 0)
    score = torch.cat([s.score_out["score"] for s in shards]).cpu().numpy()
    _, _, r = oracle.rca_rank(m.row_ptr, m.col, m.outdeg, score, cfg.alpha, cfg.iters, cfg.floor(n, 8), cfg.k,
                              tol=cfg.tol)
    got = np.concatenate([s.r[:s.n].cpu().numpy() for s in shards])
    assert np.array_equal(got, r)
    # the default key per shard (every pod's scores, the whole graph) = the oracle's, bit for bit
    from krca.rca import Explain
    ex, sall = Explain(m.row_ptr, m.col), torch.from_numpy(score).cuda()
    key_ref, _ = oracle.rca_keys(m.row_ptr, m.col, m.outdeg, score, cfg.alpha, cfg.iters, cfg.floor(n, 8), tol=cfg.tol)
    for g, s in enumerate(shards):
        lo = shard_range(n, G, g)[0]
        s.local_topk_explained(cfg.k, sall, cfg.floor(n, 8), ex, lo)
        assert np.array_equal(s.key[:s.n].cpu().numpy(), key_ref[lo:lo + s.n]), g


def _explain_graph(n, rng, hubs=True):
    """A random pull-CSR with hub rows, duplicate edges, self-loops and empty rows."""
    from krca.agents.topology import csr_from_edges
    E = n * 8
    src = rng.integers(0, n, E)
    dst = np.where(rng.random(E) < (0.3 if hubs else 0.0), rng.integers(0, max(n // 50, 1), E), rng.integers(0, n, E))
    src = np.concatenate([src, src[:n // 10]])  # duplicates
    dst = np.concatenate([dst, dst[:n // 10]])
    loops = rng.integers(0, n, n // 20)
    return csr_from_edges(n, np.concatenate([src, loops]), np.concatenate([dst, loops]))


@pytest.mark.parametrize("n", [1, 7, 3000, 200_000])
def test_rca_explain_kernel_vs_oracle(eng, n):
    """krca_rca_explain (csrc/explain.hip) against the C restatement krco_rca_explain: every pod's
    explaining anomaly d, bit for bit, for the whole range and for sub-ranges (a rank's rows), with
    few / many / no anomalous pods (floor above every score) and ties of A and of 2q."""
    rng = np.random.default_rng(n)
    rp, col, od = _explain_graph(n, rng)
    rpd, cold = torch.from_numpy(rp).cuda(), torch.from_numpy(col).cuda()
    for frac, floor in ((0.02, 4.0), (0.5, 1.0), (0.0, 100.0)):
        score = np.where(rng.random(n) < frac, 4.0 + rng.integers(0, 6, n) * 0.5, rng.random(n) * 3.0).astype(np.float32)
        sd = torch.from_numpy(score).cuda()
        for lo, hi in ((0, n), (n // 3, n - n // 4), (0, 0), (n - 1, n)):
            if hi < lo:
                continue
            got = eng.rca_explain_device(sd, floor, rpd, cold, lo, hi)[:hi - lo].cpu().numpy()
            ref = oracle.c_rca_explain(score, floor, rp, col, lo, hi)
            assert np.array_equal(got, ref), (frac, floor, lo, hi)
        full = oracle.c_rca_explain(score, floor, rp, col)
        if frac == 0.02 and n >= 3000:  # the rule fires on some pods, not on all
            assert 0 < int((full > 0).sum()) < n
    # seeds far past the quantisation's clamp (256 units: q <= 2^40), infinities and NaNs: the
    # 128-bit sums and typicality test keep device and oracle exact (int64 wrapped)
    score = np.where(rng.random(n) < 0.3, rng.choice([1e6, 3e38, np.inf, 300.0, 40.0], n), rng.random(n) * 3.0)
    score = np.where(rng.random(n) < 0.01, np.nan, score).astype(np.float32)
    got = eng.rca_explain_device(torch.from_numpy(score).cuda(), 4.0, rpd, cold, 0, n)[:n].cpu().numpy()
    assert np.array_equal(got, oracle.c_rca_explain(score, 4.0, rp, col))


def test_rca_key_explained_single_device_vs_oracle(eng):
    """The whole default ranking on one device (DeviceShard + RcaStep; and krca_ppr +
    rank_root_causes): every key bit-identical to oracle.rca_keys, fixed iterations and L1 tolerance."""
    from krca.rca import Comm, Config, DeviceShard, RcaStep, shard_graph
    n = 20000
    m = synth.make_graph(n, avg_degree=20, seed=31)
    x = synth.make_metrics(n, 8, 200, window=60, seed=31, roots=m.roots,
                           hop_sets=synth.spread_hops(m, m.roots, seed=31), **synth.SPREAD_SIGMAS).cuda()
    for cfg in (Config(), Config(tol=0.0), Config(tol=1e-9, iters=100, alpha=0.85)):
        sh = DeviceShard(eng, x, *shard_graph(m.row_ptr, m.col, m.outdeg, 0, n), n, n, 1, cfg)
        step = RcaStep(sh, Comm(), cfg, 0)
        idx, _ = step.run()
        score = sh.score_out["score"].cpu().numpy()
        key, o = oracle.rca_keys(m.row_ptr, m.col, m.outdeg, score, cfg.alpha, cfg.iters, cfg.floor(n, 8), tol=cfg.tol)
        assert np.array_equal(sh.r[:n].cpu().numpy(), o["r"])
        assert np.array_equal(sh.key[:n].cpu().numpy(), key)
        ridx = oracle.topk_ref(key, cfg.k)[0]
        assert [int(i) for i in idx] == ridx.tolist()
        got = eng.rank_root_causes(score, m.row_ptr, m.col, m.outdeg, cfg, n_metrics=8)[0]
        assert got.tolist() == ridx.tolist()


@pytest.mark.parametrize("n,G", [(9, 4), (49, 8), (30000, 3)])
def test_rca_folded_tolerance_with_empty_rank_emulated(eng, n, G):
    """Folded steps under a tolerance (the stream's re-rank loop), G shards on one device with the
    all-gather done by copies, including ranks that own no pods (shard_range(9, 4) and (49, 8)
    leave the last rank empty): every rank's control block reports the same iteration count and
    convergence after every step -- a rank without rows runs the step's reduction alone
    (krca_ppr_shard_step_folded, empty plan) -- and the ranks are bit-identical to the C oracle.
    Before that, an empty rank never advanced its count, so its convergence poll never stopped and
    its all-gathers outlived the other ranks'."""
    from krca.agents.topology import csr_from_edges
    from krca.rca import Config, DeviceShard, shard_graph, shard_range
    rng = np.random.default_rng(n)
    E = min(n * 12, n * (n - 1))
    src, dst = rng.integers(0, n, E), rng.integers(0, n, E)
    keep = src != dst
    rp_all, col_all, od_all = csr_from_edges(n, src[keep], dst[keep])
    seed = (rng.random(n) * 2.0).astype(np.float32)
    cfg = Config(alpha=0.85, seed_floor=1.0)
    tol, max_iter = 1e-9, 200
    shards = []
    for g in range(G):
        lo, hi, n_max = shard_range(n, G, g)
        rp, col, od = shard_graph(rp_all, col_all, od_all, lo, hi)
        s = DeviceShard(eng, None, rp, col, od, n, n_max, G, cfg)
        s.score_out = {"score": torch.from_numpy(np.concatenate([seed[lo:hi], np.zeros(1, np.float32)])).cuda()}
        shards.append(s)
    assert any(s.n == 0 for s in shards) or n == 30000

    def exchange():
        wall = torch.cat([s.send for s in shards])
        for s in shards:
            s.w_all.copy_(wall)

    for s in shards:
        s.init(cfg.alpha, cfg.floor(n))
    exchange()
    it = 0
    while it < max_iter:
        it += 1
        for s in shards:
            s.step_folded(cfg.alpha, tol, it, 3)
        exchange()
        states = {s.ctl_read() for s in shards}
        assert len(states) == 1, (it, states)  # every rank (empty ones too) at the same count / flag
        if states.pop()[1]:
            break
    for s in shards:
        s.finish(cfg.alpha, tol, it)
    _, r_ref, it_ref = oracle.c_ppr(rp_all, col_all, od_all, seed, cfg.alpha, max_iter, tol, cfg.floor(n))
    assert it_ref > 0 and {s.ctl_read() for s in shards} == {(it_ref, True)}
    got = np.concatenate([s.r[:s.n].cpu().numpy() for s in shards])
    assert np.array_equal(got, r_ref)


def test_stream_cold_solve_fresh_streams_bit_identical(eng):
    """Regression for a cold-solve mismatch seen once during round 3's folded-iteration work
    (call r3ac: a fresh stream's first solve came out with the uniform teleport on part of the
    pods, i.e. some workgroups had read a zero seed total).  Several fresh StreamingRCA objects,
    each pushed a history and solved cold under the L1 stop rule, one after another on the same
    device (stale device memory between them): ranks and iteration counts bit-identical to
    oracle.c_ppr every time, and the second solve (warm) to oracle.c_ppr_warm."""
    from krca.rca import Config
    from krca.stream import StreamingRCA
    P, M, T = 200_000, 4, 200
    mesh = synth.make_graph(P, avg_degree=12, seed=21)
    hops = synth.caller_hops(mesh, mesh.roots)
    x = synth.make_metrics_range(0, P, M, T + 1, seed=21, roots=mesh.roots, hop_sets=hops, device="cuda")
    cfg = Config(window=30)
    fl = cfg.floor(P, M)
    ref = None
    for trial in range(3):
        s = StreamingRCA(eng, mesh.row_ptr, mesh.col, mesh.outdeg, M, cfg, horizon=T, tol=1e-9, max_iter=100)
        s.push_metrics(x[:T])
        s.rerank()
        sc0 = s.shard.score_out["score"].cpu().numpy()
        r0 = s.shard.r[:P].cpu().numpy()
        if ref is None:
            _, r_ref, it_ref = oracle.c_ppr(mesh.row_ptr, mesh.col, mesh.outdeg, sc0, cfg.alpha, 100, 1e-9, fl)
            ref = (sc0, r_ref, it_ref)
        assert np.array_equal(sc0, ref[0]), trial
        assert np.array_equal(r0, ref[1]) and s.last_iters == ref[2], trial
        s.push_metrics(x[T:T + 1])
        s.rerank()
        r_w, it_w, _ = oracle.c_ppr_warm(mesh.row_ptr, mesh.col, mesh.outdeg, s.shard.score_out["score"].cpu().numpy(),
                                         ref[1], cfg.alpha, 100, 1e-9, fl)
        assert np.array_equal(s.shard.r[:P].cpu().numpy(), r_w) and s.last_iters == it_w, trial
        del s
    torch.cuda.synchronize()


# ---- a13 error templates -------------------------------------------------------------------
def test_template_hist_vs_oracle(eng):
    import json
    import os
    from conftest import GOLDEN
    g = json.load(open(os.path.join(GOLDEN, "logs_corpus.json")))
    docs = [c["text"] for c in g["containers"]]  # up to 300 lines: wave and workgroup paths
    docs += synth.make_log_corpus(5000, lines_per_doc=4, seed=11, hazard_rate=0.02)
    docs += ["", "\n", "id=deadbeefcafe x", "user_42 7f9c4 0xFF", "a" * 5000 + " 123", "été 42 café"]
    docs.append("\n".join("req %d from 10.0.%d.%d took %dms" % (i, i % 7, i % 250, i) for i in range(3000)))
    # workgroups whose 256 lines span more than the LDS-staged 24 KiB (the rest go through global
    # dwords), a 30 KB line, masked / unmasked hex lengths, words across dword boundaries, no final \n
    docs.append("\n".join("y" * (150 + i % 7) + " w%d deadbeef deadbee _9 a_b ABCDEF12 abcdefg" % i for i in range(700)))
    docs.append("z" * 15000 + " 42 " + "q" * 15000 + " cafebabe1 end")
    docs += ["deadbeef", "deadbee", "x_", "_", "9", "a9b c", "ab\u00e9cd 12\u00e912"]
    # UUIDs (one mask byte), also with groups holding no digit, at line ends, back to back, in
    # failed candidates that restart on an 8-hex word, and near misses (13-hex last group, "--")
    docs += ["deadbeef-cafe-babe-face-0123456789ab", "id=DEADBEEF-CAFE-BABE-FACE-ABCDEFabcdef\nnext",
             "x-deadbeef-deadbeef-cafe-babe-face-0123456789ab-z", "deadbeef-cafe-babe-face-0123456789abc",
             "aaaaaaaa-bbbb-cccc-dddd-eeeeeeeeeeee aaaaaaaa-bbbb-cccc-dddd-eeeeeeeeeeee",
             "deadbeef-cafe-deadbeef-cafe-babe-face-abcdefabcdef", "deadbeef--cafe-babe-face-0123456789ab",
             "\n".join("req %s-%s-%s-%s-%s done" % ("abcdef12"[i % 8:] + "ab" * (i % 8 // 2) + "c" * (i % 2),
                                                    "cafe", "b%03x" % i if i % 3 else "babe", "face",
                                                    "abcdefabcdef") for i in range(400))]
    for tail in range(1, 20):  # the text's last bytes in every position of a 16-byte piece
        got = eng.template_hist(*pack_documents(["w" * tail + " 1 tail" + "z" * (tail % 5), "end" * tail]))
        assert got == [oracle.template_hist("w" * tail + " 1 tail" + "z" * (tail % 5)),
                       oracle.template_hist("end" * tail)], tail
    got = eng.template_hist(*pack_documents(docs))
    for d, text in enumerate(docs):
        assert got[d] == oracle.template_hist(text), d


def test_template_hist_fragment_fuzz(eng):
    """Words, digit runs and hex runs cut at random points and scattered over lines and containers
    (no trailing separator, so a word's halves meet at container ends; 8-hex-digit runs split and
    joined; underscores, UTF-8 and the multi-byte separators beside them): every container's
    template histogram equals the oracle's."""
    rng = np.random.default_rng(29)
    frags = ["dead", "beef", "cafe", "12", "x", "_", " ", "DEADBEEF", "0", "ab12", "deadbee", "f", "9z",
             "é", "\u2028", "\x85", "\n", "\r\n", "\r", "-", "/", "GET", "worker", "id=", "0x",
             "deadbeef-", "cafe-", "face-", "abcdefabcdef", "0123456789ab", "-cafe-babe-face-"]
    docs = []
    for _ in range(3000):
        docs.append("".join(frags[int(i)] for i in rng.integers(0, len(frags), int(rng.integers(0, 14)))))
    got = eng.template_hist(*pack_documents(docs))
    for d, text in enumerate(docs):
        assert got[d] == oracle.template_hist(text), (d, repr(text))


def test_template_hist_huge_containers(eng):
    """Containers above krca_template_max_lines() lines: distinct-hash table + bucketed sorts,
    exact vs the oracle (few templates repeated many times; all-distinct templates; a mix)."""
    rng = np.random.default_rng(3)
    letters = np.array(list("abcdefghijklmnopqrstuvwxyz"))
    word = lambda n: "".join(rng.choice(letters, n))  # noqa: E731  (no digits: never masked)
    docs = ["\n".join("GET /health %d ok" % i if i % 3 else "worker %s busy" % ("ab"[i % 2]) for i in range(6000))]
    docs.append("\n".join("job %s done" % word(9) for _ in range(9000)))   # ~9000 distinct templates
    docs.append("short 1\nshort 2")
    docs.append("\n".join(("evt %s" % word(3)) if i % 2 else "tick %d" % i for i in range(40000)))
    docs.append("\n".join("x" for _ in range(4097)))                         # one template, 4097 lines
    assert max(len(d.splitlines()) for d in docs) > eng.lib.krca_template_max_lines()
    got = eng.template_hist(*pack_documents(docs))
    for d, text in enumerate(docs):
        assert got[d] == oracle.template_hist(text), d


def test_template_hist_writes_every_slot(eng):
    """krca_template_hist (+ _huge) write every slot of each container's line range: its templates,
    then 0 (include/krca.h) -- checked on outputs pre-filled with a poison pattern, for containers
    on the lane (<= 8 lines), wave (<= 64), workgroup (<= 4096) and huge paths, repeated templates."""
    docs = ["a 1\na 2\nb", "x\n" * 5 + "y", "\n".join("t %d" % (i % 3) for i in range(50)),
            "\n".join("u %s" % ("k" * (i % 7)) for i in range(3000)), "\n".join("v" for _ in range(5000)), "", "z"]
    blob, off = pack_documents(docs)
    scan = eng.log_scan_device(eng.upload_blob(blob), torch.from_numpy(off).cuda())
    ref = eng.template_hist_device(scan)  # (zero-initialised n_templates; huge containers completed)
    L = scan["n_lines_total"]
    oh = torch.full((L,), -0x5A5A5A5A5A5A5A5B, dtype=torch.int64, device="cuda")
    oc = torch.full((L,), -0x5A5A5A5B, dtype=torch.int32, device="cuda")
    nt = torch.zeros(len(docs), dtype=torch.int32, device="cuda")
    out = dict(ref)
    out.update(tmpl_hash=oh, tmpl_count=oc, n_templates=nt)
    ws = eng._workspace("tmpl_hist_t", eng.lib.krca_template_hist_ws_size(len(docs))).view(torch.int32)
    assert eng.lib.krca_template_hist(eng.ptr(ref["hash"]), eng.ptr(scan["doc_lines"]), eng.ptr(scan["doc_line0"]),
                                      len(docs), eng.ptr(ws), eng.ptr(oh), eng.ptr(oc), eng.ptr(nt), eng._stream()) == 0
    eng._template_huge(ws, ref["hash"], oh, oc, nt, scan)
    torch.cuda.synchronize()
    assert int(ws[2].item()) == 1  # one container on the huge path
    assert torch.equal(oh, ref["tmpl_hash"]) and torch.equal(oc, ref["tmpl_count"]) and torch.equal(nt, ref["n_templates"])
    d0, dl, n = scan["doc_line0"].cpu().numpy(), scan["doc_lines"].cpu().numpy(), nt.cpu().numpy()
    ohn, ocn = oh.cpu().numpy(), oc.cpu().numpy()
    for d in range(len(docs)):
        assert (ohn[d0[d] + n[d]:d0[d] + dl[d]] == 0).all() and (ocn[d0[d] + n[d]:d0[d] + dl[d]] == 0).all(), d
        assert (ocn[d0[d]:d0[d] + n[d]] > 0).all(), d


def test_template_hash_any_line_order(eng):
    """krca_template_hash on the scan's lines in a shuffled order, with some lines repeated and a few
    empty or reversed ranges: every hash equals the in-order hash of the same range (a workgroup's
    window starts at its first line; lines outside it are read directly)."""
    docs = synth.make_log_corpus(3000, lines_per_doc=3, seed=5, hazard_rate=0.05)
    docs.append("z" * 40000 + " 12 " + "q" * 30000)  # a line longer than any staged span
    blob, off = pack_documents(docs)
    scan = eng.log_scan_device(eng.upload_blob(blob), torch.from_numpy(off).cuda())
    L = scan["n_lines_total"]
    ls, le = scan["line_start"][:L].clone(), scan["line_end"][:L].clone()
    text = scan["text"]

    def run(s_, e_):
        out = torch.empty(s_.numel(), dtype=torch.int64, device="cuda")
        assert eng.lib.krca_template_hash(eng.ptr(text), text.numel(), eng.ptr(s_), eng.ptr(e_), s_.numel(),
                                          eng.ptr(out), eng._stream()) == 0
        return out

    ref = run(ls, le).cpu().numpy()
    rng = np.random.default_rng(3)
    perm = rng.permutation(L)
    perm = np.concatenate([perm, perm[:500]])  # repeated lines
    s2, e2 = ls[torch.from_numpy(perm).cuda()].contiguous(), le[torch.from_numpy(perm).cuda()].contiguous()
    got = run(s2, e2).cpu().numpy()
    assert np.array_equal(got, ref[perm])
    # empty and reversed ranges hash as the empty template
    e3 = e2.clone()
    e3[::7] = s2[::7] - 5
    got = run(s2, e3).cpu().numpy()
    empty = np.array([0xcbf29ce484222325], dtype=np.uint64).view(np.int64)[0]  # FNV-1a offset basis
    assert (got[::7] == empty).all() and np.array_equal(got[1::7], ref[perm][1::7])


def test_template_hash_examples(eng):
    assert oracle.template_of(b"GET /api/v1/items 200 15ms") == b"GET /api/\xff/items \xff \xff"
    assert oracle.template_of(b"uuid 550e8400-e29b-41d4-a716-446655440000 deadbeef") == b"uuid \xff \xff"
    assert oracle.template_of(b"deadbeef-cafe-babe-face-0123456789ab") == b"\xff"  # groups without a digit
    assert oracle.template_of(b"deadbeef-cafe-babe-face-0123456789abc") == b"\xff-cafe-babe-face-\xff"
    assert oracle.template_of(b"user_42 caf\xc3\xa9 OK") == b"\xff caf\xc3\xa9 OK"
