#!/usr/bin/env python3
"""Compile the 13 log-category regexes into the device DFA tables (csrc/log_dfa_tables.h).

Semantics reproduced exactly (ref:agents/logs_agent.py:140-151): a line of
``logs.splitlines()`` is in category c iff ``re.search(pattern_c, line, re.IGNORECASE)``.
The patterns only use literal characters, ``.`` (any code point but ``\\n``), ``\\d``
(Unicode decimal digit) and top-level alternation, so each category is a finite set of
fixed-length strings over code-point classes and ``Σ*·(p_1|…|p_k)`` has a small DFA.

Code points are mapped to SYMBOLS: two code points share a symbol iff every pattern atom
treats them alike under Python 3.10's ``re.IGNORECASE`` (e.g. U+212A KELVIN SIGN shares the
symbol of ``k``; Arabic-Indic digits share the symbol of an ASCII digit that no literal
uses).  The classes are derived by asking CPython's own ``re`` module, so the tables are
exact for the interpreter that generated them (the image's Python 3.10 / Unicode 13.0).

Line separators (``str.splitlines``: \\n \\r \\r\\n \\v \\f \\x1c \\x1d \\x1e U+0085 U+2028
U+2029) get the reserved symbol SEP and never enter the DFA.

Run:  python gen_log_dfa.py [out.h]     (re-run only if krca/patterns.py changes)
"""
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
from krca.patterns import ERROR_PATTERNS, pattern_digest  # noqa: E402

MAXCP = 0x110000


def _valid(c):
    return not (0xD800 <= c <= 0xDFFF)


def parse(pattern):
    """'(a|b|c)' -> list of alternatives, each a list of atom regex strings."""
    assert pattern[0] == "(" and pattern[-1] == ")", pattern
    body = pattern[1:-1]
    alts, cur, i = [], [], 0
    while i < len(body):
        ch = body[i]
        if ch == "|":
            alts.append(cur)
            cur = []
        elif ch == "\\":
            cur.append(body[i:i + 2])
            i += 1
        elif ch == ".":
            cur.append(".")
        else:
            assert ch not in "()[]*+?{}^$", (pattern, ch)
            cur.append(re.escape(ch))
        i += 1
    alts.append(cur)
    return alts


def separators():
    return [c for c in range(MAXCP) if _valid(c) and len(("a" + chr(c) + "b").splitlines()) == 2]


def build():
    pats = [parse(p) for _, p in ERROR_PATTERNS]
    atoms = sorted({a for alts in pats for alt in alts for a in alt})
    comp = {a: re.compile(a, re.IGNORECASE) for a in atoms}

    def sig(c):
        ch = chr(c)
        return tuple(bool(comp[a].fullmatch(ch)) for a in atoms)

    seps = set(separators())
    # ---- symbols: distinct signatures of ASCII code points, plus OTHER ------------------
    SEP = 0xFF
    sig_to_sym = {}
    ascii_sym = []
    for c in range(128):
        if c in seps:
            ascii_sym.append(SEP)
            continue
        s = sig(c)
        if s not in sig_to_sym:
            sig_to_sym[s] = len(sig_to_sym)
        ascii_sym.append(sig_to_sym[s])
    other_sig = tuple(a == "." for a in atoms)  # matches only '.'
    if other_sig not in sig_to_sym:
        sig_to_sym[other_sig] = len(sig_to_sym)
    OTHER = sig_to_sym[other_sig]

    # ---- non-ASCII: everything is OTHER except case folds, \d digits and separators ---
    special = {}
    anyletter = re.compile("[a-z]", re.IGNORECASE)
    digit = re.compile(r"\d")
    for c in range(128, MAXCP):
        if not _valid(c):
            continue
        ch = chr(c)
        if c in seps:
            special[c] = SEP
        elif anyletter.fullmatch(ch) or digit.fullmatch(ch):
            s = sig(c)
            if s not in sig_to_sym:
                sig_to_sym[s] = len(sig_to_sym)
            special[c] = sig_to_sym[s]
        elif sig(c) != other_sig:  # defensive: nothing else may differ from OTHER
            raise AssertionError(hex(c))
    ranges = []
    for c in sorted(special):
        if ranges and ranges[-1][1] == c - 1 and ranges[-1][2] == special[c]:
            ranges[-1][1] = c
        else:
            ranges.append([c, c, special[c]])
    nsym = len(sig_to_sym)
    sym_sig = [None] * nsym
    for s, i in sig_to_sym.items():
        sym_sig[i] = s
    atom_idx = {a: i for i, a in enumerate(atoms)}

    # ---- subset construction over NFA positions (pattern, alt, offset) ----------------
    def step(state, sym):
        nxt = set()
        cand = set(state) | {(p, a, 0) for p, alts in enumerate(pats) for a in range(len(alts))}
        for (p, a, i) in cand:
            alt = pats[p][a]
            if i < len(alt) and sym_sig[sym][atom_idx[alt[i]]]:
                nxt.add((p, a, i + 1))
        return frozenset(nxt)

    def out(state):
        m = 0
        for (p, a, i) in state:
            if i == len(pats[p][a]):
                m |= 1 << p
        return m

    start = frozenset()
    states = {start: 0}
    order = [start]
    trans = []
    k = 0
    while k < len(order):
        st = order[k]
        row = []
        for sym in range(nsym):
            nx = step(st, sym)
            if nx not in states:
                states[nx] = len(order)
                order.append(nx)
            row.append(states[nx])
        trans.append(row)
        k += 1
    outs = [out(s) for s in order]
    trans, outs = minimize(trans, outs)
    return dict(nsym=nsym, nstate=len(trans), ascii_sym=ascii_sym, ranges=ranges, trans=trans,
                out=outs, SEP=SEP, OTHER=OTHER, ncat=len(pats))


def minimize(trans, outs):
    """Moore partition refinement (states equivalent iff same output mask now and after every
    symbol string), then breadth-first renumbering from the start state (0 stays 0).  The
    subset construction's 502 states fold to 394: a smaller LDS table for the device walk."""
    n, nsym = len(trans), len(trans[0])
    part = list(outs)
    while True:
        keys = {}
        new = [keys.setdefault((part[s],) + tuple(part[trans[s][a]] for a in range(nsym)), len(keys))
               for s in range(n)]
        if len(keys) == len(set(part)):
            break
        part = new
    rep = {}
    for s in range(n):
        rep.setdefault(part[s], s)
    ids, order, k = {part[0]: 0}, [part[0]], 0
    while k < len(order):
        r = rep[order[k]]
        for a in range(nsym):
            c = part[trans[r][a]]
            if c not in ids:
                ids[c] = len(order)
                order.append(c)
        k += 1
    return ([[ids[part[trans[rep[c]][a]]] for a in range(nsym)] for c in order], [outs[rep[c]] for c in order])


def simulate(tables, line):
    """Python model of the device matcher on one line (no separators inside)."""
    st, m = 0, 0
    for ch in line:
        c = ord(ch)
        if c < 128:
            sym = tables["ascii_sym"][c]
        else:
            sym = tables["OTHER"]
            for lo, hi, s in tables["ranges"]:
                if lo <= c <= hi:
                    sym = s
                    break
        assert sym != tables["SEP"]
        st = tables["trans"][st][sym]
        m |= tables["out"][st]
    return m


def emit(t, path):
    import unicodedata
    L = []
    L.append("// GENERATED by csrc/gen_log_dfa.py from krca/patterns.py -- do not edit.")
    L.append("// 13-category log matcher DFA (ref:agents/logs_agent.py:20-34, re.IGNORECASE, Python 3.10).")
    L.append("#pragma once")
    L.append("#include <stdint.h>")
    L.append("#ifndef KRCA_DFA_QUAL")
    L.append("#define KRCA_DFA_QUAL static const")
    L.append("#endif")
    L.append(f"#define KRCA_DFA_NSYM {t['nsym']}")
    L.append(f"#define KRCA_DFA_NSTATE {t['nstate']}")
    L.append(f"#define KRCA_DFA_SEP {t['SEP']}")
    L.append(f"#define KRCA_DFA_OTHER {t['OTHER']}")
    L.append(f"#define KRCA_DFA_NRANGE {len(t['ranges'])}")
    L.append(f"#define KRCA_NCAT {t['ncat']}")
    L.append("// Unicode tables of the generating interpreter (IGNORECASE folds, \\d, line separators)")
    L.append(f'#define KRCA_DFA_UNIDATA "{unicodedata.unidata_version}"')
    L.append(f"#define KRCA_DFA_DIGEST 0x{pattern_digest(ERROR_PATTERNS):016X}ull  // gen_log_dfa.pattern_digest")
    L.append("KRCA_DFA_QUAL uint8_t krca_dfa_ascii_sym[128] = {" + ",".join(map(str, t["ascii_sym"])) + "};")
    L.append("// non-ASCII code point ranges [lo, hi] -> symbol (sorted); all others -> OTHER")
    L.append("KRCA_DFA_QUAL uint32_t krca_dfa_ranges[KRCA_DFA_NRANGE][3] = {")
    for lo, hi, s in t["ranges"]:
        L.append(f"  {{0x{lo:X}u, 0x{hi:X}u, {s}u}},")
    L.append("};")
    L.append("// transition table [state][symbol] and per-state category output mask")
    L.append("KRCA_DFA_QUAL uint16_t krca_dfa_trans[KRCA_DFA_NSTATE * KRCA_DFA_NSYM] = {")
    for row in t["trans"]:
        L.append("  " + ",".join(map(str, row)) + ",")
    L.append("};")
    L.append("KRCA_DFA_QUAL uint16_t krca_dfa_out[KRCA_DFA_NSTATE] = {" + ",".join(map(str, t["out"])) + "};")
    with open(path, "w") as f:
        f.write("\n".join(L) + "\n")


if __name__ == "__main__":
    t = build()
    out_path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(HERE, "log_dfa_tables.h")
    emit(t, out_path)
    print(f"symbols={t['nsym']} states={t['nstate']} ranges={len(t['ranges'])} -> {out_path}")
