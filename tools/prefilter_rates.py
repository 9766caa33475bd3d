#!/usr/bin/env python3
"""Pass rates of literal prefilters on the synthetic C5 log corpus.

A line passes a k-gram prefilter when it holds any case-folded k-gram of any category literal
(krca/patterns.py).  Prints the fraction of lines that truly match, and the pass rates of the
bigram and trigram filters: a filter is only worth a pass over the text when it rejects most
lines.   python tools/prefilter_rates.py [--docs 20000]
"""
import argparse
import os
import re
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "kubernetes-rca-system_amd"))
from krca import synth  # noqa: E402
from krca.patterns import ERROR_PATTERNS  # noqa: E402


def grams(n):
    out = set()
    for _, p in ERROR_PATTERNS:
        for alt in p[1:-1].split("|"):
            a = alt.lower()
            out.update(a[i:i + n] for i in range(len(a) - n + 1))
    return out


def passes(line, g, n):
    s = line.lower()
    return any(s[i:i + n] in g for i in range(len(s) - n + 1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=20000)
    a = ap.parse_args()
    lines = [ln for d in synth.make_log_corpus(a.docs, seed=1) for ln in d.splitlines()]
    rx = [re.compile(p, re.IGNORECASE) for _, p in ERROR_PATTERNS]
    match = np.mean([any(r.search(ln) for r in rx) for ln in lines])
    g2, g3 = grams(2), grams(3)
    p2 = np.mean([passes(ln, g2, 2) for ln in lines])
    p3 = np.mean([passes(ln, g3, 3) for ln in lines])
    print(f"lines={len(lines)} match={match:.3f} bigram_pass={p2:.3f} ({len(g2)} bigrams) "
          f"trigram_pass={p3:.3f} ({len(g3)} trigrams)")


if __name__ == "__main__":
    main()
