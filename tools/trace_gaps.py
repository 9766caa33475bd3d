"""Kernel timeline of a rocprofv3 kernel trace (csv): the last N kernels with their start offset,
duration and the idle gap before each, plus totals -- where a latency-bound sequence (a C5 window,
a PageRank solve) spends its wall time between kernels."""
import csv
import sys


def main(path, last=400):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    rows = rows[-last:]
    t0 = rows[0][0]
    busy = gaps = 0
    prev_end = None
    for s, e, n in rows:
        gap = 0 if prev_end is None else max(0, s - prev_end)
        busy += e - s
        gaps += gap
        short = n.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:48]
        print(f"{(s - t0) / 1e3:10.1f} us  dur {(e - s) / 1e3:8.1f}  gap {gap / 1e3:7.1f}  {short}")
        prev_end = e if prev_end is None else max(prev_end, e)
    print(f"kernels {len(rows)}: busy {busy / 1e3:.1f} us, gaps {gaps / 1e3:.1f} us, span {(rows[-1][1] - t0) / 1e3:.1f} us")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 400)
