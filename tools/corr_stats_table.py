"""Per-kernel average / total of the correlation kernels from a rocprofv3 --stats directory."""
import csv
import glob
import sys

d = sys.argv[1]
f = glob.glob(f"{d}/**/*kernel_stats.csv", recursive=True)[0]
rows = []
for r in csv.DictReader(open(f)):
    n = r["Name"]
    if "corr" not in n:
        continue
    m = n.replace("void ", "").replace("(anonymous namespace)::", "")
    short = m.split(">")[0] + ">" if m.startswith(("corr_tiles", "corr_theta")) else m.split("(")[0]
    rows.append((short, int(r["Calls"]), float(r["AverageNs"]) / 1e6, float(r["TotalDurationNs"]) / 1e6))
for short, c, avg, tot in sorted(rows, key=lambda t: -t[3]):
    print(f"{short:40s} calls {c:4d}  avg {avg:8.3f} ms  total {tot:8.3f} ms")
