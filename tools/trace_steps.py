"""Per-step launch statistics from a rocprofv3 kernel trace of bench.py.

Steps are delimited by k_evolution_partial (check_evolution runs once at the
end of every step); the last K complete steps are summarised: launches per
step, kernel busy time, wall span, idle time between consecutive kernels, and
the launch count per kernel.  Usage: trace_steps.py TRACE_DIR [K]"""
import collections
import csv
import glob
import re
import statistics
import sys

d = sys.argv[1]
K = int(sys.argv[2]) if len(sys.argv) > 2 else 3
f = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))


def short(n):
    m = re.search(r"k_\w+(<[^>]*>)?", n)
    return m.group(0) if m else n[:40]


ends = [i for i, r in enumerate(rows) if "k_evolution_partial" in r["Kernel_Name"]]
if len(ends) < K + 1:
    sys.exit(f"{f}: only {len(ends)} step markers")
print(f"{f}: last {K} steps (delimited by k_evolution_partial)")
per = []
for s in range(len(ends) - K, len(ends)):
    seg = rows[ends[s - 1] + 1: ends[s] + 1]
    t0 = int(seg[0]["Start_Timestamp"])
    t1 = int(seg[-1]["End_Timestamp"])
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg)
    gaps = [max(0, int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) for a, b in zip(seg, seg[1:])]
    per.append((len(seg), busy / 1e6, (t1 - t0) / 1e6, sum(gaps) / 1e6, statistics.median(gaps) / 1e3,
                sum(g for g in gaps if g < 100_000) / 1e6, collections.Counter(short(r["Kernel_Name"]) for r in seg)))
for n, busy, wall, gap, med, small, _ in per:
    print(f"  launches {n:6d}  kernel busy {busy:8.2f} ms  span {wall:8.2f} ms  idle {gap:6.2f} ms "
          f"(gaps < 100 us: {small:6.2f} ms, median gap {med:5.2f} us)")
n = statistics.fmean(p[0] for p in per)
busy = statistics.fmean(p[1] for p in per)
wall = statistics.fmean(p[2] for p in per)
print(f"mean: {n:.0f} launches/step, {busy:.2f} ms kernel time in a {wall:.2f} ms span "
      f"({100 * (wall - busy) / wall:.1f} % idle), {1e3 * (wall - busy) / n:.2f} us idle per launch")
print("launches per step by kernel:")
for k, c in per[-1][6].most_common(25):
    print(f"  {c:6d}  {k}")
