"""Per-kernel HBM traffic table from tools/gpu_pmc_all.sh: for each (kernel,
grid size) group, mean duration from the kernel trace, FETCH_SIZE x 2 (gfx950
correction, MI355X_MICROARCH.md) + WRITE_SIZE per launch, and the implied
traffic bandwidth.  Usage: pmc_all_summary.py <dir>"""
import collections
import csv
import glob
import re
import statistics
import sys

d = sys.argv[1]


def rows(pattern):
    f = glob.glob(f"{d}/{pattern}", recursive=True)
    if not f:
        sys.exit(f"missing {pattern} under {d}")
    return list(csv.DictReader(open(f[0])))


def short(name):
    m = re.search(r"k_\w+(<[^>]*>)?", name)
    return m.group(0) if m else name[:40]


def grid(r):
    for k in ("Grid_Size", "Grid_Size_X"):
        if k in r:
            return int(r[k])
    return 0


def counter(pattern, cname):
    acc = collections.defaultdict(list)
    for r in rows(pattern):
        if r["Counter_Name"] == cname:
            acc[(short(r["Kernel_Name"]), grid(r))].append(float(r["Counter_Value"]))
    return {k: statistics.fmean(v) for k, v in acc.items()}


fetch = counter("pmc_fetch/**/*counter_collection.csv", "FETCH_SIZE")
write = counter("pmc_write/**/*counter_collection.csv", "WRITE_SIZE")
durs = collections.defaultdict(list)
for r in rows("trace/**/*kernel_trace.csv"):
    durs[(short(r["Kernel_Name"]), grid(r))].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)

tot = {k: statistics.fmean(v) * len(v) for k, v in durs.items()}
print(f"{'kernel':28s} {'grid':>10s} {'n':>5s} {'avg us':>9s} {'tot ms':>8s} {'MB/launch':>10s} {'TB/s':>6s}")
for k in sorted(tot, key=lambda k: -tot[k])[:40]:
    mb = (2 * fetch.get(k, 0.0) + write.get(k, 0.0)) * 1024 / 1e6
    avg = statistics.fmean(durs[k])
    print(f"{k[0]:28s} {k[1]:10d} {len(durs[k]):5d} {avg:9.2f} {tot[k] / 1e3:8.2f} {mb:10.2f} {mb / avg:6.2f}")
