"""Counters of the level-1 AMG residual (k_amg_residual on the 5 M-row C2
level: the second-largest residual grid) with the nontemporal bit 64 off
(CFD_NT=47) and on (111), from tools/gpu_profiles_r06.sh: trace duration,
FETCH_SIZE x 2 + WRITE_SIZE per launch (gfx950 correction, MI355X_MICROARCH.md)
and the SQ wait fractions.  Usage: level1_residual_counters.py <dir>"""
import collections
import csv
import glob
import statistics
import sys

d = sys.argv[1]


def grid(r):
    for k in ("Grid_Size", "Grid_Size_X"):
        if k in r:
            return int(r[k])
    return 0


def csvrows(pattern):
    f = glob.glob(pattern, recursive=True)
    if not f:
        sys.exit(f"missing {pattern}")
    return list(csv.DictReader(open(f[0])))


print(f"{'mask':>5s} {'grid':>9s} {'n':>4s} {'avg us':>8s} {'MB/launch':>10s} {'TB/s':>6s} {'wait':>5s} {'wait_inst':>9s}")
for m in (47, 111):
    base = f"{d}/nt{m}"
    durs = collections.defaultdict(list)
    for r in csvrows(f"{base}/trace/**/*kernel_trace.csv"):
        if "k_amg_residual" in r["Kernel_Name"]:
            durs[grid(r)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    grids = sorted(durs, reverse=True)
    g1 = grids[1] if len(grids) > 1 else grids[0]  # level 1
    ctr = collections.defaultdict(list)
    for sub in ("pmc_fetch", "pmc_write", "pmc_sq"):
        for r in csvrows(f"{base}/{sub}/**/*counter_collection.csv"):
            if "k_amg_residual" in r["Kernel_Name"] and grid(r) == g1:
                ctr[r["Counter_Name"]].append(float(r["Counter_Value"]))
    c = {k: statistics.fmean(v) for k, v in ctr.items()}
    mb = (2 * c.get("FETCH_SIZE", 0.0) + c.get("WRITE_SIZE", 0.0)) / 1e3  # KB -> MB
    us = statistics.fmean(durs[g1])
    wc = max(c.get("SQ_WAVE_CYCLES", 1.0), 1.0)
    print(f"{m:5d} {g1:9d} {len(durs[g1]):4d} {us:8.2f} {mb:10.1f} {mb / us:6.2f} "
          f"{c.get('SQ_WAIT_ANY', 0.0) / wc:5.2f} {c.get('SQ_WAIT_INST_ANY', 0.0) / wc:9.2f}")
