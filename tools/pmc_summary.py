"""Summarise the rocprofv3 PMC passes of tools/gpu_profile.sh into
profiles/<round>/smoother_pmc.json: FETCH_SIZE / WRITE_SIZE per launch of the
level-0 AMG smoother (the launches with the largest grid), gfx950 FETCH
correction (x2, MI355X_MICROARCH.md), plus the trace's average duration of the
same launches.  Usage: pmc_summary.py <prof dir> <out json> <config label>"""
import csv
import glob
import json
import statistics
import sys

d, out, label = sys.argv[1], sys.argv[2], sys.argv[3]


def rows(pattern):
    f = glob.glob(f"{d}/{pattern}", recursive=True)
    if not f:
        sys.exit(f"missing {pattern} under {d}")
    return list(csv.DictReader(open(f[0])))


def level0(rs, key="Grid_Size"):
    sm = [r for r in rs if "k_amg_smooth" in r["Kernel_Name"]]
    g = max(int(r[key]) for r in sm)
    return [r for r in sm if int(r[key]) == g], g


fetch, grid = level0(rows("pmc_fetch/**/*counter_collection.csv"))
write, _ = level0(rows("pmc_write/**/*counter_collection.csv"))
fk = statistics.fmean(float(r["Counter_Value"]) for r in fetch if r["Counter_Name"] == "FETCH_SIZE")
wk = statistics.fmean(float(r["Counter_Value"]) for r in write if r["Counter_Name"] == "WRITE_SIZE")
trace = rows("trace/**/*kernel_trace.csv")
tr = [r for r in trace if "k_amg_smooth" in r["Kernel_Name"]]
tg = max(int(r["Grid_Size_X"]) for r in tr)
durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in tr if int(r["Grid_Size_X"]) == tg]
bench = json.load(open(f"{d}/bench_trace.json"))
alg = bench["roofline"]["bytes_per_launch"]
res = {
    "kernel": f"k_amg_smooth, AMG level 0 (grid {grid} threads), config {label}",
    "launches_pmc": len(fetch),
    "FETCH_SIZE_kB_per_launch": fk,
    "WRITE_SIZE_kB_per_launch": wk,
    "correction": ("gfx950: FETCH_SIZE reports 1/2 of the bytes of coalesced streaming reads "
                   "(MI355X_MICROARCH.md §HBM) -> fetch bytes = 2*FETCH_SIZE*1024; WRITE_SIZE exact"),
    "hbm_bytes_per_launch": 2 * fk * 1024 + wk * 1024,
    "algorithmic_bytes_per_launch": alg,
    "trace_avg_us": statistics.fmean(durs),
    "trace_median_us": statistics.median(durs),
    "trace_launches": len(durs),
    "bench_live_avg_us": bench["roofline"]["avg_launch_us"],
    "note": "FETCH counts L2->fabric requests incl. Infinity-Cache hits.",
}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
