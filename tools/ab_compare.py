"""Per-kernel comparison of tools/gpu_ab_prof.sh variants: ms/step of the plain
bench run, then the average duration per (kernel, grid) group of each variant's
rocprofv3 trace.  Usage: ab_compare.py VARIANT ..."""
import collections
import csv
import glob
import json
import re
import statistics
import sys

vs = sys.argv[1:]


def short(name):
    m = re.search(r"k_\w+(<[^>]*>)?", name)
    return m.group(0) if m else name[:40]


tabs = {}
for v in vs:
    d = json.load(open(f"gpurun_out/ab_{v}.json"))
    print(f"{v:12s} ms/step {d['ms_per_step']:.2f}  smoother {d['roofline']['avg_launch_us']:.1f} us")
    f = glob.glob(f"gpurun_out/abprof_{v}/**/*kernel_trace.csv", recursive=True)[0]
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        acc[(short(r["Kernel_Name"]), int(r.get("Grid_Size", r.get("Grid_Size_X", 0))))].append(
            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    tabs[v] = acc
base = tabs[vs[0]]
# every (kernel, grid) group of any variant (a fused kernel replaces the base's pair)
allk = set().union(*[set(t) for t in tabs.values()])
keys = sorted(allk, key=lambda k: -max(sum(tabs[v].get(k, [])) for v in vs))[:40]
print(f"{'kernel':34s} {'grid':>9s} " + " ".join(f"{v[:10]:>10s}" for v in vs) + "   (avg us)")
for k in keys:
    cells = [f"{statistics.fmean(tabs[v][k]):10.2f}" if k in tabs[v] else f"{'-':>10s}" for v in vs]
    print(f"{k[0][:34]:34s} {k[1]:9d} " + " ".join(cells))
tot = {v: sum(sum(x) for x in tabs[v].values()) / 1e3 for v in vs}
print("total kernel ms:", " ".join(f"{v}={tot[v]:.1f}" for v in vs))
