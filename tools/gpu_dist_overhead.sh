# Kernel-time breakdown of the distributed algorithm on one GPU: C1 single vs
# C1 with --inproc-ranks R (each rank ~1 M cells), rocprofv3 kernel traces.
set -o pipefail
ROOT=$GRAFT_REPO_ROOT
R=${1:-2}
OUT=$ROOT/gpurun_out/distov
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/single -o run -- \
  python3 $ROOT/bench.py --config c1 --no-cpu-baseline --steps 2 --warmup 1 > $OUT/single.json 2> $OUT/single.log && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/inproc -o run -- \
  python3 $ROOT/bench.py --config c1 --inproc-ranks $R --no-cpu-baseline --steps 2 --warmup 1 > $OUT/inproc.json 2> $OUT/inproc.log && \
python3 - $OUT $R <<'PY'
import csv, glob, sys, collections, json, re
d, R = sys.argv[1], int(sys.argv[2])
def load(sub):
    f = glob.glob(f"{d}/{sub}/**/*kernel_stats.csv", recursive=True)[0]
    out = collections.Counter()
    for r in csv.DictReader(open(f)):
        m = re.search(r"k_\w+", r["Name"])
        out[m.group(0) if m else r["Name"][:30]] += float(r["TotalDurationNs"]) / 1e6
    return out
s, p = load("single"), load("inproc")
for k in sorted(set(s) | set(p), key=lambda k: -(p[k] - R * s[k])):
    if abs(p[k] - R * s[k]) > 0.5:
        print(f"{k:34s} single x{R} {R*s[k]:9.2f} ms   inproc {p[k]:9.2f} ms   diff {p[k]-R*s[k]:+8.2f}")
print("total kernel ms: single x R", round(R * sum(s.values()), 1), " inproc", round(sum(p.values()), 1))
for n in ("single", "inproc"):
    j = json.load(open(f"{d}/{n}.json")); print(n, "ms/step", round(j["ms_per_step"], 1), "cells", j["config"]["cells_total"])
PY
