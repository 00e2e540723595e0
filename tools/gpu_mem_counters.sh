# Memory-pipeline counters of the bandwidth kernels (one --pmc pass within the
# per-block limits: 2 TA, 2 TD, 4 TCP, 2 TCC, 1 GRBM), one C2 bench step.
set -o pipefail
ROOT=$GRAFT_REPO_ROOT
OUT=$ROOT/gpurun_out/memctr
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum \
  TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCR_TCP_STALL_CYCLES_sum \
  TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE \
  --kernel-include-regex "k_spmv|k_precond|k_amg_smooth|k_amg_residual|k_cgs_dots|k_cgs_update" --output-format csv -d $OUT -o run -- \
  python3 $ROOT/bench.py --config c2 --no-cpu-baseline --ref-workloads 0 --steps 1 --warmup 1 --mesh-cache /tmp/memctr_c2.bin > $OUT/bench.json 2> $OUT/bench.log && \
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections, re
d = sys.argv[1]
f = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    k = (re.search(r"k_\w+(<[^>]*>)?", r["Kernel_Name"]).group(0), int(r.get("Grid_Size", r.get("Grid_Size_X", 0))))
    acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
names = sorted({n for k in acc for n in acc[k]})
print("# per-dispatch averages; *_BUSY / *STALL* as a fraction of per-XCD active cycles (GRBM_GUI_ACTIVE / 8: rocprofv3 sums it over the 8 XCDs) x 256 CUs")
for k in sorted(acc, key=lambda k: -sum(acc[k].get("GRBM_GUI_ACTIVE", [0]))):
    m = {n: sum(acc[k][n]) / max(len(acc[k][n]), 1) for n in names}
    gui = max(m.get("GRBM_GUI_ACTIVE", 8.0), 8.0) / 8.0  # per-XCD cycles
    hit, miss = m.get("TCC_HIT_sum", 0.0), m.get("TCC_MISS_sum", 0.0)
    print(f"{k[0]:28s} {k[1]:9d} cycles/XCD {gui:8.0f}  TA busy {m.get('TA_TA_BUSY_sum',0)/gui/256:5.2f}"
          f"  TA stalled by TC {m.get('TA_ADDR_STALLED_BY_TC_CYCLES_sum',0)/gui/256:5.2f}"
          f"  TD busy {m.get('TD_TD_BUSY_sum',0)/gui/256:5.2f}  TD stalled by TC {m.get('TD_TC_STALL_sum',0)/gui/256:5.2f}"
          f"  TCP pending stall {m.get('TCP_PENDING_STALL_CYCLES_sum',0)/gui/256:5.2f}"
          f"  TCP<-TCR stall {m.get('TCP_TCR_TCP_STALL_CYCLES_sum',0)/gui/256:5.2f}"
          f"  L2 hit {hit / max(hit + miss, 1):5.2f}  TCP->TCC reads {m.get('TCP_TCC_READ_REQ_sum',0):.3g}")
PY
