# SQ issue/stall counters for the row kernels (one --pmc pass, <= 8 SQ counters).
set -o pipefail
ROOT=$GRAFT_REPO_ROOT
OUT=$ROOT/gpurun_out/sq
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM SQ_WAVES \
  --kernel-include-regex "k_spmv|k_precond|k_amg_smooth|k_amg_residual|k_cgs_dots|k_cgs_update|k_amg_restrict|k_amg_resrestrict" --output-format csv -d $OUT -o run -- \
  python3 $ROOT/bench.py --config c2 --no-cpu-baseline --ref-workloads 0 --steps 1 --warmup 1 > $OUT/bench.json 2> $OUT/bench.log && \
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections, re
d = sys.argv[1]
f = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    k = (re.search(r"k_\w+(<[^>]*>)?", r["Kernel_Name"]).group(0), int(r.get("Grid_Size", r.get("Grid_Size_X", 0))))
    acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
names = ["SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_INSTS_VALU", "SQ_INSTS_VMEM", "SQ_WAVES"]
for k in sorted(acc, key=lambda k: -sum(acc[k]["SQ_WAVE_CYCLES"])):
    m = {n: sum(acc[k][n]) / max(len(acc[k][n]), 1) for n in names}
    wc = max(m["SQ_WAVE_CYCLES"], 1)
    print(f"{k[0]:28s} {k[1]:9d} waves {m['SQ_WAVES']:9.0f} wait {m['SQ_WAIT_ANY']/wc:5.2f} winst {m['SQ_WAIT_INST_ANY']/wc:5.2f} active {m['SQ_ACTIVE_INST_ANY']/wc:5.2f} valu {m['SQ_ACTIVE_INST_VALU']/wc:5.2f} valu/wave {m['SQ_INSTS_VALU']/max(m['SQ_WAVES'],1):7.1f} vmem/wave {m['SQ_INSTS_VMEM']/max(m['SQ_WAVES'],1):6.1f}")
PY
