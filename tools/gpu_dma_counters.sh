# Round 5: counters of the Schur prediction, plain vs LDS-DMA (CFD_PREDICT_DMA),
# C2, one bench step each: SQ issue / wait fractions, memory pipeline, and
# FETCH_SIZE / WRITE_SIZE -- separate --pmc passes, per-kernel averages.
set -o pipefail
ROOT=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
RX="k_precond_predict"
run() {  # name env counters...
  local name=$1 ev=$2; shift 2
  local out=$ROOT/gpurun_out/dmactr_$name
  mkdir -p $out
  (export $ev && timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-include-regex "$RX" --output-format csv -d $out -o run -- \
    python3 $ROOT/bench.py --config c2 --no-cpu-baseline --ref-workloads 0 --steps 1 --warmup 1 --mesh-cache /tmp/dmactr_c2.bin \
    > $out/bench.json 2> $out/bench.log)
}
for v in plain:CFD_PREDICT_DMA=0 dma:CFD_PREDICT_DMA=1; do
  n=${v%%:*}; e=${v#*:}
  run ${n}_sq $e SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES || exit $?
  run ${n}_mem $e TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE || exit $?
  run ${n}_fetch $e FETCH_SIZE || exit $?
  run ${n}_write $e WRITE_SIZE || exit $?
done
python3 - "$ROOT/gpurun_out" <<'PY'
import csv, glob, sys, collections, re
root = sys.argv[1]
def load(name):
    f = glob.glob(f"{root}/dmactr_{name}/**/*counter_collection.csv", recursive=True)[0]
    acc = collections.defaultdict(list)
    k0 = None
    for r in csv.DictReader(open(f)):
        k0 = re.search(r"k_\w+", r["Kernel_Name"]).group(0)
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return k0, {n: sum(v) / len(v) for n, v in acc.items()}
for v in ("plain", "dma"):
    k, sq = load(v + "_sq")
    _, mem = load(v + "_mem")
    _, fe = load(v + "_fetch")
    _, wr = load(v + "_write")
    wc = max(sq["SQ_WAVE_CYCLES"], 1)
    gui = mem["GRBM_GUI_ACTIVE"] / 8.0
    hit, miss = mem["TCC_HIT_sum"], mem["TCC_MISS_sum"]
    print(f"{k:26s} waves {sq['SQ_WAVES']:8.0f}  SQ_WAIT_ANY {sq['SQ_WAIT_ANY']/wc:5.2f}  SQ_WAIT_INST_ANY {sq['SQ_WAIT_INST_ANY']/wc:5.2f}"
          f"  active {sq['SQ_ACTIVE_INST_ANY']/wc:5.2f}  vmem/wave {sq['SQ_INSTS_VMEM']/max(sq['SQ_WAVES'],1):6.1f}"
          f"  lds/wave {sq['SQ_INSTS_LDS']/max(sq['SQ_WAVES'],1):6.1f}")
    print(f"{'':26s} TA busy {mem['TA_TA_BUSY_sum']/gui/256:5.2f}  TA stalled by TC {mem['TA_ADDR_STALLED_BY_TC_CYCLES_sum']/gui/256:5.2f}"
          f"  TD busy {mem['TD_TD_BUSY_sum']/gui/256:5.2f}  TD stalled by TC {mem['TD_TC_STALL_sum']/gui/256:5.2f}"
          f"  L2 hit {hit/max(hit+miss,1):5.2f}  HBM MB/launch {(2*fe['FETCH_SIZE'] + wr['WRITE_SIZE'])/1e3:8.1f} (FETCH_SIZE x 2 + WRITE_SIZE, KB units)")
PY
