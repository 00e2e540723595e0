# Per-step counter traffic (tools/step_traffic.py) + the level-0 smoother PMC
# summary (tools/pmc_summary.py) for profiles/<round>; each rocprofv3 pass runs
# on its own with its own time limit.
set -o pipefail
R=${1:-r03}
CFG=${2:-c2}
ROOT=$GRAFT_REPO_ROOT
OUT=$ROOT/gpurun_out/steptraffic_${R}_$CFG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
MC=$ROOT/gpurun_out/mesh_$CFG.bin
B="python3 $ROOT/bench.py --config $CFG --no-cpu-baseline --ref-workloads 0 --mesh-cache $MC"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  $B --steps 3 --warmup 2 > $OUT/bench_trace.json 2> $OUT/bench_trace.log && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- \
  $B --steps 1 --warmup 1 > $OUT/bench_fetch.json 2> $OUT/bench_fetch.log && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- \
  $B --steps 1 --warmup 1 > $OUT/bench_write.json 2> $OUT/bench_write.log && \
rm -f $MC && \
python3 $ROOT/tools/step_traffic.py $OUT $CFG $OUT/${CFG}_step_traffic.json && \
python3 $ROOT/tools/summarize_stats.py $OUT/trace > $OUT/kernel_top.txt && \
python3 $ROOT/tools/pmc_summary.py $OUT $OUT/smoother_pmc.json $CFG && \
python3 $ROOT/tools/pmc_all_summary.py $OUT > $OUT/kernel_traffic.txt
