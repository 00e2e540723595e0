# rocprofv3 evidence for profiles/<round>: kernel trace + stats of the bench
# command, then FETCH_SIZE and WRITE_SIZE in separate PMC passes restricted to
# the AMG smoother kernel; summaries written under gpurun_out/prof_<round>.
set -o pipefail
R=${1:-r01}
CFG=${2:-c2}
ROOT=$GRAFT_REPO_ROOT
OUT=$ROOT/gpurun_out/prof_$R
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 $ROOT/bench.py --config $CFG --no-cpu-baseline --steps 3 --warmup 2 > $OUT/bench_trace.json 2> $OUT/bench_trace.log && \
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_amg_smooth --output-format csv -d $OUT/pmc_fetch -o run -- \
  python3 $ROOT/bench.py --config $CFG --no-cpu-baseline --steps 1 --warmup 2 > $OUT/bench_fetch.json 2> $OUT/bench_fetch.log && \
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_amg_smooth --output-format csv -d $OUT/pmc_write -o run -- \
  python3 $ROOT/bench.py --config $CFG --no-cpu-baseline --steps 1 --warmup 2 > $OUT/bench_write.json 2> $OUT/bench_write.log && \
python3 $ROOT/tools/summarize_stats.py $OUT/trace > $OUT/kernel_top.txt && \
python3 $ROOT/tools/pmc_summary.py $OUT $OUT/smoother_pmc.json $CFG

# Per-kernel HBM traffic of every kernel (profiles/r01/c2_kernel_traffic.txt):
#   bash tools/gpu_pmc_all.sh c2   (FETCH_SIZE and WRITE_SIZE passes, no kernel filter)
# Default bench line with the CPU baseline (profiles/r01/bench_c2.json):
#   python bench.py
