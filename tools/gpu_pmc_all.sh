# Per-kernel HBM traffic for every kernel of one bench step: FETCH_SIZE and
# WRITE_SIZE in separate rocprofv3 --pmc passes (no kernel filter), plus a
# kernel trace for durations; summarised by tools/pmc_all_summary.py.
set -o pipefail
CFG=${1:-c2}
ROOT=$GRAFT_REPO_ROOT
OUT=$ROOT/gpurun_out/pmc_all_$CFG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
MC=$ROOT/gpurun_out/mesh_$CFG.bin
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 $ROOT/bench.py --config $CFG --no-cpu-baseline --ref-workloads 0 --steps 1 --warmup 1 --mesh-cache $MC > $OUT/bench_trace.json 2> $OUT/bench_trace.log && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- \
  python3 $ROOT/bench.py --config $CFG --no-cpu-baseline --ref-workloads 0 --steps 1 --warmup 1 --mesh-cache $MC > $OUT/bench_fetch.json 2> $OUT/bench_fetch.log && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- \
  python3 $ROOT/bench.py --config $CFG --no-cpu-baseline --ref-workloads 0 --steps 1 --warmup 1 --mesh-cache $MC > $OUT/bench_write.json 2> $OUT/bench_write.log && \
rm -f $MC && \
python3 $ROOT/tools/pmc_all_summary.py $OUT > $OUT/summary.txt && cat $OUT/summary.txt
