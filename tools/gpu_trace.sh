# rocprofv3 kernel trace + stats of the bench for each config given (default c1 c2).
set -o pipefail
ROOT=$GRAFT_REPO_ROOT
TAG=${TAG:-trace}
cd /tmp && export TMPDIR=/tmp
for CFG in ${@:-c1 c2}; do
  OUT=$ROOT/gpurun_out/${TAG}_$CFG
  mkdir -p $OUT
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
    python3 $ROOT/bench.py --config $CFG --no-cpu-baseline --ref-workloads 0 --steps 3 --warmup 2 > $OUT/bench.json 2> $OUT/bench.log || exit $?
  python3 $ROOT/tools/summarize_stats.py $OUT || exit $?
done
