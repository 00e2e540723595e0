# Round 4: is C0 (10 k Voronoi cells) host-launch-bound?  Kernel trace of 2
# timed steps; tools/trace_steps.py compares the summed kernel time with the
# wall span of the trace.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
ROOT=$GRAFT_REPO_ROOT
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/c0trace -o run -- \
  python3 $ROOT/bench.py --config c0 --no-cpu-baseline --ref-workloads 0 --steps 3 --warmup 1 > $ROOT/gpurun_out/c0trace.json 2> $ROOT/gpurun_out/c0trace.log) || exit $?
python tools/trace_steps.py gpurun_out/c0trace 2 > gpurun_out/c0_busy.txt && cat gpurun_out/c0_busy.txt
