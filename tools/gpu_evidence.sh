# Round evidence at the current sources: every -m gpu test, smoke, the default
# bench line (C2 + CPU baseline + the reference's own workloads) and C1.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
tag=${1:-r03}
bash tools/gpu_tests.sh all_$tag tests || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$tag.log 2>&1 || exit $?
cat gpurun_out/smoke_$tag.log
timeout -k 10 600 python -u bench.py > gpurun_out/bench_c2_$tag.json 2> gpurun_out/bench_c2_$tag.log || exit $?
cat gpurun_out/bench_c2_$tag.json
timeout -k 10 300 python -u bench.py --config c1 --ref-workloads 0 --no-cpu-baseline > gpurun_out/bench_c1_$tag.json 2> gpurun_out/bench_c1_$tag.log || exit $?
cat gpurun_out/bench_c1_$tag.json
