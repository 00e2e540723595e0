set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
NO_BENCH=1 bash tools/gpu_tests_bench.sh || exit $?
timeout -k 10 300 python3 tools/ref_workload_run.py all > gpurun_out/ref_all.json 2> gpurun_out/ref_all.log || exit $?
cut -c1-130 gpurun_out/ref_all.json
timeout -k 10 240 python -u bench.py --config c0 --ref-workloads 0 --no-cpu-baseline > gpurun_out/bench_c0b.json 2> gpurun_out/bench_c0b.log || exit $?
cut -c1-250 gpurun_out/bench_c0b.json
