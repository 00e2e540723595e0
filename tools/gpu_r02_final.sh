# Round-2 evidence: GPU tests, smoke, the default bench line (C2 with the CPU
# baseline and the reference workloads), and the C1 bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
NO_BENCH=1 bash tools/gpu_tests_bench.sh || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 900 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.log || exit $?
timeout -k 10 300 python -u bench.py --config c1 --ref-workloads 0 > gpurun_out/bench_c1.json 2> gpurun_out/bench_c1.log || exit $?
tail -2 gpurun_out/smoke.log
cut -c1-300 gpurun_out/bench_default.json gpurun_out/bench_c1.json
