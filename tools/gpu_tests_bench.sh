# GPU tests (one process, per-test timeout) then the default bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/gpu_tests.log | head -40; exit $rc; fi
[ -n "$NO_BENCH" ] && exit 0
timeout -k 10 900 python -u bench.py --ref-workloads 0 --no-cpu-baseline > gpurun_out/bench_default.json 2> gpurun_out/bench_default.log || exit $?
cat gpurun_out/bench_default.json
