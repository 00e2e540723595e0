# GPU tests (one process, per-test timeout), smoke, then the default bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/gpu_tests.log | head -30; exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
cat gpurun_out/smoke.log
timeout -k 10 900 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.log || exit $?
cat gpurun_out/bench_default.json
