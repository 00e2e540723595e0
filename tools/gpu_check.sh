# GPU parity tests then a c2 kernel trace (TAG=... for the output dir name).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/gpu_tests.log | head -20; exit $rc; fi
TAG=${TAG:-trace} bash tools/gpu_trace.sh ${@:-c2}
