# GPU test run: pytest on the given test paths / -k filters (default: every
# -m gpu test), one process, per-test timeout, output in gpurun_out/.
# Usage: bash tools/gpu_tests.sh <tag> [pytest args...]
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
tag=$1; shift
[ $# -eq 0 ] && set -- tests
timeout -k 10 1100 python -u -m pytest "$@" -x -v -m gpu --timeout 600 --timeout-method thread > gpurun_out/gpu_tests_$tag.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_tests_$tag.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/gpu_tests_$tag.log | head -40; fi
exit $rc
