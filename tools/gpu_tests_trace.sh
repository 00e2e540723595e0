# GPU tests, then the default bench line, then a C2 kernel trace.
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_tests_bench.sh && TAG=${TAG:-trace} bash tools/gpu_trace.sh c2
