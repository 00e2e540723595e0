# Round-5 evidence at the current sources, part A: every -m gpu test (C3 / C4
# oracle legs included) and smoke.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
tag=${1:-r05}
bash tools/gpu_tests.sh all_$tag tests || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$tag.log 2>&1 || exit $?
cat gpurun_out/smoke_$tag.log
