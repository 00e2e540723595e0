# Round-6 evidence: the default bench line (C2 + CPU baseline + the
# reference's own workloads), C1 with its CPU baseline (VERDICT r05 Next 7),
# C0 (Voronoi), and smoke.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
tag=${1:-r06}
timeout -k 10 600 python -u bench.py > gpurun_out/bench_c2_$tag.json 2> gpurun_out/bench_c2_$tag.log || exit $?
cat gpurun_out/bench_c2_$tag.json
timeout -k 10 400 python -u bench.py --config c1 --ref-workloads 0 > gpurun_out/bench_c1_$tag.json 2> gpurun_out/bench_c1_$tag.log || exit $?
cat gpurun_out/bench_c1_$tag.json
timeout -k 10 300 python -u bench.py --config c0 --ref-workloads 0 > gpurun_out/bench_c0_$tag.json 2> gpurun_out/bench_c0_$tag.log || exit $?
cat gpurun_out/bench_c0_$tag.json
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$tag.log 2>&1 || exit $?
cat gpurun_out/smoke_$tag.log
