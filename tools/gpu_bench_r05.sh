# Round-5 evidence, part B: the default bench line (C2 + CPU baseline + the
# reference's own workloads), C1, C0 (Voronoi), and the in-process
# rehearsals with the comm-timing table (C1 x2 quick, C4 x8).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
tag=${1:-r05}
timeout -k 10 600 python -u bench.py --round r05 > gpurun_out/bench_c2_$tag.json 2> gpurun_out/bench_c2_$tag.log || exit $?
cat gpurun_out/bench_c2_$tag.json
timeout -k 10 300 python -u bench.py --round r05 --config c1 --ref-workloads 0 --no-cpu-baseline > gpurun_out/bench_c1_$tag.json 2> gpurun_out/bench_c1_$tag.log || exit $?
cat gpurun_out/bench_c1_$tag.json
timeout -k 10 300 python -u bench.py --round r05 --config c0 --ref-workloads 0 > gpurun_out/bench_c0_$tag.json 2> gpurun_out/bench_c0_$tag.log || exit $?
cat gpurun_out/bench_c0_$tag.json
timeout -k 10 300 python -u bench.py --round r05 --config c1 --inproc-ranks 2 --steps 2 --warmup 1 --ref-workloads 0 --no-cpu-baseline > gpurun_out/bench_inproc2_c1_$tag.json 2> gpurun_out/bench_inproc2_c1_$tag.log || exit $?
cat gpurun_out/bench_inproc2_c1_$tag.json
exit 0  # C4: tools/gpu_inproc8_r05.sh (both aggregation modes)
timeout -k 10 600 python -u bench.py --round r05 --inproc-ranks 8 --steps 3 --warmup 2 --ref-workloads 0 --no-cpu-baseline > gpurun_out/bench_inproc8_$tag.json 2> gpurun_out/bench_inproc8_$tag.log || exit $?
cat gpurun_out/bench_inproc8_$tag.json
