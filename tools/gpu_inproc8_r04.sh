# Round-4 evidence, part D: C4 as 8 in-process ranks on one GPU (the whole
# distributed algorithm), with the comm-timing table of the extra step.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py --round r04 --inproc-ranks 8 --steps 3 --warmup 2 --ref-workloads 0 --no-cpu-baseline > gpurun_out/bench_inproc8_r04.json 2> gpurun_out/bench_inproc8_r04.log || exit $?
cat gpurun_out/bench_inproc8_r04.json
