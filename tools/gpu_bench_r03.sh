# Default bench line (C2, one GPU) and the C4 in-process 8-rank rehearsal
# (collective counts per FGMRES iteration on the distributed path).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
tag=${1:-r03}
[ "${SKIP_C2:-0}" = 1 ] || timeout -k 10 600 python -u bench.py > gpurun_out/bench_c2_$tag.json 2> gpurun_out/bench_c2_$tag.log || exit $?
[ "${SKIP_C2:-0}" = 1 ] || cat gpurun_out/bench_c2_$tag.json
timeout -k 10 540 python -u bench.py --inproc-ranks 8 --steps 3 --warmup 2 --ref-workloads 0 --no-cpu-baseline \
  > gpurun_out/bench_inproc8_$tag.json 2> gpurun_out/bench_inproc8_$tag.log || exit $?
cat gpurun_out/bench_inproc8_$tag.json
