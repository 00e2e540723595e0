# Round-4 final evidence: bench lines (C2 with CPU baseline + the reference's
# workloads, C1, C0, in-process 2 ranks) and the SQ / memory-pipeline counters
# of the bandwidth kernels at C2.
set -o pipefail
cd $GRAFT_REPO_ROOT
SKIP_C4=1 bash tools/gpu_bench_r04.sh r04final || exit $?
bash tools/gpu_sq.sh > gpurun_out/c2_sq_counters_r04.txt 2>&1 || exit $?
bash tools/gpu_mem_counters.sh > gpurun_out/c2_mem_counters_r04.txt 2>&1 || exit $?
cat gpurun_out/c2_sq_counters_r04.txt gpurun_out/c2_mem_counters_r04.txt
