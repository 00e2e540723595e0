# SQ counters of the C2 row kernels (current kernels) + the C1 kernel trace.
set -o pipefail
R=$GRAFT_REPO_ROOT
bash $R/tools/gpu_sq.sh > $R/gpurun_out/sq_summary.txt || exit $?
TAG=final bash $R/tools/gpu_trace.sh c1 > $R/gpurun_out/c1_top.txt || exit $?
python3 $R/tools/trace_steps.py $R/gpurun_out/final_c1 > $R/gpurun_out/c1_steps.txt
head -12 $R/gpurun_out/sq_summary.txt; head -4 $R/gpurun_out/c1_steps.txt
