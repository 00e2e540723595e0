# Round-5 evidence, part C: rocprofv3 kernel stats + PMC traffic of one whole
# step (FETCH_SIZE / WRITE_SIZE in separate passes) at C2 and C1.
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_step_traffic.sh r05 c2 || exit $?
bash tools/gpu_step_traffic.sh r05 c1 || exit $?
ls gpurun_out/steptraffic_r05_c2 gpurun_out/steptraffic_r05_c1
