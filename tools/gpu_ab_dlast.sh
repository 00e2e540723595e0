# Round 4: the CGS dots read the newest basis vector V_j with the default
# policy (allocating it in the Infinity Cache for the update right after).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
CFG=c2 STEPS=10 bash tools/gpu_ab_prof.sh base dlast base > gpurun_out/ab_dlast_c2.txt 2>&1 || exit $?
head -12 gpurun_out/ab_dlast_c2.txt
CFG=c1 STEPS=10 bash tools/gpu_ab_prof.sh base dlast > gpurun_out/ab_dlast_c1.txt 2>&1 || exit $?
head -12 gpurun_out/ab_dlast_c1.txt
