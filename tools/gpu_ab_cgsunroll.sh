# Round 5: streaming CGS loops with 2 / 4 basis vectors' loads issued together
# (build-time CFD_CGS_UNROLL; variants un2 / un4 in _lib/ab/) vs the in-tree
# library: C1 twice, C2 once.
set -o pipefail
cd $GRAFT_REPO_ROOT
CFG=c1 bash tools/gpu_ab_prof.sh base un2 un4 > gpurun_out/ab_cgsunroll_c1.txt 2>&1 || { tail -20 gpurun_out/ab_cgsunroll_c1.txt; exit 1; }
head -8 gpurun_out/ab_cgsunroll_c1.txt
CFG=c1 bash tools/gpu_ab_prof.sh un4 un2 base > gpurun_out/ab_cgsunroll2_c1.txt 2>&1 || { tail -20 gpurun_out/ab_cgsunroll2_c1.txt; exit 1; }
head -8 gpurun_out/ab_cgsunroll2_c1.txt
CFG=c2 STEPS=5 bash tools/gpu_ab_prof.sh base un2 un4 > gpurun_out/ab_cgsunroll_c2.txt 2>&1 || { tail -20 gpurun_out/ab_cgsunroll_c2.txt; exit 1; }
head -8 gpurun_out/ab_cgsunroll_c2.txt
