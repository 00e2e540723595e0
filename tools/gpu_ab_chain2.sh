# Round 5: compile-time A/B of the chain-shortening images (branch-free
# kernels): old = r04 kernels (CFD_RR_PERM=0, CFD_AGGC=0), perm = member
# image only, base = both (in-tree).  C1 twice, then C2.
set -o pipefail
cd $GRAFT_REPO_ROOT
CFG=c1 bash tools/gpu_ab_prof.sh old perm base > gpurun_out/ab_chain2_c1a.txt 2>&1 || { tail -20 gpurun_out/ab_chain2_c1a.txt; exit 1; }
head -30 gpurun_out/ab_chain2_c1a.txt
CFG=c1 bash tools/gpu_ab_prof.sh base perm old > gpurun_out/ab_chain2_c1b.txt 2>&1 || { tail -20 gpurun_out/ab_chain2_c1b.txt; exit 1; }
head -4 gpurun_out/ab_chain2_c1b.txt
CFG=c2 bash tools/gpu_ab_prof.sh old base > gpurun_out/ab_chain2_c2.txt 2>&1 || { tail -20 gpurun_out/ab_chain2_c2.txt; exit 1; }
head -30 gpurun_out/ab_chain2_c2.txt
