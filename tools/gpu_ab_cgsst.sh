# Round 4: CGS new-basis store policy (nontemporal vs default) at C2 and C1,
# now that the prediction's matrix loads no longer allocate in the Infinity
# Cache; and the level-0 pre-smoother with a split load policy.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
CFG=c2 STEPS=10 bash tools/gpu_ab_prof.sh base cgsst > gpurun_out/ab_cgsst_c2.txt 2>&1 || exit $?
head -20 gpurun_out/ab_cgsst_c2.txt
CFG=c2 STEPS=10 bash tools/gpu_env_ab.sh base:CFD_NT_PRE_SPLIT=0 sp25:CFD_NT_PRE_SPLIT=0.25 sp50:CFD_NT_PRE_SPLIT=0.5 sp75:CFD_NT_PRE_SPLIT=0.75 > gpurun_out/ab_presplit_c2.txt 2>&1 || exit $?
head -20 gpurun_out/ab_presplit_c2.txt
CFG=c1 STEPS=10 bash tools/gpu_ab_prof.sh base cgsst > gpurun_out/ab_cgsst_c1.txt 2>&1 || exit $?
head -20 gpurun_out/ab_cgsst_c1.txt
