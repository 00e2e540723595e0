# Round 4: CGS new-basis store policy (nontemporal vs default) at C2 and C1,
# now that the prediction's matrix loads no longer allocate in the Infinity Cache.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
CFG=c2 STEPS=10 bash tools/gpu_ab_prof.sh base cgsst > gpurun_out/ab_cgsst_c2.txt 2>&1 || exit $?
cat gpurun_out/ab_cgsst_c2.txt | head -20
CFG=c1 STEPS=10 bash tools/gpu_ab_prof.sh base cgsst > gpurun_out/ab_cgsst_c1.txt 2>&1 || exit $?
cat gpurun_out/ab_cgsst_c1.txt | head -20
