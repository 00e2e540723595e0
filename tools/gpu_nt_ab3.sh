# Round 4: nontemporal policy, third round: the pre-smoother and the coarse
# residuals on top of the default mask (47).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
CFG=c2 STEPS=10 bash tools/gpu_env_ab.sh m47:CFD_NT=47 m63:CFD_NT=63 m111:CFD_NT=111 m127:CFD_NT=127 m47b:CFD_NT=47 > gpurun_out/ab_nt3_c2.txt 2>&1 || exit $?
head -40 gpurun_out/ab_nt3_c2.txt
