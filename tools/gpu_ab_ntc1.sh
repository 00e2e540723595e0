# Round 4: the nontemporal mask at C1 after the CGS keep change (47 default,
# 0 none, 32 prolongation only, 15 post/residual/predict/SpMV).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
CFG=c1 bash tools/gpu_ab_env.sh nt47=CFD_NT=47 nt0=CFD_NT=0 nt32=CFD_NT=32 nt15=CFD_NT=15 nt47b=CFD_NT=47 nt0b=CFD_NT=0 > gpurun_out/ab_ntc1.txt 2>&1 || exit $?
head -24 gpurun_out/ab_ntc1.txt
