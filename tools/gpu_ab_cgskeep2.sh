# Round 4: CGS keep-in-cache at C1 (the 1 M-cell basis: 12 MB per vector):
# rev-only (1 MB), 64 / 128 / 192 MB, two rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
CFG=c1 bash tools/gpu_ab_env.sh k0=CFD_CGS_KEEP_MB=0 k1=CFD_CGS_KEEP_MB=1 k64=CFD_CGS_KEEP_MB=64 k128=CFD_CGS_KEEP_MB=128 k192=CFD_CGS_KEEP_MB=192 k0b=CFD_CGS_KEEP_MB=0 k64b=CFD_CGS_KEEP_MB=64 k128b=CFD_CGS_KEEP_MB=128 > gpurun_out/ab_cgskeep2_c1.txt 2>&1 || exit $?
head -14 gpurun_out/ab_cgskeep2_c1.txt
