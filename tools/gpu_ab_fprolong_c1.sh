# Round 4: fused prolongation threshold at C1 (level 0 = 1,001,745 rows sits
# just under the 2^20 default): 2^20 vs 2^19 (level 0 separate).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
CFG=c1 bash tools/gpu_ab_env.sh r20=CFD_AMG_FUSED_PROLONG_ROWS=1048576 r19=CFD_AMG_FUSED_PROLONG_ROWS=524288 r20b=CFD_AMG_FUSED_PROLONG_ROWS=1048575 r19b=CFD_AMG_FUSED_PROLONG_ROWS=524287 > gpurun_out/ab_fprolong_c1.txt 2>&1 || exit $?
head -16 gpurun_out/ab_fprolong_c1.txt
