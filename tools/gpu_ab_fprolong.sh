# Round 4: the prolongation fused into the post-smoother on the big levels
# too (CFD_AMG_FUSED_PROLONG_ROWS: default 2^20; 2^23 adds level 1, 2^24
# level 0), re-measured under the nontemporal policy -- same-box A/B at C2.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
CFG=c2 bash tools/gpu_ab_env.sh r20=CFD_AMG_FUSED_PROLONG_ROWS=1048576 r23=CFD_AMG_FUSED_PROLONG_ROWS=8388608 r24=CFD_AMG_FUSED_PROLONG_ROWS=16777216 r20b=CFD_AMG_FUSED_PROLONG_ROWS=1048576 r23b=CFD_AMG_FUSED_PROLONG_ROWS=8388608 r24b=CFD_AMG_FUSED_PROLONG_ROWS=16777216 > gpurun_out/ab_fprolong_c2.txt 2>&1 || exit $?
head -24 gpurun_out/ab_fprolong_c2.txt
