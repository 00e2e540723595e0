# Round 5: fused residual + restriction on C1's 500 k-row level 1 (rows limit
# 600 000) and also its 1 M-row level 0 (1 100 000) vs the 2^18 default.
set -o pipefail
cd $GRAFT_REPO_ROOT
CFG=c1 bash tools/gpu_ab_env.sh def_c1=CFD_AMG_FUSED_RR_ROWS=262144 l1_c1=CFD_AMG_FUSED_RR_ROWS=600000 l01_c1=CFD_AMG_FUSED_RR_ROWS=1100000 > gpurun_out/ab_rr_c1.txt 2>&1 || { tail -20 gpurun_out/ab_rr_c1.txt; exit 1; }
head -24 gpurun_out/ab_rr_c1.txt
CFG=c1 bash tools/gpu_ab_env.sh l01_c1=CFD_AMG_FUSED_RR_ROWS=1100000 l1_c1=CFD_AMG_FUSED_RR_ROWS=600000 def_c1=CFD_AMG_FUSED_RR_ROWS=262144 > gpurun_out/ab_rr2_c1.txt 2>&1 || { tail -20 gpurun_out/ab_rr2_c1.txt; exit 1; }
head -4 gpurun_out/ab_rr2_c1.txt
