# Round 4: single-workgroup tail threshold at C1 (levels 8.5 k / 2.3 k / 633 rows).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
CFG=c1 bash tools/gpu_ab_env.sh t4096=CFD_AMG_TAIL_ROWS=4096 t10k=CFD_AMG_TAIL_ROWS=10000 t1024=CFD_AMG_TAIL_ROWS=1024 t4096b=CFD_AMG_TAIL_ROWS=4096 t10kb=CFD_AMG_TAIL_ROWS=10000 > gpurun_out/ab_tail_c1.txt 2>&1 || exit $?
head -8 gpurun_out/ab_tail_c1.txt
grep -E "tail|resrestrict|k_amg_smooth<true, 1, true" gpurun_out/ab_tail_c1.txt
