# Round 5: C0 launch chains -- first slot group covering every coupled slot
# (variant u10: CFD_{PREDICT,CORRECT,SPMV}_U1=10) and 4-slot AMG groups
# (variant amgu4: CFD_AMG_U=4) against the in-tree library, same box, twice.
set -o pipefail
cd $GRAFT_REPO_ROOT
CFG=c0 bash tools/gpu_ab_prof.sh base u10 amgu4 > gpurun_out/ab_small_c0.txt 2>&1 || { tail -20 gpurun_out/ab_small_c0.txt; exit 1; }
head -40 gpurun_out/ab_small_c0.txt
CFG=c0 bash tools/gpu_ab_prof.sh amgu4 u10 base > gpurun_out/ab_small2_c0.txt 2>&1 || { tail -20 gpurun_out/ab_small2_c0.txt; exit 1; }
head -4 gpurun_out/ab_small2_c0.txt
