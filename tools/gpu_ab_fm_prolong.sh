# Round 5: the reference's fine_mesh workload (1.06 M cells: level 0 just
# above the fused prolongation's 2^20-row limit) with the fused form on
# level 0 (CFD_AMG_FUSED_PROLONG_ROWS=1200000) vs the default, alternating.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in def fused def fused; do
  if [ $v = fused ]; then export CFD_AMG_FUSED_PROLONG_ROWS=1200000; else unset CFD_AMG_FUSED_PROLONG_ROWS; fi
  timeout -k 10 300 python -u tools/ref_workload_run.py fine_mesh > gpurun_out/ref_fm_$v.txt 2>&1 || { tail -20 gpurun_out/ref_fm_$v.txt; exit 1; }
  echo "$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ref_fm_$v.txt)"
done
