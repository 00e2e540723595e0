# SQ counters of the fused Jacobi relaxation (reference solver benchmark):
# LDS bank conflicts vs LDS-array cycles, LDS issue stalls, wave state split.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY --kernel-include-regex relax_pressure_fused --output-format csv -d $R/gpurun_out/relax_sq -o run -- python3 $R/tools/ref_workload_run.py solver_step > $R/gpurun_out/relax_sq.log 2>&1
rc=$?
ls $R/gpurun_out/relax_sq
exit $rc
