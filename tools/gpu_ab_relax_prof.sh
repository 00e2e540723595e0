# Kernel-trace A/B of the fused Jacobi relaxation: rocprofv3 stats per library.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in ${VARIANTS:-old new}; do
  export CFD2_AMD_LIB=$PWD/cfd-demo2_amd/cfd2_amd/_lib/ab/libcfd2_amd_$v.so
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abprof_$v -o run -- python3 tools/ref_workload_run.py solver_step > gpurun_out/abprof_$v.log 2>&1 || exit $?
  f=$(ls gpurun_out/abprof_$v/*/run_kernel_stats.csv 2>/dev/null || ls gpurun_out/abprof_$v/run_kernel_stats.csv)
  echo "== $v"; grep -E "relax|Name" $f | cut -c1-200
done
