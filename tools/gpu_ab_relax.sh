# Same-box A/B of the fused Jacobi relaxation (old vs new library): parity test
# with the new library, then the reference's solver benchmark alternating libs.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_relax_fused.py -x -v --timeout 120 --timeout-method thread > gpurun_out/ab_relax_tests.log 2>&1 || { tail -30 gpurun_out/ab_relax_tests.log; exit 1; }
tail -2 gpurun_out/ab_relax_tests.log
for v in ${VARIANTS:-old new old new}; do
  CFD2_AMD_LIB=$PWD/cfd-demo2_amd/cfd2_amd/_lib/ab/libcfd2_amd_$v.so timeout -k 10 200 python -u tools/ref_workload_run.py solver_step > gpurun_out/ab_relax_$v.json 2> gpurun_out/ab_relax_$v.log || exit $?
  echo "$v $(cat gpurun_out/ab_relax_$v.json | tr -d '\n' | cut -c1-300)"
done
