# Round 5: fused Jacobi relaxation with the DPP neighbour path on regular row
# groups (in-tree) vs the round-4 kernel (variant nodpp, CFD_RELAX_DPP=0 in
# _lib/ab/): relaxation parity tests, then the reference's 8,125-cell solver
# workload alternating, and one rocprofv3 --stats run of each.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_relax_fused.py tests/test_gpu_parity.py -k "relax or jacobi or coupled_schemes or midrun" -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_relaxdpp.log 2>&1 || { tail -30 gpurun_out/gpu_tests_relaxdpp.log; exit 1; }
tail -2 gpurun_out/gpu_tests_relaxdpp.log
for v in base nodpp base nodpp; do
  if [ $v = base ]; then lib=$R/cfd-demo2_amd/cfd2_amd/_lib/libcfd2_amd.so; else lib=$R/cfd-demo2_amd/cfd2_amd/_lib/ab/libcfd2_amd_$v.so; fi
  CFD2_AMD_LIB=$lib timeout -k 10 300 python -u tools/ref_workload_run.py solver_step > gpurun_out/ref_ss_$v.txt 2>&1 || { tail -20 gpurun_out/ref_ss_$v.txt; exit 1; }
  echo "$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ref_ss_$v.txt)"
done
for v in base nodpp; do
  if [ $v = base ]; then lib=$R/cfd-demo2_amd/cfd2_amd/_lib/libcfd2_amd.so; else lib=$R/cfd-demo2_amd/cfd2_amd/_lib/ab/libcfd2_amd_$v.so; fi
  (cd /tmp && export TMPDIR=/tmp && CFD2_AMD_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/relaxprof_$v -o run -- \
    python3 $R/tools/ref_workload_run.py solver_step > $R/gpurun_out/relaxprof_$v.json 2> $R/gpurun_out/relaxprof_$v.log) || exit 1
  python3 tools/summarize_stats.py gpurun_out/relaxprof_$v | grep -E "relax|total" 
done
