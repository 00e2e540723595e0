# Fused Jacobi relax: its parity tests + the Jacobi / small-mesh parity tests,
# then the reference workloads timed (solver_step is the Jacobi benchmark).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_relax_fused.py tests/test_gpu_parity.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/relax_tests.log 2>&1
rc=$?
tail -3 gpurun_out/relax_tests.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/relax_tests.log | head -30; exit $rc; fi
timeout -k 10 300 python3 tools/ref_workload_run.py all > gpurun_out/ref_all.json 2> gpurun_out/ref_all.log || exit $?
cut -c1-700 gpurun_out/ref_all.json
