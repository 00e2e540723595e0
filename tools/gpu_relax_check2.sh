set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_relax_fused.py -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/relax_tests.log 2>&1
rc=$?
tail -3 gpurun_out/relax_tests.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/relax_tests.log | head -30; exit $rc; fi
bash tools/gpu_ref_trace.sh
