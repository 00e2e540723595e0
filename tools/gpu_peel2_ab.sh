set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c2.py tests/test_gpu_dist.py -x -q -m gpu -k "variants or c2 or amg_test" --timeout 300 --timeout-method thread > gpurun_out/peel2_tests.log 2>&1 || { tail -30 gpurun_out/peel2_tests.log; exit 1; }
tail -2 gpurun_out/peel2_tests.log
CFD_AMG_PEEL2=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_c2.py tests/test_gpu_dist.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/peel2_tests2.log 2>&1 || { tail -30 gpurun_out/peel2_tests2.log; exit 1; }
tail -2 gpurun_out/peel2_tests2.log
bash tools/gpu_env_ab.sh p0:CFD_AMG_PEEL2=0 p1:CFD_AMG_PEEL2=1 p0b:CFD_AMG_PEEL2=0 p1b:CFD_AMG_PEEL2=1 > gpurun_out/peel2_ab.txt 2>&1
rc=$?
grep -E "k_amg_smooth|k_amg_residual|ms/step|total" gpurun_out/peel2_ab.txt | head -30
exit $rc
