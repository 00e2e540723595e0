# Level-0 AMG regular groups (derived columns): full GPU suite, then same-box A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
NO_BENCH=1 bash tools/gpu_tests_bench.sh || exit $?
bash tools/gpu_env_ab.sh areg0:CFD_AMG_REG=0 areg1:CFD_AMG_REG=1 areg0b:CFD_AMG_REG=0 areg1b:CFD_AMG_REG=1 > gpurun_out/amgreg_ab.txt 2>&1
rc=$?
grep -E "k_amg_smooth|k_amg_residual|ms/step|areg" gpurun_out/amgreg_ab.txt | head -30
exit $rc
