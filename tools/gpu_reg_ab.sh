# Regular coupled rows (derived columns): full GPU suite, then same-box A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
NO_BENCH=1 bash tools/gpu_tests_bench.sh || exit $?
bash tools/gpu_env_ab.sh reg0:CFD_COUPLED_REG=0 reg1:CFD_COUPLED_REG=1 reg0b:CFD_COUPLED_REG=0 reg1b:CFD_COUPLED_REG=1 > gpurun_out/reg_ab.txt 2>&1
rc=$?
grep -E "k_spmv2|k_precond_predict2|k_precond_correct2|ms/step|reg" gpurun_out/reg_ab.txt | head -30
exit $rc
