# Round 4: level-0 regular waves (lengths, ranks and columns derived, not
# loaded) -- AMG parity tests, then same-box A/B at C2 and C1: off
# (CFD_AMG_REG=0), per wave (1, default), per quad (2).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_dist.py -x -q --timeout 300 --timeout-method thread -k "amg or c1 or c2 or variant or dist or halo or group" > gpurun_out/reg_tests.log 2>&1 || { tail -30 gpurun_out/reg_tests.log; exit 1; }
tail -3 gpurun_out/reg_tests.log
CFG=c2 bash tools/gpu_ab_env.sh noreg=CFD_AMG_REG=0 reg=CFD_AMG_REG=1 lane=CFD_AMG_REG=2 noreg2=CFD_AMG_REG=0 > gpurun_out/ab_reg_c2.txt 2>&1 || exit $?
head -16 gpurun_out/ab_reg_c2.txt
CFG=c1 bash tools/gpu_ab_env.sh noreg=CFD_AMG_REG=0 reg=CFD_AMG_REG=1 lane=CFD_AMG_REG=2 > gpurun_out/ab_reg_c1.txt 2>&1 || exit $?
head -16 gpurun_out/ab_reg_c1.txt
