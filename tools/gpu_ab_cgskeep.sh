# Round 4: the CGS dots pass's last blocks read the basis with the default
# policy (CFD_CGS_KEEP_MB of lines kept in the Infinity Cache) and the update
# walks the blocks top-down to find them -- parity, then same-box A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_dist.py -x -q --timeout 300 --timeout-method thread -k "variant or c2 or fixed or group_amg" > gpurun_out/cgskeep_tests.log 2>&1 || { tail -30 gpurun_out/cgskeep_tests.log; exit 1; }
tail -2 gpurun_out/cgskeep_tests.log
CFG=c2 bash tools/gpu_ab_env.sh k0=CFD_CGS_KEEP_MB=0 k128=CFD_CGS_KEEP_MB=128 k224=CFD_CGS_KEEP_MB=224 k0b=CFD_CGS_KEEP_MB=0 k128b=CFD_CGS_KEEP_MB=128 k224b=CFD_CGS_KEEP_MB=224 > gpurun_out/ab_cgskeep_c2.txt 2>&1 || exit $?
head -12 gpurun_out/ab_cgskeep_c2.txt
CFG=c1 bash tools/gpu_ab_env.sh k0=CFD_CGS_KEEP_MB=0 k128=CFD_CGS_KEEP_MB=128 k224=CFD_CGS_KEEP_MB=224 > gpurun_out/ab_cgskeep_c1.txt 2>&1 || exit $?
head -8 gpurun_out/ab_cgskeep_c1.txt
