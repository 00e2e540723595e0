# Round 4: CGS keep-in-cache as the default below 2^22 cells (64 MB) --
# parity (GPU tests that run meshes below and above the threshold), then
# same-box A/B: C1 / C0 default vs off, C2 update top-down alone vs default.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_dist.py tests/test_voronoi.py -x -q --timeout 300 --timeout-method thread -k "not c3 and not c4 and not sweep" > gpurun_out/cgskeep3_tests.log 2>&1 || { tail -30 gpurun_out/cgskeep3_tests.log; exit 1; }
tail -2 gpurun_out/cgskeep3_tests.log
CFG=c1 bash tools/gpu_ab_env.sh off=CFD_CGS_KEEP_MB=0 on=CFD_NT=47 off2=CFD_CGS_KEEP_MB=0 on2=CFD_NT=47 > gpurun_out/ab_cgskeep3_c1.txt 2>&1 || exit $?
head -8 gpurun_out/ab_cgskeep3_c1.txt
CFG=c0 bash tools/gpu_ab_env.sh off=CFD_CGS_KEEP_MB=0 on=CFD_NT=47 off2=CFD_CGS_KEEP_MB=0 on2=CFD_NT=47 > gpurun_out/ab_cgskeep3_c0.txt 2>&1 || exit $?
head -8 gpurun_out/ab_cgskeep3_c0.txt
CFG=c2 bash tools/gpu_ab_env.sh k0=CFD_CGS_KEEP_MB=0 rev=CFD_CGS_KEEP_MB=1 k0b=CFD_CGS_KEEP_MB=0 revb=CFD_CGS_KEEP_MB=1 > gpurun_out/ab_cgskeep3_c2.txt 2>&1 || exit $?
head -10 gpurun_out/ab_cgskeep3_c2.txt
