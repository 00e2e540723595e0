# Round 4: GPU tests after the knob prune, then same-box A/B of the
# nontemporal matrix-load policy per kernel (CFD_NT bit mask, Solver::nt_mask).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/gpu_tests.sh prune tests/test_gpu_parity.py tests/test_gpu_configs.py::test_c2_headline_schedule_bitexact || exit $?
CFG=${CFG:-c2} STEPS=10 bash tools/gpu_env_ab.sh base:CFD_NT=0 post:CFD_NT=1 res:CFD_NT=2 pred:CFD_NT=4 spmv:CFD_NT=8 pre:CFD_NT=16 all:CFD_NT=15 > gpurun_out/ab_nt_c2.txt 2>&1 || exit $?
cat gpurun_out/ab_nt_c2.txt
