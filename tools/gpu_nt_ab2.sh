# Round 4: new GPU tests (mid-step group failure, comm timing, NT variants),
# then same-box A/B of nontemporal-policy combinations (CFD_NT bit mask).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/gpu_tests.sh r4new tests/test_gpu_edge.py tests/test_gpu_dist.py::test_comm_timing_categories_and_bits "tests/test_gpu_parity.py::test_amg_kernel_variants_parity" || exit $?
CFG=${CFG:-c2} STEPS=10 bash tools/gpu_env_ab.sh base:CFD_NT=0 nt15:CFD_NT=15 nt47:CFD_NT=47 nt79:CFD_NT=79 nt111:CFD_NT=111 nt239:CFD_NT=239 > gpurun_out/ab_nt2_c2.txt 2>&1 || exit $?
cat gpurun_out/ab_nt2_c2.txt
timeout -k 10 120 ./tools/bin/xcd_barrier_probe > gpurun_out/xcd_barrier_probe.txt 2>&1 || exit $?
cat gpurun_out/xcd_barrier_probe.txt
timeout -k 10 300 ./tools/bin/stream_probe 1 > gpurun_out/stream_probe_r04_x1.txt 2>&1 || exit $?
timeout -k 10 300 ./tools/bin/stream_probe 4 > gpurun_out/stream_probe_r04_x4.txt 2>&1 || exit $?
cat gpurun_out/stream_probe_r04_x1.txt gpurun_out/stream_probe_r04_x4.txt
