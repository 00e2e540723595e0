# VERDICT r05 Next 4, second half: k_precond_predict2 with its first-needed
# fields (row ranges, j, grid size, binv, w_in, lg, drank) as leading arguments,
# the 14 dwords the command processor preloads into SGPRs, so no wave waits on
# a kernarg load before its first global load (the hidden grid-size load
# included).  Variant library _lib/ab/libcfd2_amd_phead.so (built on the CPU
# host from the patch recorded in profiles/r06/ab_phead.patch).
# 1. bit-exact: the GPU parity and reference-kernel suites on the variant;
# 2. same-box C2 A/B, 3 alternating rounds (tools/gpu_ab_r06_regression.sh);
# 3. per-kernel times under rocprofv3 (tools/gpu_ab_prof.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
CFD2_AMD_LIB=$GRAFT_REPO_ROOT/cfd-demo2_amd/cfd2_amd/_lib/ab/libcfd2_amd_phead.so timeout -k 10 600 \
  python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_wgsl_pin.py \
  > gpurun_out/phead_tests.log 2>&1 || exit $?
tail -3 gpurun_out/phead_tests.log
ROUNDS=3 bash tools/gpu_ab_r06_regression.sh base phead > gpurun_out/phead_ab.txt 2>&1 || { cat gpurun_out/phead_ab.txt; exit 1; }
cat gpurun_out/phead_ab.txt
bash tools/gpu_ab_prof.sh base phead > gpurun_out/phead_prof.txt 2>&1 || { tail -20 gpurun_out/phead_prof.txt; exit 1; }
cat gpurun_out/phead_prof.txt
