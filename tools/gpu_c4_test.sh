# The C4 parity test alone (timing of the driver's -m gpu run).
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_tests.sh c4 tests/test_gpu_configs.py::test_c4_group8_one_gpu_and_oracle -s || exit $?
grep -E "C4|passed|failed" gpurun_out/gpu_tests_c4.log
