# Round 4: the coarsest level's 10 sweeps in one wavefront (no block
# barriers) inside the single-workgroup tail -- parity, then same-box A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_dist.py -x -q --timeout 300 --timeout-method thread -k "not c3 and not c4" > gpurun_out/tailwave_tests.log 2>&1 || { tail -30 gpurun_out/tailwave_tests.log; exit 1; }
tail -2 gpurun_out/tailwave_tests.log
CFG=c1 STEPS=10 bash tools/gpu_ab_prof.sh oldtail base oldtail base > gpurun_out/ab_tailwave_c1.txt 2>&1 || exit $?
head -8 gpurun_out/ab_tailwave_c1.txt; grep tail_blob gpurun_out/ab_tailwave_c1.txt
CFG=c2 STEPS=5 bash tools/gpu_ab_prof.sh oldtail base > gpurun_out/ab_tailwave_c2.txt 2>&1 || exit $?
head -4 gpurun_out/ab_tailwave_c2.txt; grep tail_blob gpurun_out/ab_tailwave_c2.txt
