# Round 5: k_amg_smooth with its first-needed level fields as leading
# (SGPR-preloaded) arguments (in-tree) vs the library before (variant old in
# _lib/ab/): parity files, then C1 twice and C0 once.
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_voronoi.py tests/test_gpu_edge.py tests/test_gpu_dist.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_smhead.log 2>&1 || { tail -30 gpurun_out/gpu_tests_smhead.log; exit 1; }
tail -2 gpurun_out/gpu_tests_smhead.log
CFG=c1 bash tools/gpu_ab_prof.sh old base > gpurun_out/ab_smhead_c1.txt 2>&1 || { tail -20 gpurun_out/ab_smhead_c1.txt; exit 1; }
grep -E "ms/step|amg_smooth" gpurun_out/ab_smhead_c1.txt
CFG=c1 bash tools/gpu_ab_prof.sh base old > gpurun_out/ab_smhead2_c1.txt 2>&1 || { tail -20 gpurun_out/ab_smhead2_c1.txt; exit 1; }
head -2 gpurun_out/ab_smhead2_c1.txt
CFG=c0 bash tools/gpu_ab_prof.sh old base > gpurun_out/ab_smhead_c0.txt 2>&1 || { tail -20 gpurun_out/ab_smhead_c0.txt; exit 1; }
grep -E "ms/step|amg_smooth" gpurun_out/ab_smhead_c0.txt
