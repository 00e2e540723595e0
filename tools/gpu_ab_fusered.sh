# Round 5: CGS totals reduced inside the update kernel (default on meshes up
# to 256 reduction units) vs k_cgs_reduce launched (CFD_CGS_FUSE_REDUCE=0),
# same box, C0 twice alternating; then the parity files that cover it.
set -o pipefail
cd $GRAFT_REPO_ROOT
CFG=c0 bash tools/gpu_ab_env.sh sep_c0=CFD_CGS_FUSE_REDUCE=0 fused_c0=CFD_CGS_FUSE_REDUCE=1 > gpurun_out/ab_fusered_c0.txt 2>&1 || { tail -20 gpurun_out/ab_fusered_c0.txt; exit 1; }
head -16 gpurun_out/ab_fusered_c0.txt
CFG=c0 bash tools/gpu_ab_env.sh fused_c0=CFD_CGS_FUSE_REDUCE=1 sep_c0=CFD_CGS_FUSE_REDUCE=0 > gpurun_out/ab_fusered2_c0.txt 2>&1 || { tail -20 gpurun_out/ab_fusered2_c0.txt; exit 1; }
head -3 gpurun_out/ab_fusered2_c0.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edge.py tests/test_voronoi.py tests/test_gpu_graph.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_fusered.log 2>&1 || { tail -30 gpurun_out/gpu_tests_fusered.log; exit 1; }
tail -2 gpurun_out/gpu_tests_fusered.log
