# Round 5: the norm + Givens step run by the last block of the latency-form
# CGS update (default, CFD_CGS_FUSE_GIVENS=1) vs k_norm_givens launched (=0):
# parity first, then same-box A/B at C0 and the reference 8,125-cell workload.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_voronoi.py tests/test_gpu_graph.py tests/test_gpu_edge.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_fusegiv.log 2>&1 || { tail -30 gpurun_out/gpu_tests_fusegiv.log; exit 1; }
tail -2 gpurun_out/gpu_tests_fusegiv.log
CFG=c0 bash tools/gpu_ab_env.sh sep_c0=CFD_CGS_FUSE_GIVENS=0 ngf_c0=CFD_CGS_FUSE_GIVENS=1 > gpurun_out/ab_cgsngf_c0.txt 2>&1 || { tail -20 gpurun_out/ab_cgsngf_c0.txt; exit 1; }
head -16 gpurun_out/ab_cgsngf_c0.txt
CFG=c0 bash tools/gpu_ab_env.sh ngf_c0=CFD_CGS_FUSE_GIVENS=1 sep_c0=CFD_CGS_FUSE_GIVENS=0 > gpurun_out/ab_fusegiv2_c0.txt 2>&1 || { tail -20 gpurun_out/ab_fusegiv2_c0.txt; exit 1; }
head -3 gpurun_out/ab_fusegiv2_c0.txt
for v in 0 1 0 1; do
  CFD_CGS_FUSE_GIVENS=$v timeout -k 10 300 python -u tools/ref_workload_run.py solver_step > gpurun_out/ref_solver_step_giv$v.txt 2>&1 || { tail -20 gpurun_out/ref_solver_step_giv$v.txt; exit 1; }
  echo "CFD_CGS_FUSE_GIVENS=$v"; tail -2 gpurun_out/ref_solver_step_giv$v.txt
done
