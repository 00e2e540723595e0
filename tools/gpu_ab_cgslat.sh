# Round 5: CGS dots / update in the latency form on small meshes (default,
# CFD_CGS_LAT=1) vs the streaming form (=0): parity first, then same-box A/B
# at C0 (two passes) and the reference's 8,125-cell solver workload.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_voronoi.py tests/test_gpu_graph.py tests/test_gpu_edge.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_cgslat.log 2>&1 || { tail -30 gpurun_out/gpu_tests_cgslat.log; exit 1; }
tail -2 gpurun_out/gpu_tests_cgslat.log
CFG=c0 bash tools/gpu_ab_env.sh str_c0=CFD_CGS_LAT=0 lat_c0=CFD_CGS_LAT=1 > gpurun_out/ab_cgslat_c0.txt 2>&1 || { tail -20 gpurun_out/ab_cgslat_c0.txt; exit 1; }
head -16 gpurun_out/ab_cgslat_c0.txt
CFG=c0 bash tools/gpu_ab_env.sh lat_c0=CFD_CGS_LAT=1 str_c0=CFD_CGS_LAT=0 > gpurun_out/ab_cgslat2_c0.txt 2>&1 || { tail -20 gpurun_out/ab_cgslat2_c0.txt; exit 1; }
head -3 gpurun_out/ab_cgslat2_c0.txt
for v in 0 1 0 1; do
  CFD_CGS_LAT=$v timeout -k 10 300 python -u tools/ref_workload_run.py solver_step > gpurun_out/ref_solver_step_lat$v.txt 2>&1 || { tail -20 gpurun_out/ref_solver_step_lat$v.txt; exit 1; }
  echo "CFD_CGS_LAT=$v"; tail -2 gpurun_out/ref_solver_step_lat$v.txt
done
