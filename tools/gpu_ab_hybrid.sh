# Round 5: the level above a shifted LDS image inside the tail kernel with its
# matrix in global memory (CFD_AMG_TAIL_HYBRID=1, default) vs two row-kernel
# launches (=0): parity first, then same-box A/B at C0 and C1, two passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -k "hybrid or blob_shift or variants or c1_scale or voronoi" tests/test_voronoi.py tests/test_gpu_graph.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_hybrid.log 2>&1 || { tail -30 gpurun_out/gpu_tests_hybrid.log; exit 1; }
tail -2 gpurun_out/gpu_tests_hybrid.log
for cfg in c0 c1; do
  CFG=$cfg bash tools/gpu_ab_env.sh off_$cfg=CFD_AMG_TAIL_HYBRID=0 hyb_$cfg=CFD_AMG_TAIL_HYBRID=1 > gpurun_out/ab_hybrid_$cfg.txt 2>&1 || { tail -20 gpurun_out/ab_hybrid_$cfg.txt; exit 1; }
  head -30 gpurun_out/ab_hybrid_$cfg.txt
  CFG=$cfg bash tools/gpu_ab_env.sh hyb_$cfg=CFD_AMG_TAIL_HYBRID=1 off_$cfg=CFD_AMG_TAIL_HYBRID=0 > gpurun_out/ab_hybrid2_$cfg.txt 2>&1 || { tail -20 gpurun_out/ab_hybrid2_$cfg.txt; exit 1; }
  head -3 gpurun_out/ab_hybrid2_$cfg.txt
done
