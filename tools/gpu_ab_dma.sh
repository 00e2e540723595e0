# Round 5: the LDS-DMA Schur prediction (CFD_PREDICT_DMA=1) and the SpMV fused
# with the CGS dots (CFD_SPMV_DOTS=1).  Parity first,
# then same-box A/B with per-kernel times at C2 (and C1 with CFGS="c2 c1").
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest "tests/test_gpu_parity.py::test_predict_dma_parity" "tests/test_gpu_parity.py::test_spmv_dots_parity" -x -v -m gpu \
  --timeout 240 --timeout-method thread > gpurun_out/gpu_tests_dma.log 2>&1 || { tail -30 gpurun_out/gpu_tests_dma.log; exit 1; }
tail -2 gpurun_out/gpu_tests_dma.log
for cfg in ${CFGS:-c2}; do
  CFG=$cfg bash tools/gpu_ab_env.sh base_$cfg=CFD_PREDICT_DMA=0 dma_$cfg=CFD_PREDICT_DMA=1 sd_$cfg=CFD_SPMV_DOTS=1 > gpurun_out/ab_dma_$cfg.txt 2>&1 || { tail -20 gpurun_out/ab_dma_$cfg.txt; exit 1; }
  head -16 gpurun_out/ab_dma_$cfg.txt
done
