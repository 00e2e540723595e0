# Round 5: shorter dependent chains on the latency-bound AMG levels -- the
# R-ordered member image of k_amg_resrestrict (CFD_AMG_RR_PERM) and the
# column-aggregate image of the fused post-smoother (CFD_AMG_AGGC_ROWS).
# Parity subset first, then same-box A/B at C1 and C2.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "variants or c1_scale or rebuild or refresh" \
  tests/test_gpu_c2.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_chain.log 2>&1 \
  || { tail -30 gpurun_out/gpu_tests_chain.log; exit 1; }
tail -2 gpurun_out/gpu_tests_chain.log
for cfg in ${CFGS:-c1 c2}; do
  CFG=$cfg bash tools/gpu_ab_env.sh "base_$cfg=CFD_AMG_RR_PERM=0 CFD_AMG_AGGC_ROWS=0" "perm_$cfg=CFD_AMG_AGGC_ROWS=0" \
    "aggc18_$cfg=CFD_AMG_AGGC_ROWS=262144" "aggc20_$cfg=CFD_AMG_AGGC_ROWS=1048576" > gpurun_out/ab_chain_$cfg.txt 2>&1 \
    || { tail -20 gpurun_out/ab_chain_$cfg.txt; exit 1; }
  head -30 gpurun_out/ab_chain_$cfg.txt
done
