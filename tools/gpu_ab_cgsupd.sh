# Round 5 small-mesh A/Bs, same box:
#  1. CGS update on the default policy when the basis fits the kept bytes
#     (default) vs nontemporal (CFD_CGS_UPDATE_NT=1), C0 and C1, two passes;
#  2. LDS tail in TK=8 chunks (in-tree library) vs per entry (variant tk1,
#     CFD_TAIL_TK=1 in _lib/ab/), C0 and C1;
# then the parity subset that covers both.
set -o pipefail
cd $GRAFT_REPO_ROOT
for cfg in c0 c1; do
  CFG=$cfg bash tools/gpu_ab_env.sh nt_$cfg=CFD_CGS_UPDATE_NT=1 def_$cfg=CFD_CGS_UPDATE_NT=0 > gpurun_out/ab_cgsupd_$cfg.txt 2>&1 || { tail -20 gpurun_out/ab_cgsupd_$cfg.txt; exit 1; }
  head -16 gpurun_out/ab_cgsupd_$cfg.txt
  CFG=$cfg bash tools/gpu_ab_env.sh def_$cfg=CFD_CGS_UPDATE_NT=0 nt_$cfg=CFD_CGS_UPDATE_NT=1 > gpurun_out/ab_cgsupd2_$cfg.txt 2>&1 || { tail -20 gpurun_out/ab_cgsupd2_$cfg.txt; exit 1; }
  head -3 gpurun_out/ab_cgsupd2_$cfg.txt
done
for cfg in c0 c1; do
  CFG=$cfg bash tools/gpu_ab_prof.sh tk1 base > gpurun_out/ab_tailtk_$cfg.txt 2>&1 || { tail -20 gpurun_out/ab_tailtk_$cfg.txt; exit 1; }
  head -3 gpurun_out/ab_tailtk_$cfg.txt; grep tail_blob gpurun_out/ab_tailtk_$cfg.txt || true
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "variants or c1_scale or coupled_schemes or blob_shift" tests/test_gpu_robustness.py tests/test_voronoi.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_cgsupd.log 2>&1 || { tail -20 gpurun_out/gpu_tests_cgsupd.log; exit 1; }
tail -2 gpurun_out/gpu_tests_cgsupd.log
