# Round 4: Schur prediction / correction, the face sweeps and the level-0
# pre-smoother in block dispatch order from 2^22 rows on
# (CoupledMatrix::schur_flat, AmgLevelDev::flat) -- parity tests, then
# same-box A/B at C2: remap everywhere / flat without / with the pre-smoother.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread -k "variant or c2 or c1" > gpurun_out/flat_tests.log 2>&1 || { tail -30 gpurun_out/flat_tests.log; exit 1; }
tail -3 gpurun_out/flat_tests.log
CFG=c2 bash tools/gpu_ab_env.sh remap=CFD_FLAT_ROWS=4294967295 flat=CFD_FLAT_PRE=0 flatpre=CFD_FLAT_PRE=1 remap2=CFD_FLAT_ROWS=4294967295 flat2=CFD_FLAT_PRE=0 flatpre2=CFD_FLAT_PRE=1 > gpurun_out/ab_flat_c2.txt 2>&1 || exit $?
head -18 gpurun_out/ab_flat_c2.txt
