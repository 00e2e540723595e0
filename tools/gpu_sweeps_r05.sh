# Wide seeded parity sweeps on the final round-5 sources (partition-aware AMG mode and graph replay drawn per case):
# (round 2: fused / 4-row Jacobi sweeps, regular coupled rows; round 3: fused prolongation): 400 small cases, then 80 larger cases on up to 8 ranks.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
CFD_SWEEP_CASES=400 timeout -k 10 600 python -u -m pytest tests/test_gpu_sweep.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/sweep400_r05.log 2>&1 || { tail -30 gpurun_out/sweep400_r05.log; exit 1; }
tail -2 gpurun_out/sweep400_r05.log
CFD_SWEEP_CASES=80 CFD_SWEEP_H_SCALE=0.5 CFD_SWEEP_MANY_RANKS=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_sweep.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/sweep80_r05.log 2>&1 || { tail -30 gpurun_out/sweep80_r05.log; exit 1; }
tail -2 gpurun_out/sweep80_r05.log
