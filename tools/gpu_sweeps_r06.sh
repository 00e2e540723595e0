# Round-6 fresh parity sweeps (seeds no earlier sweep drew): 400 small cases
# from seed 1000 (one in four in the reference-semantics test mode on one
# GPU), then 80 larger cases from seed 5000 on up to 8 ranks.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
CFD_SWEEP_SEED0=1000 CFD_SWEEP_CASES=400 timeout -k 10 700 python -u -m pytest tests/test_gpu_sweep.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/sweep400_r06.log 2>&1 || { tail -30 gpurun_out/sweep400_r06.log; exit 1; }
tail -2 gpurun_out/sweep400_r06.log
CFD_SWEEP_SEED0=5000 CFD_SWEEP_CASES=80 CFD_SWEEP_H_SCALE=0.5 CFD_SWEEP_MANY_RANKS=1 timeout -k 10 450 python -u -m pytest tests/test_gpu_sweep.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/sweep80_r06.log 2>&1 || { tail -30 gpurun_out/sweep80_r06.log; exit 1; }
tail -2 gpurun_out/sweep80_r06.log
