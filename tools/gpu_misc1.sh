# Voronoi GPU tests, then a natural-convergence C2 measurement (3 steps).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_voronoi.py -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --no-cpu-baseline --outer 0 --inner 0 --steps 3 --warmup 2 > gpurun_out/natural.json 2> gpurun_out/natural.log || exit $?
cat gpurun_out/natural.log
python -c "import json; d=json.load(open('gpurun_out/natural.json')); print('natural', d['ms_per_step'], d['value'], d['linear_iterations_last_step'])"
