# Round 5: register-carried Givens chain -- parity files, then C1 and C0
# rocprofv3 --stats runs (k_norm_givens against 5.5 / 4.5-5.0 us).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_voronoi.py tests/test_gpu_edge.py tests/test_gpu_graph.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_givens.log 2>&1 || { tail -30 gpurun_out/gpu_tests_givens.log; exit 1; }
tail -2 gpurun_out/gpu_tests_givens.log
for c in c1 c0; do
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/givprof_$c -o run -- \
    python3 $R/bench.py --config $c --no-cpu-baseline --ref-workloads 0 --steps 3 --warmup 1 > $R/gpurun_out/givprof_$c.json 2> $R/gpurun_out/givprof_$c.log) || exit 1
  python3 tools/summarize_stats.py gpurun_out/givprof_$c | grep -E "norm_givens|total"
done
