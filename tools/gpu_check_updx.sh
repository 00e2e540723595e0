# Round 5: latency-form k_update_x_lat on small meshes -- parity files, then a
# C0 rocprofv3 --stats run (update kernel time against round 5's 15 us).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_voronoi.py tests/test_gpu_edge.py tests/test_gpu_relax_fused.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_updx.log 2>&1 || { tail -30 gpurun_out/gpu_tests_updx.log; exit 1; }
tail -2 gpurun_out/gpu_tests_updx.log
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/c0prof_updx -o run -- \
  python3 $R/bench.py --config c0 --no-cpu-baseline --ref-workloads 0 --steps 3 --warmup 1 > $R/gpurun_out/c0prof_updx.json 2> $R/gpurun_out/c0prof_updx.log) || exit 1
python3 tools/summarize_stats.py gpurun_out/c0prof_updx > gpurun_out/c0_kernel_top_updx.txt && grep -E "update_x|triangular|total" gpurun_out/c0_kernel_top_updx.txt
for i in 1 2; do timeout -k 10 300 python -u bench.py --config c0 --no-cpu-baseline --ref-workloads 0 > gpurun_out/b_c0_updx$i.json 2> gpurun_out/b_c0_updx$i.log || exit 1; grep -o '"ms_per_step": [0-9.]*' gpurun_out/b_c0_updx$i.json; done
