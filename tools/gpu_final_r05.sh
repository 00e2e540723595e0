# Round 5 late check: parity files, a C0 kernel profile (triangular solve),
# then the bench lines (C2 + CPU baseline + reference workloads, C1, C0, in-process x2).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_voronoi.py tests/test_gpu_edge.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_late.log 2>&1 || { tail -30 gpurun_out/gpu_tests_late.log; exit 1; }
tail -2 gpurun_out/gpu_tests_late.log
R=$GRAFT_REPO_ROOT
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/c0prof_late -o run -- \
  python3 $R/bench.py --config c0 --no-cpu-baseline --ref-workloads 0 --steps 3 --warmup 1 > $R/gpurun_out/c0prof_late.json 2> $R/gpurun_out/c0prof_late.log) || exit 1
python3 tools/summarize_stats.py gpurun_out/c0prof_late > gpurun_out/c0_kernel_top_late.txt && grep -E "triangular|total" gpurun_out/c0_kernel_top_late.txt
bash tools/gpu_bench_r05.sh r05d
