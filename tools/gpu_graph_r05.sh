# Round 5: hipGraph replay of the FGMRES iteration.  The new / changed GPU
# tests first, then a same-box A/B of eager launches vs graph replay at C0
# (10 k Voronoi cells) and C1 (1 M cells), alternating, bench lines in
# gpurun_out/graph_<cfg>_<variant><k>.json.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_graph.py tests/test_capi_c.py \
  "tests/test_gpu_parity.py::test_amg_blob_shift_parity" "tests/test_gpu_edge.py::test_group_midstep_failure_needs_restore" \
  "tests/test_gpu_dist.py::test_group_variants_parity" \
  -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_graph.log 2>&1 || { tail -40 gpurun_out/gpu_tests_graph.log; exit 1; }
tail -3 gpurun_out/gpu_tests_graph.log
for cfg in ${CFGS:-c0 c1}; do
  for k in 1 2; do
    for v in eager graph; do
      g=0; [ $v = graph ] && g=1
      CFD_GRAPH=$g timeout -k 10 300 python bench.py --config $cfg --steps ${STEPS:-10} --no-cpu-baseline --ref-workloads 0 \
        --mesh-cache /tmp/graph_mesh_$cfg.bin > gpurun_out/graph_${cfg}_$v$k.json 2> gpurun_out/graph_${cfg}_$v$k.log || exit $?
      python -c "import json; d=json.load(open('gpurun_out/graph_${cfg}_$v$k.json')); print('$cfg $v$k', round(d['ms_per_step'],3), 'ms/step; smoother', round(d['roofline']['avg_launch_us'],2), 'us; graph', d.get('graph'))"
    done
  done
done
