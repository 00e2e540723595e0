set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_relax_fused.py tests/test_gpu_dist.py -x -v -m gpu -k "relax or precond" --timeout 200 --timeout-method thread > gpurun_out/relax4_tests.log 2>&1
rc=$?
tail -3 gpurun_out/relax4_tests.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/relax4_tests.log | head -30; exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/jprobe -o run -- \
  python3 $R/tools/jacobi_probe.py > $R/gpurun_out/jprobe.txt 2>&1 && \
python3 $R/tools/summarize_stats.py $R/gpurun_out/jprobe > $R/gpurun_out/jprobe_top.txt
cat $R/gpurun_out/jprobe.txt | tail -2; grep -E "relax" $R/gpurun_out/jprobe_top.txt
