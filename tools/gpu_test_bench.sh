# GPU parity tests, then c1 + c2 benchmarks (no CPU baseline).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -5 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/gpu_tests.log | head -20; exit $rc; fi
timeout -k 10 300 python bench.py --config c1 --no-cpu-baseline > gpurun_out/bench_c1.json 2> gpurun_out/bench_c1.log && \
timeout -k 10 400 python bench.py --config c2 --no-cpu-baseline > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.log && \
python -c "
import json
for c in ('c1','c2'):
    d=json.load(open('gpurun_out/bench_%s.json'%c)); r=d['roofline']
    print(c, 'value %.4g'%d['value'], 'ms/step %.2f'%d['ms_per_step'], 'smoother %.0f GB/s (%.1f%%) avg %.1f us'%(r['achieved'], 100*r['frac'], r['avg_launch_us']))
"
