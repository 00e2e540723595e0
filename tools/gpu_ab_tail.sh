# A/B of the single-workgroup AMG tail threshold on c2 (bench only).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for t in ${@:-0 16384}; do
  CFD_AMG_TAIL_ROWS=$t timeout -k 10 400 python bench.py --config c2 --no-cpu-baseline > gpurun_out/bench_c2_tail$t.json 2> gpurun_out/bench_c2_tail$t.log || exit $?
  python -c "
import json
d=json.load(open('gpurun_out/bench_c2_tail$t.json')); r=d['roofline']
print('tail<=$t', 'value %.4g'%d['value'], 'ms/step %.2f'%d['ms_per_step'], 'smoother %.0f GB/s (%.1f%%)'%(r['achieved'], 100*r['frac']))
"
done
