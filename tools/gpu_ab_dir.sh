# Same-box A/B of library variants: bench c2 (or $CFG) once per variant name.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
CFG=${CFG:-c2}
for v in "$@"; do
  lib=cfd-demo2_amd/cfd2_amd/_lib/ab/libcfd2_amd_$v.so
  CFD2_AMD_LIB=$PWD/$lib timeout -k 10 400 python bench.py --config $CFG --no-cpu-baseline --mesh-cache /tmp/ab_mesh_$CFG.bin > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.log || exit $?
  python -c "
import json
d=json.load(open('gpurun_out/ab_$v.json')); r=d['roofline']
print('$v', 'ms/step %.2f'%d['ms_per_step'], 'smoother %.0f GB/s avg %.1f us'%(r['achieved'], r['avg_launch_us']))
"
done
