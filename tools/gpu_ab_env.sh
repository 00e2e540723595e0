# Same-box A/B of runtime settings: each argument is NAME:VAR=VAL[,VAR=VAL]
# (e.g. lds:CFD_AMG_TAIL_LDS=1 glob:CFD_AMG_TAIL_LDS=0); bench $CFG (c2) each.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
CFG=${CFG:-c2}
for spec in "$@"; do
  name=${spec%%:*}
  envs=${spec#*:}
  timeout -k 10 400 env ${envs//,/ } python bench.py --config $CFG --no-cpu-baseline --ref-workloads 0 --mesh-cache /tmp/ab_mesh_$CFG.bin > gpurun_out/abe_$name.json 2> gpurun_out/abe_$name.log || exit $?
  python -c "
import json
d=json.load(open('gpurun_out/abe_$name.json')); r=d['roofline']
print('$name', 'ms/step %.2f'%d['ms_per_step'], 'smoother %.0f GB/s avg %.1f us'%(r['achieved'], r['avg_launch_us']))
"
done
