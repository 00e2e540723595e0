# Same-box A/B of an environment knob on the reference's two benchmarks:
# ENVS="A B ..." where each entry is NAME=VALUE (or "-" for none).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for e in $ENVS; do
  if [ "$e" = "-" ]; then envset=""; else envset="$e"; fi
  env $envset timeout -k 10 300 python -u tools/ref_workload_run.py all > gpurun_out/ab_env.json 2> gpurun_out/ab_env.log || exit $?
  python -c "
import json; d=json.load(open('gpurun_out/ab_env.json'))
print('$e', {k: round(x['ms_per_step'], 3) for k, x in d.items()})"
done
