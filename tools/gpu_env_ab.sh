# Same-box A/B of runtime settings: each argument is "name:ENV=V[,ENV=V]"; bench
# (CFG, default c2) once plain and once under rocprofv3 --kernel-trace --stats
# per setting; tools/ab_compare.py prints the per-kernel table.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
CFG=${CFG:-c2}
ROOT=$GRAFT_REPO_ROOT
names=()
for spec in "$@"; do
  v=${spec%%:*}
  envs=${spec#*:}
  names+=("$v")
  envarg=$(echo "$envs" | tr ',' ' ')
  env $envarg timeout -k 10 300 python bench.py --config $CFG --steps ${STEPS:-10} --no-cpu-baseline --ref-workloads 0 --mesh-cache /tmp/ab_mesh_$CFG.bin > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.log || exit $?
  (cd /tmp && export TMPDIR=/tmp && export $envarg && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/abprof_$v -o run -- \
    python3 $ROOT/bench.py --config $CFG --no-cpu-baseline --ref-workloads 0 --steps 2 --warmup 1 --mesh-cache /tmp/ab_mesh_$CFG.bin > $ROOT/gpurun_out/abprof_$v.json 2> $ROOT/gpurun_out/abprof_$v.log) || exit $?
done
python tools/ab_compare.py "${names[@]}"
