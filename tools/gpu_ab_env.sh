# Same-box A/B of environment variants of the in-tree library, with per-kernel
# times (as tools/gpu_ab_prof.sh for library variants).  Arguments: name=ENV
# pairs, e.g. noreg=CFD_AMG_REG=0 reg=CFD_AMG_REG=1; tools/ab_compare.py
# prints the per-kernel table by name.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
CFG=${CFG:-c2}
ROOT=$GRAFT_REPO_ROOT
names=()
for a in "$@"; do
  v=${a%%=*}; e=${a#*=}
  names+=("$v")
  env $e timeout -k 10 300 python bench.py --config $CFG --steps ${STEPS:-10} --no-cpu-baseline --ref-workloads 0 --mesh-cache /tmp/ab_mesh_$CFG.bin > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.log || exit $?
  (cd /tmp && export TMPDIR=/tmp && export $e && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/abprof_$v -o run -- \
    python3 $ROOT/bench.py --config $CFG --no-cpu-baseline --ref-workloads 0 --steps 2 --warmup 1 --mesh-cache /tmp/ab_mesh_$CFG.bin > $ROOT/gpurun_out/abprof_$v.json 2> $ROOT/gpurun_out/abprof_$v.log) || exit $?
done
python tools/ab_compare.py "${names[@]}"
