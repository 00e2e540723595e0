# Same-box A/B of library variants with per-kernel times: each variant runs
# bench (CFG, default c2) once plain (ms/step) and once under rocprofv3
# --kernel-trace --stats; tools/ab_compare.py prints the per-kernel table.
# Variant libraries: cfd-demo2_amd/cfd2_amd/_lib/ab/libcfd2_amd_<name>.so
# (tools/ab_variants.py builds them under _lib/variants/, which never travels;
# copy the ones to compare into _lib/ab/ for the run and delete them after);
# "base" is the in-tree library.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
CFG=${CFG:-c2}
ROOT=$GRAFT_REPO_ROOT
for v in "$@"; do
  if [ "$v" = base ]; then lib=$ROOT/cfd-demo2_amd/cfd2_amd/_lib/libcfd2_amd.so; else lib=$ROOT/cfd-demo2_amd/cfd2_amd/_lib/ab/libcfd2_amd_$v.so; fi
  CFD2_AMD_LIB=$lib timeout -k 10 300 python bench.py --config $CFG --steps ${STEPS:-10} --no-cpu-baseline --ref-workloads 0 --mesh-cache /tmp/ab_mesh_$CFG.bin > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.log || exit $?
  (cd /tmp && export TMPDIR=/tmp && CFD2_AMD_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/abprof_$v -o run -- \
    python3 $ROOT/bench.py --config $CFG --no-cpu-baseline --ref-workloads 0 --steps 2 --warmup 1 --mesh-cache /tmp/ab_mesh_$CFG.bin > $ROOT/gpurun_out/abprof_$v.json 2> $ROOT/gpurun_out/abprof_$v.log) || exit $?
done
python tools/ab_compare.py "$@"
