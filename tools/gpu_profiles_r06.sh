# Round-6 evidence at the final sources: rocprofv3 kernel stats + PMC traffic
# of one whole step (FETCH_SIZE / WRITE_SIZE in separate passes) at C2 and C1,
# then the level-1 AMG residual's counters with the nontemporal bit 64 off /
# on (VERDICT r05 Next 4): FETCH / WRITE and the SQ wait fractions.
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_step_traffic.sh r06 c2 || exit $?
bash tools/gpu_step_traffic.sh r06 c1 || exit $?
ROOT=$GRAFT_REPO_ROOT
OUT=$ROOT/gpurun_out/nt64_r06
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
MC=$ROOT/gpurun_out/mesh_c2.bin
B="python3 $ROOT/bench.py --config c2 --no-cpu-baseline --ref-workloads 0 --mesh-cache $MC --steps 1 --warmup 1"
for m in 47 111; do
  export CFD_NT=$m
  timeout -s KILL 300 rocprofv3 --kernel-trace --kernel-include-regex k_amg_residual --output-format csv -d $OUT/nt$m/trace -o run -- $B > $OUT/nt$m.trace.json 2> $OUT/nt$m.trace.log || exit $?
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_amg_residual --output-format csv -d $OUT/nt$m/pmc_fetch -o run -- $B > $OUT/nt$m.fetch.json 2> $OUT/nt$m.fetch.log || exit $?
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_amg_residual --output-format csv -d $OUT/nt$m/pmc_write -o run -- $B > $OUT/nt$m.write.json 2> $OUT/nt$m.write.log || exit $?
  timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY --kernel-include-regex k_amg_residual --output-format csv -d $OUT/nt$m/pmc_sq -o run -- $B > $OUT/nt$m.sq.json 2> $OUT/nt$m.sq.log || exit $?
  unset CFD_NT
done
rm -f $MC
python3 $ROOT/tools/level1_residual_counters.py $OUT > $OUT/level1_residual_nt.txt
cat $OUT/level1_residual_nt.txt
