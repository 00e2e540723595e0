# Round-6 same-box A/B at C2 (VERDICT r05 Next 3 + 4): alternating plain bench
# runs of each variant, ROUNDS times; per run ms/step and the level-0 smoother's
# HIP-event launch time.  Variants (tools/ab_r06_build.py):
#   base    in-tree library (round-5 kernels + round-6 host changes)
#   r04     abtrees/r04 (the BENCH_r04 head, its own bench.py / package)
#   nokpre  base without kernarg preload
#   nohead  base with the smoother's leading-argument change reverted
#   nt64    base with CFD_NT=111 (the level-1 residual nontemporal too)
#   phead   base with the Schur prediction's first-needed fields and grid size
#           as leading (preloaded) arguments (/tmp patch, tools/gpu_ab_phead.sh)
# Usage: bash tools/gpu_ab_r06_regression.sh [variants...]
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
CFG=${CFG:-c2}
ROUNDS=${ROUNDS:-3}
VARS=${*:-base r04 nokpre nohead nt64}
for k in $(seq 1 $ROUNDS); do
  for v in $VARS; do
    bench=$R/bench.py; lib=$R/cfd-demo2_amd/cfd2_amd/_lib/libcfd2_amd.so; extra=""
    case $v in
      r04) bench=$R/abtrees/r04/bench.py; lib=$R/abtrees/r04/cfd-demo2_amd/cfd2_amd/_lib/libcfd2_amd.so ;;
      nokpre|nohead|phead) lib=$R/cfd-demo2_amd/cfd2_amd/_lib/ab/libcfd2_amd_$v.so ;;
      nt64) extra="CFD_NT=111" ;;
    esac
    env $extra CFD2_AMD_LIB=$lib timeout -k 10 300 python $bench --config $CFG --steps ${STEPS:-10} --no-cpu-baseline \
      --ref-workloads 0 --mesh-cache /tmp/ab_mesh_$CFG.bin > gpurun_out/abr_${v}_$k.json 2> gpurun_out/abr_${v}_$k.log || exit $?
    python - "$v" "$k" <<'PY'
import json, sys
v, k = sys.argv[1:]
d = json.load(open(f"gpurun_out/abr_{v}_{k}.json"))
print(f"round {k} {v:8s} ms/step {d['ms_per_step']:8.2f}  level-0 smoother {d['roofline']['avg_launch_us']:6.2f} us  build {d.get('build_id')}", flush=True)
PY
  done
done
