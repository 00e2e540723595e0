# Same-box A/B of runtime settings in alternating rounds: each argument is
# "name:ENV=V[,ENV=V]" (name:- for the defaults); ROUNDS (default 3) plain
# bench runs of every setting in turn (CFG, default c2), then one rocprofv3
# --kernel-trace --stats run per setting; prints ms/step and the level-0
# smoother time per run, the means, and the per-kernel table (ab_compare.py).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
CFG=${CFG:-c2}
ROUNDS=${ROUNDS:-3}
ROOT=$GRAFT_REPO_ROOT
names=()
for spec in "$@"; do names+=("${spec%%:*}"); rm -f gpurun_out/ab_${spec%%:*}_r*.json; done
for k in $(seq 1 $ROUNDS); do
  for spec in "$@"; do
    v=${spec%%:*}; envs=${spec#*:}; [ "$envs" = "-" ] && envs=""
    envarg=$(echo "$envs" | tr ',' ' ')
    env $envarg timeout -k 10 300 python bench.py --config $CFG --steps ${STEPS:-10} --no-cpu-baseline --ref-workloads 0 \
      --mesh-cache /tmp/ab_mesh_$CFG.bin > gpurun_out/ab_${v}_r$k.json 2> gpurun_out/ab_${v}_r$k.log || exit $?
    cp gpurun_out/ab_${v}_r$k.json gpurun_out/ab_$v.json
    python -c "import json,sys; d=json.load(open('gpurun_out/ab_${v}_r$k.json')); print(f'round $k ${v}: ms/step {d[\"ms_per_step\"]:.2f}  smoother {d[\"roofline\"][\"avg_launch_us\"]:.2f} us', flush=True)"
  done
done
python - "${names[@]}" <<'PY'
import json, statistics as st, sys, glob
for v in sys.argv[1:]:
    ms = [json.load(open(f))["ms_per_step"] for f in sorted(glob.glob(f"gpurun_out/ab_{v}_r*.json"))]
    print(f"mean {v:12s} ms/step {st.fmean(ms):.2f} ({min(ms):.2f}-{max(ms):.2f}, {len(ms)} runs)")
PY
for spec in "$@"; do
  v=${spec%%:*}; envs=${spec#*:}; [ "$envs" = "-" ] && envs=""
  envarg=$(echo "$envs" | tr ',' ' ')
  (cd /tmp && export TMPDIR=/tmp && { [ -z "$envarg" ] || export $envarg; } && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/abprof_$v -o run -- \
    python3 $ROOT/bench.py --config $CFG --no-cpu-baseline --ref-workloads 0 --steps 2 --warmup 1 --mesh-cache /tmp/ab_mesh_$CFG.bin > $ROOT/gpurun_out/abprof_$v.json 2> $ROOT/gpurun_out/abprof_$v.log) || exit $?
done
python tools/ab_compare.py "${names[@]}"
