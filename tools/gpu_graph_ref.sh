# Round 5: hipGraph replay on the reference's own criterion workloads (natural
# convergence schedule: the host reads a residual every FGMRES iteration),
# alternating eager / graph runs on one box.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for k in 1 2; do
  for g in 0 1; do
    CFD_GRAPH=$g timeout -k 10 400 python -u tools/ref_workload_run.py all > gpurun_out/refwl_g${g}_$k.json 2> gpurun_out/refwl_g${g}_$k.log || exit $?
    python -c "
import json; d=json.load(open('gpurun_out/refwl_g${g}_$k.json'))
print('graph=$g run $k', {w: (round(v['ms_per_step'], 3), sum(v['fgmres_iterations_per_step'])) for w, v in d.items()})"
  done
done
