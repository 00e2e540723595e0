# Round-2 evidence refresh on the current tree: GPU tests + smoke + default
# bench (C2, CPU baseline, reference workloads) + C1 line, then the per-step
# counter traffic / smoother PMC passes (tools/gpu_step_traffic.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_r02_final.sh || exit $?
bash tools/gpu_step_traffic.sh r02 c2
