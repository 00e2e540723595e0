# The driver's multi-process launch of bench.py (one process per rank,
# torch.distributed.run) rehearsed on one GPU with the host-staged transport:
# exercises the --gpus N line end to end, comm-timing table included.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
CFD_DIST_TRANSPORT=host CFD_BENCH_DEVICE=0 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --config c1 --steps 2 --warmup 1 \
  > gpurun_out/bench_mp2_host_c1.json 2> gpurun_out/bench_mp2_host_c1.log || exit $?
cat gpurun_out/bench_mp2_host_c1.json
