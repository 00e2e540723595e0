set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --config c1 --no-cpu-baseline > gpurun_out/bench_c1.json 2> gpurun_out/bench_c1.log && \
timeout -k 10 600 python bench.py --config c2 > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.log && \
cat gpurun_out/bench_c1.json gpurun_out/bench_c2.json
