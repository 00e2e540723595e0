set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --config c1 --ref-workloads 0 --no-cpu-baseline > gpurun_out/r4_base_c1.json 2> gpurun_out/r4_base_c1.log || exit $?
timeout -k 10 400 python -u bench.py --ref-workloads 0 --no-cpu-baseline > gpurun_out/r4_base_c2.json 2> gpurun_out/r4_base_c2.log || exit $?
cat gpurun_out/r4_base_c1.json gpurun_out/r4_base_c2.json
