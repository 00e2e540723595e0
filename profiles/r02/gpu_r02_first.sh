# Round-2 first look: smoke, then the default bench line (C2, with the CPU baseline).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 600 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.log
rc=$?
cat gpurun_out/smoke.log gpurun_out/bench_default.json
exit $rc
