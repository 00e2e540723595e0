# The reference's own criterion workloads alone (no profiler), then the
# small one (solver_step) under a kernel trace: GPU busy vs span per step.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 $R/tools/ref_workload_run.py all > $R/gpurun_out/ref_all.json 2> $R/gpurun_out/ref_all.log && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ref_ss -o run -- \
  python3 $R/tools/ref_workload_run.py solver_step > $R/gpurun_out/ref_ss.json 2> $R/gpurun_out/ref_ss.log && \
python3 $R/tools/trace_steps.py $R/gpurun_out/ref_ss > $R/gpurun_out/ref_ss_steps.txt && \
python3 $R/tools/summarize_stats.py $R/gpurun_out/ref_ss > $R/gpurun_out/ref_ss_top.txt
cut -c1-600 $R/gpurun_out/ref_all.json
head -8 $R/gpurun_out/ref_ss_steps.txt
