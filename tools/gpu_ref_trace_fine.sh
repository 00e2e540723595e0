# The reference's fine_mesh criterion workload (1.06 M cells, AMG, natural
# convergence) under a kernel trace: GPU busy vs span per step.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ref_fm -o run -- \
  python3 $R/tools/ref_workload_run.py fine_mesh > $R/gpurun_out/ref_fm.json 2> $R/gpurun_out/ref_fm.log && \
python3 $R/tools/trace_steps.py $R/gpurun_out/ref_fm > $R/gpurun_out/ref_fm_steps.txt && \
python3 $R/tools/summarize_stats.py $R/gpurun_out/ref_fm > $R/gpurun_out/ref_fm_top.txt
cut -c1-400 $R/gpurun_out/ref_fm.json
head -12 $R/gpurun_out/ref_fm_steps.txt
head -20 $R/gpurun_out/ref_fm_top.txt
