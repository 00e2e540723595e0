# Round 4: the single-workgroup tail's first level at C2 (24.6 us per V-cycle
# against 15.3 at C1): level sizes, then same-box A/B of CFD_AMG_TAIL_ROWS.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python - > gpurun_out/c2_levels.txt 2>&1 <<'PY' || exit 1
import sys; sys.path.insert(0, "cfd-demo2_amd")
import bench
from cfd2_amd import GpuSolver, default_config
from cfd2_amd.mesh import bench_channel, channel_obstacle_h
for cells in (1e6, 1e7):
    m = bench_channel(channel_obstacle_h(cells))
    s = GpuSolver(m, config=default_config(fixed_outer=1, fixed_inner=2))
    bench.setup_solver(s)
    s.step()
    print(int(cells), [r for r, _ in s.amg_levels()])
PY
cat gpurun_out/c2_levels.txt
CFG=c2 bash tools/gpu_ab_env.sh t4096=CFD_AMG_TAIL_ROWS=4096 t1024=CFD_AMG_TAIL_ROWS=1024 t16k=CFD_AMG_TAIL_ROWS=16384 t4096b=CFD_AMG_TAIL_ROWS=4096 t1024b=CFD_AMG_TAIL_ROWS=1024 > gpurun_out/ab_tail_c2.txt 2>&1 || exit $?
head -12 gpurun_out/ab_tail_c2.txt
grep -E "tail|resrestrict|k_amg_smooth<true, 1, true" gpurun_out/ab_tail_c2.txt
