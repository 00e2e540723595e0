"""Per-phase cycles of the single-workgroup AMG tail (k_amg_tail_blob) from a
diagnostic build: python tools/ab_variants.py st=CFD_TAIL_STAMPS=100, copy the
library into _lib/ab/, then on the GPU box
  CFD2_AMD_LIB=.../libcfd2_amd_st.so python tools/tail_stamps.py c1
Runs the bench workload's t = 0 step and one 5 x 30 step and prints the
s_memtime deltas of the 100th tail launch, phase by phase."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cfd-demo2_amd"))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from cfd2_amd import GpuSolver, default_config  # noqa: E402
from cfd2_amd._ffi import lib  # noqa: E402
from cfd2_amd.mesh import bench_channel  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c1"
mesh = bench_channel(bench.CONFIGS[cfg][0])
s = GpuSolver(mesh, config=default_config(fixed_outer=5, fixed_inner=30))
bench.setup_solver(s)
s.step()
s.step()
s.synchronize()
out = (C.c_uint32 * 64)()
f = lib().cfd_debug_tail_stamps
f.argtypes = [C.POINTER(C.c_uint32), C.c_int]
assert f(out, 64) == 0
n = out[0]
d = [int(out[q]) for q in range(1, min(n, 64))]
print(f"{cfg}: {n - 1} phases, {sum(d)} cycles: " + " ".join(map(str, d)))
