"""Jacobi-path relaxation at C1 scale (1.0 M cells, BASELINE configs[1] mesh):
one GpuSolver with one-row-per-thread sweeps (CFD_RELAX4=0) and one with the
4-rows-per-thread kernel, 2 steps of 1 Picard x 3 FGMRES iterations each
(199 sweeps per preconditioner application); asserts identical fields and
prints wall times.  Run under rocprofv3 --kernel-trace --stats for per-sweep
kernel times."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cfd-demo2_amd"))
import numpy as np  # noqa: E402
from cfd2_amd import GpuSolver, default_config  # noqa: E402
from cfd2_amd.mesh import bench_channel  # noqa: E402

mesh = bench_channel(0.001723, 100)
out = {}
for flag in ("0", "1"):
    os.environ["CFD_RELAX4"] = flag
    s = GpuSolver(mesh, config=default_config(fixed_outer=1, fixed_inner=3))
    s.set_dt(1e-3)
    s.set_viscosity(0.01)
    s.set_alpha_p(0.3)
    s.set_alpha_u(0.7)
    a = mesh.arrays()
    u = np.zeros((mesh.num_cells(), 2))
    u[np.asarray(a["cell_cx"]) < 0.02, 0] = 1.0
    s.set_u(u)
    s.initialize_history()
    s.set_precond_type(0)
    s.step()
    s.synchronize()
    t0 = time.perf_counter()
    s.step()
    s.synchronize()
    out[flag] = (np.asarray(s.get_u()), np.asarray(s.get_p()), time.perf_counter() - t0)
    s.close()
(u0, p0, t0), (u1, p1, t1) = out["0"], out["1"]
assert np.array_equal(u0, u1) and np.array_equal(p0, p1), "relax kernels differ"
print(f"{mesh.num_cells()} cells: step with 1-row sweeps {t0 * 1e3:.1f} ms, 4-row sweeps {t1 * 1e3:.1f} ms; fields identical")
