"""BASELINE configs[2] (the 10 M-cell bench mesh) bit-exact against the
oracle: the production-size hierarchy (predicated MODE-0 coarse levels, the
full tail), every kernel at its real grid size.  ~25 s (the oracle steps
10 M cells on 16 host threads); CFD_C2_PARITY=0 skips it."""
import os

import numpy as np
import pytest

from cfd2_amd import GpuSolver, default_config
from tests.meshes import bench_mesh
from tests.oracle_py import OracleSolver, olib
from tests.test_gpu_parity import _assert_same_fields, _assert_same_info

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(os.environ.get("CFD_C2_PARITY") == "0",
                                                  reason="CFD_C2_PARITY=0")]


def test_c2_one_step_bitexact():
    olib().oracle_set_threads(min(16, os.cpu_count() or 1))
    mesh = bench_mesh(5.449e-4, 100)
    assert mesh.num_cells() > 9_000_000
    cfg = dict(fixed_outer=2, fixed_inner=6)
    g = GpuSolver(mesh, config=default_config(**cfg))
    o = OracleSolver(mesh, config=default_config(**cfg))
    for s in (g, o):
        s.set_dt(1e-3)
        s.set_viscosity(0.01)
        s.set_density(1.0)
        s.set_alpha_u(0.7)
        s.set_alpha_p(0.3)
        s.set_precond_type(1)
        s.initialize_history()
        c = s.constants
        c.time = 0.05  # inlet on: the first step solves
        s.constants = c
    g.step()
    o.step()
    _assert_same_fields(g, o, "C2 step 0")
    _assert_same_info(g, o, "C2 step 0")
    assert g.amg_levels() == o.amg_levels()
    assert np.abs(g.get_u()).max() > 0.1
