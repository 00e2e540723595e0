"""HIP kernels vs the REFERENCE'S OWN SHADERS (tests/golden/wgsl_ref.npz).

prepare_coupled.wgsl + coupled_assembly_merged.wgsl, executed on the CPU from
the reference's source (tests/golden/make_wgsl_golden.py, schedule B: the
whole dispatch resident -- prepare's neighbour reads see the pre-kernel
state), on a random state for every scheme / time scheme: k_prepare and
k_assemble through the C ABI must give the same bits in every output buffer
(fluxes, gradients, d_p, the coupled CSR values in the reference's order, rhs,
the scalar pressure matrix, the diagonal inverses).  No oracle in between."""
import os

import numpy as np
import pytest

from cfd2_amd import GpuSolver
from tests.meshes import channel_obstacle

pytestmark = pytest.mark.gpu
FIX = os.path.join(os.path.dirname(__file__), "golden", "wgsl_ref.npz")
F = np.float32


@pytest.mark.parametrize("scheme,time_scheme", [(0, 0), (1, 0), (2, 0), (0, 1)])
def test_hip_kernels_equal_reference_shaders(scheme, time_scheme):
    mesh = channel_obstacle()
    g = GpuSolver(mesh)
    rng = np.random.default_rng(11 + scheme + 3 * time_scheme)
    u0 = rng.uniform(-1, 1, size=(mesh.num_cells(), 2))
    u1 = rng.uniform(-1, 1, size=(mesh.num_cells(), 2))
    g.set_u(u1)
    g.initialize_history()
    g.set_u(u0)
    g.set_dt(0.002)
    g.set_dt(0.003)
    g.set_scheme(scheme)
    g.set_time_scheme(time_scheme)
    c = g.constants
    c.time = 0.05
    g.constants = c
    g.debug_prepare_assemble(False)
    g.debug_prepare_assemble(True)
    got = dict(fluxes=g.debug_buffer(0), grad_u=g.debug_buffer(1), grad_v=g.debug_buffer(2),
               rhs=g.debug_buffer(3), diag_u_inv=g.debug_buffer(5), diag_v_inv=g.debug_buffer(6),
               diag_p_inv=g.debug_buffer(7), scalar_matrix=g.debug_buffer(8), matrix=g.debug_buffer(9),
               grad_p=g.debug_buffer(10), d_p=g.get_d_p().astype(F))
    key = f"kernels_s{scheme}t{time_scheme}"
    with np.load(FIX) as z:
        for k, v in got.items():
            ref = z[f"{key}/{k}"]
            assert v.shape == ref.shape, k
            assert np.array_equal(v, ref), f"{key} {k}: max diff {np.abs(v - ref).max()}"
