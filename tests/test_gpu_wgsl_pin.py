"""The HIP path vs the REFERENCE'S OWN SHADERS (tests/golden/wgsl_ref.npz).

prepare_coupled.wgsl + coupled_assembly_merged.wgsl, executed on the CPU from
the reference's source (tests/golden/make_wgsl_golden.py, schedule B: the
whole dispatch resident -- prepare's neighbour reads see the pre-kernel
state), on a random state for every scheme / time scheme: k_prepare and
k_assemble through the C ABI must give the same bits in every output buffer
(fluxes, gradients, d_p, the coupled CSR values in the reference's order, rhs,
the scalar pressure matrix, the diagonal inverses).  No oracle in between.

Whole steps: with cfd_debug_reference_semantics(4) the HIP path sums like the
reference (64-DOF workgroup trees, serial / strided finishing sums, serial
f64 check_evolution) and must then give, step by step, the bits of the
reference's shaders under schedule B -- again with no oracle in between."""
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


def _gpu_cases():
    """(case, mode) of the fixture: A (flags 15), B (flags 4), C (flags 13)"""
    from tests.golden.make_wgsl_golden import cases
    return [(c[0], m) for c in cases() for m in c[5]]


@pytest.mark.parametrize("name,mode", _gpu_cases())
def test_hip_reference_semantics_equal_reference_kernels(name, mode):
    """Whole steps: the HIP path in the reference-semantics test mode
    (cfd_debug_reference_semantics with the mode's oracle flags: 4 -- the
    reference's reduction order; 13 -- also the in-place AMG smoother with
    its workgroups in order and restrict_residual's clamped rows; 15 -- also
    prepare's racy reads with its workgroups in order) == the reference's
    eight shaders run under the mode's schedule (fixture B: the whole
    dispatch resident; C: the V-cycle's workgroups in order; A: every
    dispatch's workgroups in order), bit for
    bit at every step -- fields (SHA-256 of the f32 bytes), FGMRES iteration
    counts, outer residuals, the linear residual and the stop counters -- on
    the reference's own tests (amg_test, coupled_schemes), the fixed 3 x 10
    schedule and the 10 k-cell Voronoi channel (BASELINE configs[0])."""
    from cfd2_amd import default_config
    from tests.golden.make_wgsl_golden import MODES, cases, digest, info_vec
    _, mk, setup, kw, steps, _ = [c for c in cases() if c[0] == name][0]
    mesh = mk()
    g = GpuSolver(mesh, config=default_config(**kw))
    g.debug_reference_semantics(MODES[mode][2])
    setup(g, mesh)
    with np.load(FIX) as z:
        for k in range(steps):
            g.step()
            assert digest(g) == str(z[f"{name}/{mode}/digests"][k]), f"{name}/{mode} step {k}: fields differ"
            np.testing.assert_array_equal(info_vec(g), z[f"{name}/{mode}/info"][k], err_msg=f"{name}/{mode} step {k}")


@pytest.mark.parametrize("flags", [1, 2, 3, 6, 8, 9, 12, 13, 15])
def test_hip_reference_semantics_equal_oracle(flags):
    """every combination the GPU offers == the oracle with the same flags
    (amg_test setup, AMG, 2 steps of 2 x 5)"""
    from cfd2_amd import default_config
    from tests.golden.make_wgsl_golden import digest, info_vec
    from tests.meshes import backwards_step
    from tests.oracle_py import OracleSolver
    from tests.test_oracle import setup_amg_test
    mesh = backwards_step()
    kw = dict(convergence_lag=0, fixed_outer=2, fixed_inner=5)
    g = GpuSolver(mesh, config=default_config(**kw))
    o = OracleSolver(mesh, config=default_config(**kw))
    g.debug_reference_semantics(flags)
    o.set_semantics(flags)
    for s in (g, o):
        setup_amg_test(s, mesh, 1)
    for k in range(2):
        for s in (g, o):
            s.step()
        assert digest(g) == digest(o), (flags, k)
        np.testing.assert_array_equal(info_vec(g), info_vec(o))


def test_reference_semantics_refuses_what_the_gpu_lacks():
    from tests.meshes import backwards_step
    g = GpuSolver(backwards_step())
    for bad in (16, 17, 32, 31):
        with pytest.raises(Exception):
            g.debug_reference_semantics(bad)


def test_reference_order_switches_back_to_canonical():
    """the canonical mode stays the default; switching back restores it"""
    from tests.meshes import backwards_step
    from tests.oracle_py import OracleSolver
    from tests.test_oracle import setup_amg_test
    mesh = backwards_step()
    g = GpuSolver(mesh)
    o = OracleSolver(mesh)
    for s in (g, o):
        setup_amg_test(s, mesh, 1)
    g.debug_reference_semantics(13)
    g.debug_reference_semantics(0)
    for s in (g, o):
        s.step()
    assert np.array_equal(g.get_p(), o.get_p()) and np.array_equal(g.get_u(), o.get_u())


def test_hip_reference_order_equals_reference_kernels_c1():
    """BASELINE configs[1] scale: the C1-only kernel forms (the paired AMG
    levels down and up, the blob tail, 16-bit ELL levels, the nontemporal
    variants) in the reference reduction order == the reference's kernels
    (tests/golden/wgsl_ref_c1.npz) at every step"""
    from cfd2_amd import default_config
    from tests.golden.make_wgsl_golden import C1, digest, info_vec
    name, mk, setup, kw, steps = C1
    mesh = mk()
    g = GpuSolver(mesh, config=default_config(**kw))
    g.debug_reference_semantics(4)
    setup(g, mesh)
    with np.load(os.path.join(os.path.dirname(__file__), "golden", "wgsl_ref_c1.npz")) as z:
        for k in range(steps):
            g.step()
            assert digest(g) == str(z[f"{name}/B/digests"][k]), f"C1 step {k}"
            np.testing.assert_array_equal(info_vec(g), z[f"{name}/B/info"][k], err_msg=f"C1 step {k}")
