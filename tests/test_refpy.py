"""The oracle pinned by a second, independently written restatement
(tests/refpy.py: numpy, written from the WGSL shaders and the Rust control
flow, not from oracle/oracle.cpp).  Both follow the reference's float32
operation order, so they must agree BIT FOR BIT -- per kernel (prepare /
assemble buffers of every scheme and time scheme) and over whole steps (fixed
schedule with lag 0, and the reference's natural schedule with the lag-1
readbacks) on the meshes of the reference's own solver tests
(amg_test / coupled_schemes_test, BackwardsStep h=0.05) and the C0 channel
(BASELINE configs[0]).  The north-star tolerance (relative L2 <= 1e-5) is
asserted first, the bit-exact bar after it."""
import numpy as np
import pytest

from cfd2_amd import default_config
from tests import refpy
from tests.meshes import backwards_step, bench_mesh, channel_obstacle
from tests.oracle_py import OracleSolver
from tests.test_oracle import setup_amg_test, setup_schemes_test


def _same(a, b, ctx):
    a, b = np.asarray(a), np.asarray(b)
    den = max(np.linalg.norm(b), 1e-30)
    assert np.linalg.norm(a - b) / den <= 1e-5, f"{ctx}: rel-L2 {np.linalg.norm(a - b) / den}"
    assert np.array_equal(a, b), f"{ctx}: not bit-exact (max diff {np.abs(a - b).max()})"


def _same_step(o, r, ctx):
    _same(o.get_u(), r.get_u(), f"{ctx} u")
    _same(o.get_p(), r.get_p(), f"{ctx} p")
    _same(o.get_d_p(), r.get_d_p(), f"{ctx} d_p")
    i = o.step_info()
    assert i.total_linear_iterations == r.info["total_iterations"], ctx
    assert i.outer_iterations == r.info["outer_iterations"], ctx
    assert np.float32(i.outer_residual_u) == np.float32(r.info["res_u"]), ctx
    assert np.float32(i.outer_residual_p) == np.float32(r.info["res_p"]), ctx
    assert np.float32(i.stats_p.residual) == np.float32(r.info["residual"]), ctx
    assert (i.degenerate_count, i.steady_state_count, bool(i.should_stop)) == (
        r.info["degenerate"], r.info["steady"], r.info["should_stop"]), ctx


@pytest.mark.parametrize("scheme,time_scheme", [(0, 0), (1, 0), (2, 0), (0, 1)])
def test_kernels_prepare_assemble(scheme, time_scheme):
    """prepare_coupled + coupled_assembly_merged, every output buffer: fluxes,
    gradients, d_p, coupled CSR values, rhs, scalar matrix, diagonal inverses
    (Upwind / SOU / QUICK deferred correction, Euler / BDF2, every boundary type)."""
    mesh = channel_obstacle()
    o = OracleSolver(mesh)
    r = refpy.RefSolver(mesh)
    rng = np.random.default_rng(11 + scheme + 3 * time_scheme)
    u0 = rng.uniform(-1, 1, size=(mesh.num_cells(), 2))
    u1 = rng.uniform(-1, 1, size=(mesh.num_cells(), 2))
    for s in (o, r):
        s.set_u(u1)
        s.initialize_history()  # old = old_old = u1 (BDF2 reads both)
        s.set_u(u0)
        s.set_dt(0.002)
        s.set_dt(0.003)  # dt_old = 0.002: a non-trivial BDF2 ratio
        s.set_scheme(scheme)
        s.set_time_scheme(time_scheme)
        c = s.constants
        c.time = 0.05  # inlet ramp active
        s.constants = c
    o.debug_prepare_assemble(False)
    M = r.M
    st, old = r.ring[r.i_state], r.ring[r.i_old]
    refpy.prepare(M, st, old, r.c)  # d_p / grad_p from the zero state
    o.debug_prepare_assemble(True)
    fl, gu, gv = refpy.prepare(M, st, old, r.c)  # Rhie-Chow with non-zero d_p / grad_p
    mv, rhs, sv, dui, dvi, dpi = refpy.assemble(M, st, old, r.ring[r.i_old_old], fl, gu, gv, r.c)
    ctx = f"scheme {scheme}/{time_scheme}"
    _same(o.debug_buffer(0), fl, f"{ctx} fluxes")
    _same(o.debug_buffer(1), gu.reshape(-1), f"{ctx} grad_u")
    _same(o.debug_buffer(2), gv.reshape(-1), f"{ctx} grad_v")
    _same(o.debug_buffer(10), st.grad_p.reshape(-1), f"{ctx} grad_p")
    _same(o.get_d_p(), st.d_p.astype(np.float64), f"{ctx} d_p")
    _same(o.debug_buffer(9), mv, f"{ctx} coupled matrix")
    _same(o.debug_buffer(3), rhs, f"{ctx} rhs")
    _same(o.debug_buffer(8), sv, f"{ctx} scalar matrix")
    _same(o.debug_buffer(5), dui, f"{ctx} diag_u_inv")
    _same(o.debug_buffer(7), dpi, f"{ctx} diag_p_inv")


@pytest.mark.parametrize("precond", [0, 1])
def test_fixed_schedule_steps(precond):
    """tests/amg_test.rs setup, 3 steps of 3 Picard x 10 FGMRES (lag 0): Schur
    prediction / Jacobi relaxation or one AMG V-cycle / correction, CGS +
    Givens, triangular solve, under-relaxation: fields and step statistics."""
    mesh = backwards_step()
    cfg = dict(convergence_lag=0, fixed_outer=3, fixed_inner=10)
    o = OracleSolver(mesh, config=default_config(**cfg))
    r = refpy.RefSolver(mesh, **cfg)
    for s in (o, r):
        setup_amg_test(s, mesh, precond)
    for k in range(3):
        o.step()
        r.step()
        _same_step(o, r, f"precond {precond} step {k}")
    if precond == 1:
        assert o.amg_levels() == r.amg.sizes()


@pytest.mark.parametrize("precond", [0, 1])
def test_natural_schedule_amg_test(precond):
    """tests/amg_test.rs itself: natural convergence (lagged FGMRES and outer
    checks, restarts, stagnation), 5 steps; then the reference's assertion
    0 < max|p| < 1000 (amg_test.rs:84-86)."""
    mesh = backwards_step()
    o = OracleSolver(mesh)
    r = refpy.RefSolver(mesh)
    for s in (o, r):
        setup_amg_test(s, mesh, precond)
    for k in range(5):
        o.step()
        r.step()
        _same_step(o, r, f"amg_test precond {precond} step {k}")
    assert 0.0 < np.abs(r.get_p()).max() < 1000.0


@pytest.mark.parametrize("scheme,time_scheme", [(0, 0), (1, 0), (2, 0), (0, 1)])
def test_coupled_schemes_steps(scheme, time_scheme):
    """tests/coupled_schemes_test.rs: 2 natural steps per scheme; finite fields."""
    mesh = backwards_step()
    o = OracleSolver(mesh)
    r = refpy.RefSolver(mesh)
    for s in (o, r):
        setup_schemes_test(s, mesh, scheme, time_scheme)
    for k in range(2):
        o.step()
        r.step()
        _same_step(o, r, f"schemes {scheme}/{time_scheme} step {k}")
    assert np.all(np.isfinite(r.get_u())) and np.all(np.isfinite(r.get_p()))


@pytest.mark.parametrize("kind", ["voronoi", "cutcell"])
def test_c0_channel_fixed_schedule(kind):
    """BASELINE configs[0] (~10 k Voronoi cells, channel + obstacle, bench
    physics; also its cut-cell counterpart), AMG: two steps of 2 Picard x 8
    FGMRES, inlet on."""
    if kind == "voronoi":
        from cfd2_amd.mesh import bench_voronoi_channel
        mesh = bench_voronoi_channel()
    else:
        mesh = bench_mesh(0.0172, 100)
    assert 9000 < mesh.num_cells() < 11000
    cfg = dict(convergence_lag=0, fixed_outer=2, fixed_inner=8)
    o = OracleSolver(mesh, config=default_config(**cfg))
    r = refpy.RefSolver(mesh, **cfg)
    for s in (o, r):
        s.set_dt(1e-3)
        s.set_viscosity(0.01)
        s.set_density(1.0)
        s.set_alpha_u(0.7)
        s.set_alpha_p(0.3)
        s.set_precond_type(1)
        s.initialize_history()
        c = s.constants
        c.time = 0.05
        s.constants = c
    for k in range(2):
        o.step()
        r.step()
        _same_step(o, r, f"C0 step {k}")


def test_divergence_like_reference():
    """A NaN velocity (set_u clobbers the state, solver.rs:9-21) reaches the
    linear residual: both restatements stop at the same step with the
    reference's panic message (coupled_solver.rs:344-346)."""
    mesh = backwards_step()
    o = OracleSolver(mesh)
    r = refpy.RefSolver(mesh)
    u = np.zeros((mesh.num_cells(), 2))
    u[7, 0] = np.nan
    for s in (o, r):
        setup_amg_test(s, mesh, 1)
        s.set_u(u)
    with pytest.raises(RuntimeError, match="Diverged: NaN detected in linear residual"):
        o.step()
    with pytest.raises(FloatingPointError, match="Diverged: NaN detected in linear residual"):
        r.step()
