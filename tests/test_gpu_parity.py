"""HIP path vs CPU oracle (tests/oracle_py.py) through the C ABI.

Parity bar: the HIP kernels reproduce the oracle's f32 arithmetic operation
for operation (-ffp-contract=off, canonical reduction order), so fields,
matrices and step statistics must be BIT-EXACT (np.array_equal).  North-star
tolerance (fields within 1e-5 relative) is checked as well, as a weaker bound.
"""
import numpy as np
import pytest

from cfd2_amd import GpuSolver, default_config
from tests.meshes import backwards_step, bench_mesh, channel_obstacle
from tests.oracle_py import OracleSolver

pytestmark = pytest.mark.gpu

DEBUG_IDS = list(range(13))


def _pair(mesh, **cfg):
    c = default_config(**cfg)
    return GpuSolver(mesh, config=c), OracleSolver(mesh, config=default_config(**cfg))


def _setup_amg_test(s, mesh, precond):
    """tests/amg_test.rs:22-43."""
    s.set_dt(0.001)
    s.set_viscosity(0.001)
    s.set_density(1.0)
    s.set_alpha_p(0.3)
    s.set_alpha_u(0.7)
    s.set_scheme(0)
    a = mesh.arrays()
    u = np.zeros((mesh.num_cells(), 2))
    u[(a["cell_cx"] < 0.05) & (a["cell_cy"] > 0.5), 0] = 1.0
    s.set_u(u)
    s.initialize_history()
    s.set_precond_type(precond)


def _setup_schemes_test(s, mesh, scheme, time_scheme):
    """tests/coupled_schemes_test.rs:28-49 (set_u then set_p zeroes u; dt written directly)."""
    n = mesh.num_cells()
    s.set_u(np.tile([0.1, 0.0], (n, 1)))
    s.set_p(np.zeros(n))
    c = s.constants
    c.dt = 0.001
    s.constants = c
    s.set_density(1.0)
    s.set_viscosity(0.01)
    s.set_alpha_u(0.9)
    s.set_alpha_p(0.9)
    s.set_scheme(scheme)
    s.set_time_scheme(time_scheme)
    s.update_constants()


def _assert_same_fields(g, o, ctx=""):
    ug, uo = g.get_u(), o.get_u()
    pg, po = g.get_p(), o.get_p()
    dg, do = g.get_d_p(), o.get_d_p()
    assert np.all(np.isfinite(ug)) and np.all(np.isfinite(pg)), ctx
    # north-star tolerance first (informative), then the bit-exact bar
    for a, b, name in ((ug, uo, "u"), (pg, po, "p"), (dg, do, "d_p")):
        den = max(np.linalg.norm(b), 1e-30)
        assert np.linalg.norm(a - b) / den <= 1e-5, f"{ctx} {name} rel-L2 > 1e-5"
        assert np.array_equal(a, b), f"{ctx} {name} not bit-exact (max diff {np.abs(a - b).max()})"


def _assert_same_info(g, o, ctx=""):
    ig, io = g.step_info(), o.step_info()
    for f in ("should_stop", "degenerate_count", "steady_state_count", "outer_iterations",
              "total_linear_iterations"):
        assert getattr(ig, f) == getattr(io, f), f"{ctx} step_info.{f}: {getattr(ig, f)} vs {getattr(io, f)}"
    assert ig.outer_residual_u == io.outer_residual_u, ctx
    assert ig.outer_residual_p == io.outer_residual_p, ctx
    assert ig.stats_p.iterations == io.stats_p.iterations, ctx
    assert ig.stats_p.residual == io.stats_p.residual, ctx


@pytest.mark.parametrize("scheme,time_scheme", [(0, 0), (1, 0), (2, 0), (0, 1)])
def test_prepare_assemble_kernels_bitexact(scheme, time_scheme):
    """prepare_coupled + coupled_assembly_merged: every output buffer bit-exact."""
    mesh = channel_obstacle()
    g, o = _pair(mesh)
    rng = np.random.default_rng(1234)
    u0 = rng.uniform(-1, 1, size=(mesh.num_cells(), 2))
    for s in (g, o):
        s.set_u(u0)
        s.initialize_history()
        s.set_dt(0.002)
        s.set_scheme(scheme)
        s.set_time_scheme(time_scheme)
        c = s.constants
        c.time = 0.05  # inlet ramp active
        s.constants = c
        s.debug_prepare_assemble(False)  # d_p / grad_p from the zero state
        s.debug_prepare_assemble(True)   # Rhie-Chow with non-zero d_p / grad_p
    for bid in DEBUG_IDS:
        a, b = g.debug_buffer(bid), o.debug_buffer(bid)
        assert a.shape == b.shape, bid
        assert np.all(np.isfinite(a)), bid
        assert np.array_equal(a, b), f"debug buffer {bid}: max diff {np.abs(a - b).max()}"


@pytest.mark.parametrize("precond", [0, 1])
def test_amg_test_parity_and_bounds(precond):
    """tests/amg_test.rs: 5 steps; 0 < max|p| < 1000; GPU == oracle bit-exact each step."""
    mesh = backwards_step()
    g, o = _pair(mesh)
    for s in (g, o):
        _setup_amg_test(s, mesh, precond)
    for k in range(5):
        g.step()
        o.step()
        _assert_same_fields(g, o, f"step {k}")
        _assert_same_info(g, o, f"step {k}")
    max_p = np.abs(g.get_p()).max()
    assert 0.0 < max_p < 1000.0
    if precond == 1:
        assert g.amg_levels() == o.amg_levels()


@pytest.mark.parametrize("scheme,time_scheme", [(0, 0), (1, 0), (2, 0), (0, 1)])
def test_coupled_schemes_parity(scheme, time_scheme):
    """tests/coupled_schemes_test.rs: 2 steps per scheme, all fields finite, GPU == oracle."""
    mesh = backwards_step()
    g, o = _pair(mesh)
    for s in (g, o):
        _setup_schemes_test(s, mesh, scheme, time_scheme)
    for k in range(2):
        g.step()
        o.step()
        _assert_same_fields(g, o, f"scheme {scheme}/{time_scheme} step {k}")
        _assert_same_info(g, o)


def test_divergence_channel_obstacle_gpu():
    """tests/gpu_divergence_test.rs:6-92 at its own length: up to 200 adaptive
    steps (CFL 0.5 on the 0.025 cell size, dt clamped to [1e-5, 0.1]) with the
    should_stop break, max|u| <= 20 checked every 10 steps as the reference
    does -- and GPU == oracle bit-exact after every step (same host-side dt
    sequence: both solvers' dt comes from the GPU's velocities, which equal
    the oracle's)."""
    mesh = channel_obstacle()
    g, o = _pair(mesh)
    a = mesh.arrays()
    u = np.zeros((mesh.num_cells(), 2))
    u[a["cell_cx"] < 0.025, 0] = 1.0
    for s in (g, o):
        s.set_dt(0.01)
        s.set_viscosity(0.01)
        s.set_density(1.0)
        s.set_scheme(0)
        s.set_u(u)
    steps = 0
    for step in range(200):
        uu = g.get_u()
        vmax = float(np.sqrt((uu ** 2).sum(1)).max())
        if vmax > 1e-6:
            dt = float(np.clip(0.5 * 0.025 / vmax, 1e-5, 0.1))
            g.set_dt(dt)
            o.set_dt(dt)
        g.step()
        o.step()
        steps += 1
        _assert_same_fields(g, o, f"gpu_divergence_test step {step}")
        _assert_same_info(g, o, f"gpu_divergence_test step {step}")
        if g.should_stop:
            assert g.degenerate_count <= 10, "Solver stopped due to degenerate solution!"
            break
        if step % 10 == 0:
            assert vmax <= 20.0 and np.isfinite(vmax), f"Divergence detected at step {step}"
    assert steps >= 10


@pytest.mark.parametrize("lag", [0, 1])
def test_fixed_schedule_and_lag_parity(lag):
    """Fixed benchmark schedule (K outer x M inner) and both lag models: bit-exact."""
    mesh = channel_obstacle(h=0.03)
    for cfg in (dict(fixed_outer=3, fixed_inner=12, convergence_lag=lag),
                dict(convergence_lag=lag)):
        g, o = _pair(mesh, **cfg)
        for s in (g, o):
            _setup_amg_test(s, mesh, 1)
        for k in range(3):
            g.step()
            o.step()
            _assert_same_fields(g, o, f"{cfg} step {k}")
            _assert_same_info(g, o, f"{cfg} step {k}")


def test_bench_geometry_parity_medium():
    """SURVEY §8(d) geometry at ~100k cells, fixed schedule, AMG: one step bit-exact."""
    mesh = bench_mesh(0.0055, 30)
    g, o = _pair(mesh, fixed_outer=2, fixed_inner=8)
    for s in (g, o):
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
    g.step()
    o.step()
    _assert_same_fields(g, o, "bench geometry")
    assert g.amg_levels() == o.amg_levels()


@pytest.mark.parametrize("name", ["schemes", "amg"])
def test_golden_fixtures_gpu(name):
    """HIP path reproduces the committed golden vectors (tests/golden) bit-for-bit."""
    import os
    from tests.golden.make_golden import run_case
    ref = np.load(os.path.join(os.path.dirname(__file__), "golden", f"{name}.npz"), allow_pickle=False)
    got = run_case(name, GpuSolver)
    for k in ref.files:
        assert np.array_equal(ref[k], got[k]), k


@pytest.mark.parametrize("n", [1, 2, 7, 130])
@pytest.mark.parametrize("precond", [0, 1])
def test_tiny_strips_parity(n, precond):
    """Degenerate sizes (single cell, 1-D strips; 130 cells = two AMG levels):
    GPU == oracle bit-exact, including padded 4-row groups at the end."""
    from tests.synthetic import strip
    m = strip(n)
    g, o = GpuSolver(m), OracleSolver(m)
    for s in (g, o):
        s.set_dt(0.01)
        s.set_viscosity(0.01)
        s.set_density(1.0)
        s.set_precond_type(precond)
        s.initialize_history()
        c = s.constants
        c.time = 0.1
        s.constants = c
    for k in range(3):
        g.step()
        o.step()
        _assert_same_fields(g, o, f"strip {n} step {k}")
        _assert_same_info(g, o, f"strip {n} step {k}")


def test_c1_scale_parity_and_true_residual():
    """BASELINE configs[1] scale (~1M cells, bench geometry and physics), fixed
    schedule 1 x 6: GPU == oracle bit-exact after the t = 0 step and one real
    step; and the solver's x satisfies the assembled system to its reported
    residual (f64 recomputation with scipy, size-independent check)."""
    sp = pytest.importorskip("scipy.sparse")
    from tests import numpy_ref
    mesh = bench_mesh(0.001723, 100)
    assert abs(mesh.num_cells() - 1.0e6) / 1.0e6 < 0.03
    cfg = dict(fixed_outer=1, fixed_inner=6, convergence_lag=0)
    g, o = _pair(mesh, **cfg)
    for s in (g, o):
        s.set_dt(1e-3)
        s.set_viscosity(0.01)
        s.set_density(1.0)
        s.set_alpha_u(0.7)
        s.set_alpha_p(0.3)
        s.set_precond_type(1)
        s.initialize_history()
    for k in range(2):
        g.step()
        o.step()
        _assert_same_fields(g, o, f"C1 step {k}")
        _assert_same_info(g, o, f"C1 step {k}")
    # true residual of the assembled system (f64) vs the solver's own final residual
    ig = g.step_info().stats_p
    rhs = g.debug_buffer(3).astype(np.float64)
    x = g.debug_buffer(4).astype(np.float64)
    vals = g.debug_buffer(9).astype(np.float64)
    A = _coupled_csr(mesh, vals)
    r = np.linalg.norm(rhs - A @ x)
    assert np.isfinite(r) and r <= 1e-3 * np.linalg.norm(rhs) + 2 * ig.residual, (r, ig.residual)


def _coupled_csr(mesh, vals):
    """Reference coupled CSR (init/linear_solver/mod.rs:180-216) as scipy from the
    scalar pattern: block row i holds sub-rows u, v, p, each listing
    (3j, 3j+1, 3j+2) for the neighbours j of i in ascending order."""
    import scipy.sparse as sp
    srow, scol = _scalar_csr_fast(mesh)
    n = len(srow) - 1
    deg = np.diff(srow)
    base3 = (3 * scol[:, None] + np.arange(3)[None, :]).reshape(-1)
    pos = np.arange(9 * len(scol))
    row = np.repeat(np.arange(n), 9 * deg)
    off = pos - 9 * srow[row]
    sub = off // (3 * deg[row])
    cols = base3[3 * srow[row] + off % (3 * deg[row])]
    return sp.csr_matrix((vals, (3 * row + sub, cols)), shape=(3 * n, 3 * n))


def _scalar_csr_fast(mesh):
    a = mesh.arrays()
    n = len(a["cell_cx"])
    own = a["face_owner"].astype(np.int64)
    nb = a["face_neighbor"].astype(np.int64)
    m = nb != 0xFFFFFFFF
    r = np.concatenate([np.arange(n), own[m], nb[m]])
    c = np.concatenate([np.arange(n), nb[m], own[m]])
    key = np.unique(r * n + c)
    rr, cc = key // n, key % n
    srow = np.zeros(n + 1, dtype=np.int64)
    np.add.at(srow, rr + 1, 1)
    return np.cumsum(srow), cc


def test_reproduce_divergence_gpu():
    """tests/reproduce_divergence.rs: BackwardsStep h=0.025, water, alpha 0.7/0.3,
    adaptive dt (CFL 0.2, growth <= 1.2, dt <= 0.1), all 50 steps with the
    should_stop break: outer residuals finite and < 1e10, and GPU == oracle
    bit-exact after every step (same host-side dt sequence)."""
    from tests.meshes import STEP
    from cfd2_amd.mesh import generate_cut_cell_mesh
    mesh = generate_cut_cell_mesh(STEP, 0.025, 0.025, 1.2, (3.5, 1.0))
    mesh.smooth(STEP, 0.3, 50)
    min_cell = float(np.sqrt(mesh.arrays()["cell_vol"]).min())
    g, o = _pair(mesh)
    sols = [g, o]
    dts = {}
    for s in sols:
        s.set_density(1000.0)
        s.set_viscosity(0.001)
        s.set_scheme(0)
        s.set_alpha_u(0.7)
        s.set_alpha_p(0.3)
        n = mesh.num_cells()
        s.set_u(np.zeros((n, 2)))
        s.set_p(np.zeros(n))
        s.set_dt(0.001)
        dts[id(s)] = np.float32(0.001)
    for step in range(50):
        for s in sols:
            s.step()
            assert not (s.should_stop and s.degenerate_count > 10)
            i = s.step_info()
            for r in (i.outer_residual_u, i.outer_residual_p):
                assert np.isfinite(r) and r <= 1e10, (step, r)
            u = s.get_u()
            vmax = float(np.sqrt((u ** 2).sum(1)).max())
            if vmax > 1e-6:
                dt = float(dts[id(s)])
                new_dt = dt * 0.2 / (vmax * dt / min_cell)
                new_dt = min(new_dt, dt * 1.2, 0.1)
                s.set_dt(new_dt)
                dts[id(s)] = np.float32(new_dt)
        _assert_same_fields(g, o, f"reproduce_divergence step {step}")
        _assert_same_info(g, o, f"reproduce_divergence step {step}")
        if g.should_stop:
            break


def test_fine_mesh_obstacle_gpu():
    """tests/gpu_fine_mesh_obstacle.rs (#[ignore] in the reference: beyond its
    dispatch limit): ChannelWithObstacle r=0.2, h=0.001 (~2.87 M cells), dt 1e-4,
    nu 1e-3, u = (1, 0) for cx < 0.01, Jacobi preconditioner, natural
    convergence, 10 steps: no NaN, no degenerate stop."""
    mesh = channel_obstacle(h=0.001, smooth_iters=50)
    n = mesh.num_cells()
    assert 2.7e6 < n < 3.0e6
    g = GpuSolver(mesh)
    g.set_dt(1e-4)
    g.set_density(1.0)
    g.set_viscosity(0.001)
    u = np.zeros((n, 2))
    u[mesh.arrays()["cell_cx"] < 0.01, 0] = 1.0
    g.set_u(u)
    for _ in range(10):
        g.step()
        if g.should_stop:
            assert g.degenerate_count <= 10
            break
        uu = g.get_u()
        assert np.all(np.isfinite(uu))


def _amg_setup_pair(mesh, monkeypatch, **cfg):
    """The same AMG problem solved with the device setup (default on one GPU)
    and with CFD_AMG_SETUP=host; both after one step at t = 0.05 (inlet on)."""
    out = []
    for path in ("device", "host"):
        if path == "host":
            monkeypatch.setenv("CFD_AMG_SETUP", "host")
        else:
            monkeypatch.delenv("CFD_AMG_SETUP", raising=False)
        s = GpuSolver(mesh, config=default_config(**cfg))
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
        s.step()
        out.append(s)
    monkeypatch.delenv("CFD_AMG_SETUP", raising=False)
    return out


@pytest.mark.parametrize("which", ["amg_test", "bench_100k", "c1", "voronoi"])
def test_amg_device_setup_matches_host(which, monkeypatch):
    """the device-side AMG setup (Galerkin product and
    level packing on the GPU, aggregation on the host) builds a hierarchy
    byte-identical to the host setup -- every level's matrix, diagonal, P and
    R -- so the steps that follow are bit-identical too."""
    if which == "amg_test":
        mesh = backwards_step()
    elif which == "bench_100k":
        mesh = bench_mesh(0.0055, 30)
    elif which == "c1":
        mesh = bench_mesh(0.001723, 100)
    else:
        from tests.voronoi import voronoi_channel
        mesh = voronoi_channel(4000, seed=12345)
    dev, host = _amg_setup_pair(mesh, monkeypatch, fixed_outer=1, fixed_inner=4)
    pd, dd = dev.amg_setup_info()
    ph, dh = host.amg_setup_info()
    assert (pd, ph) == (2, 1), "device setup must be the path taken on one GPU"
    assert dev.amg_levels() == host.amg_levels()
    assert len(dd) >= (3 if which in ("bench_100k", "c1") else 1)
    assert dd == dh, [i for i, (a, b) in enumerate(zip(dd, dh)) if a != b]
    _assert_same_fields(dev, host, f"{which} device vs host AMG setup")
    _assert_same_info(dev, host, which)


@pytest.mark.parametrize("interval", [1, 2])
def test_amg_rebuild_interval_parity(interval):
    """Opt-in hierarchy rebuild every `interval` steps:
    GPU == oracle bit-exact, and the device hierarchy really changes."""
    mesh = backwards_step()
    g, o = _pair(mesh, amg_rebuild_interval=interval, fixed_outer=3, fixed_inner=10)
    for s in (g, o):
        _setup_amg_test(s, mesh, 1)
    digests = []
    for k in range(6):
        g.step()
        o.step()
        _assert_same_fields(g, o, f"rebuild/{interval} step {k}")
        _assert_same_info(g, o, f"rebuild/{interval} step {k}")
        digests.append(g.amg_setup_info()[1])
    assert digests[0] == digests[1] == digests[2]  # stale-ring steps: same source matrix
    assert digests[5] != digests[0]


def test_amg_refresh_matches_full_rebuild(monkeypatch):
    """The numeric re-setup (Galerkin fill + packing over the kept structure)
    produces the same hierarchy bytes and fields as dropping and rebuilding."""
    mesh = channel_obstacle(h=0.03)
    runs = {}
    for refresh in ("1", "0"):
        monkeypatch.setenv("CFD_AMG_SETUP", "device" if refresh == "1" else "rebuild")
        g = GpuSolver(mesh, config=default_config(amg_rebuild_interval=1, fixed_outer=2, fixed_inner=8))
        _setup_amg_test(g, mesh, 1)
        out = []
        for _ in range(6):
            g.step()
            out.append((g.get_u(), g.get_p(), g.amg_setup_info()[1]))
        runs[refresh] = out
    for k, (a, b) in enumerate(zip(runs["1"], runs["0"])):
        assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]), f"step {k} fields"
        assert a[2] == b[2], f"step {k} AMG level digests"


def test_log_level_reference_lines(capfd):
    """cfg.log_level = 1 prints the reference's progress lines (coupled_solver.rs:126,333,434;
    coupled_solver_fgmres.rs:1897,2264,2430) on stderr, with Rust's {:.2e} formatting."""
    import re
    mesh = backwards_step()
    g = GpuSolver(mesh, config=default_config(log_level=1))
    _setup_amg_test(g, mesh, 1)
    capfd.readouterr()
    g.step()
    err = capfd.readouterr().err
    info = g.step_info()
    assert "Coupled Iteration: 1\n" in err
    assert f"Coupled Iteration: {info.outer_iterations}\n" in err
    assert "FGMRES: Initial residual = " in err or "FGMRES: Initial guess already converged" in err
    solves = re.findall(r"Coupled linear solve: (\d+) iterations, residual (\S+), converged=(true|false)", err)
    assert len(solves) == info.outer_iterations
    last = solves[-1]
    assert int(last[0]) == info.stats_p.iterations
    assert re.fullmatch(r"-?\d\.\d\de-?\d+", last[1]), last[1]  # 1.23e-5, never 1.23e-05
    assert float(last[1]) == pytest.approx(info.stats_p.residual, rel=6e-3)
    quiet = GpuSolver(mesh)
    _setup_amg_test(quiet, mesh, 1)
    capfd.readouterr()
    quiet.step()
    assert capfd.readouterr().err == ""


VARIANTS = [
    {"CFD_AMG_FULL": "0"},            # predicated slot loads (production: coarse levels > 2^19 rows)
    {"CFD_AMG_FULL": "1"},            # unconditional slot loads on every level
    {"CFD_AMG_TAIL": "lds"},          # LDS tail with vectors only (fallback when the image does not fit)
    {"CFD_AMG_TAIL": "global"},       # global-memory single-workgroup tail (fallback when the vectors do not fit)
    {"CFD_AMG_TAIL_ROWS": "0"},       # no tail kernel: every level launched
    {"CFD_SMALL_MESH_FORMS": "0"},    # streaming CGS dots / update / update_x, k_cgs_reduce launched,
                                      # per-sweep Jacobi relaxation (production: > 131 k cells)
    {"CFD_AMG_FUSED_RR_ROWS": "0"},   # separate residual + restriction kernels on every level
    {"CFD_AMG_TAIL_ROWS": "0", "CFD_AMG_FULL": "0"},  # fused residual-restriction on every level, predicated loads
    {"CFD_AMG_FUSED_RR_ROWS": "4000000000"},          # fused residual-restriction on the big levels too
    {"CFD_AMG_FUSED_PROLONG_ROWS": "0"},              # separate prolongation + post-smoother launches
    {"CFD_AMG_FUSED_PROLONG_ROWS": "4000000000", "CFD_AMG_TAIL_ROWS": "0", "CFD_AMG_FULL": "0"},  # fused, every level
    {"CFD_NT": "127", "CFD_AMG_TAIL_ROWS": "0", "CFD_AMG_FUSED_PROLONG_ROWS": "0"},  # nontemporal loads everywhere
    {"CFD_NT": "127", "CFD_AMG_FULL": "0", "CFD_AMG_FUSED_RR_ROWS": "0"},            # ... with predicated slot loads
]


@pytest.mark.parametrize("env", VARIANTS, ids=lambda e: ",".join(f"{k}={v}" for k, v in e.items()))
@pytest.mark.parametrize("mesh_name", ["amg_test", "graded"])
def test_amg_kernel_variants_parity(env, mesh_name, monkeypatch):
    """Every V-cycle code path the level sizes select in production (some only
    at 10 M cells) forced on a small mesh: GPU == oracle bit-exact."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    if mesh_name == "amg_test":
        mesh = backwards_step()
    else:
        from cfd2_amd.mesh import ChannelWithObstacle, generate_cut_cell_mesh
        geo = ChannelWithObstacle(length=3.0, height=1.0, obstacle_center=(1.0, 0.5), obstacle_radius=0.15)
        mesh = generate_cut_cell_mesh(geo, 0.02, 0.08, 1.2, (3.0, 1.0))
    g, o = _pair(mesh, fixed_outer=3, fixed_inner=10)
    for s in (g, o):
        _setup_amg_test(s, mesh, 1)
    for k in range(3):
        g.step()
        o.step()
        _assert_same_fields(g, o, f"{env} {mesh_name} step {k}")
        _assert_same_info(g, o, f"{env} {mesh_name} step {k}")


@pytest.mark.parametrize("shift", ["0", "1", "4"])
def test_amg_blob_shift_parity(shift, monkeypatch, capfd):
    """CFD_AMG_TAIL=blob<K>: how many levels the LDS-image tail may start below
    the first tail level when that level's image does not fit one CU's LDS
    (production: C1's 3.9 k-row level; default K = 2).  Forced here by a tail
    from level 1 (CFD_AMG_TAIL_ROWS) on a mesh whose level 1 is too large for
    the image: K = 0 runs the vectors-only LDS tail, larger K the image tail
    from a lower level -- GPU == oracle bit-exact either way.  The setup line
    comes with cfg.log_level 2."""
    monkeypatch.setenv("CFD_AMG_TAIL_ROWS", "1000000")
    monkeypatch.setenv("CFD_AMG_TAIL", "blob" + shift)
    mesh = channel_obstacle(h=0.012)
    g = GpuSolver(mesh, config=default_config(fixed_outer=2, fixed_inner=8, log_level=2))
    o = OracleSolver(mesh, config=default_config(fixed_outer=2, fixed_inner=8))
    for s in (g, o):
        _setup_amg_test(s, mesh, 1)
    capfd.readouterr()
    for k in range(2):
        g.step()
        o.step()
        _assert_same_fields(g, o, f"blob shift {shift} step {k}")
        _assert_same_info(g, o, f"blob shift {shift} step {k}")
    import re
    m = re.search(r"tail from level (-?\d+) \(LDS image from level (-?\d+)\)", capfd.readouterr().err)
    assert m, "no AMG setup line"
    tail, blob = int(m.group(1)), int(m.group(2))
    if shift == "0":
        assert blob == -1 and tail == 1, (tail, blob)  # level 1's image does not fit: no image tail
    elif blob >= 0:
        assert blob == tail and 1 < tail <= 1 + int(shift), (tail, blob)
    else:
        assert tail == 1 and shift != "4", (tail, blob)  # four levels down the image fits


def test_midrun_api_changes_parity():
    """The reference API used mid-run the way the GUI does (src/ui/app.rs):
    dt / viscosity / scheme / time-scheme / preconditioner switches, a direct
    `constants` write, set_u and set_p clobbers and initialize_history between
    steps -- GPU == oracle bit-exact after every step."""
    mesh = channel_obstacle(h=0.04)
    g, o = _pair(mesh)
    a = mesh.arrays()
    n = mesh.num_cells()
    u0 = np.zeros((n, 2))
    u0[a["cell_cx"] < 0.05, 0] = 1.0

    def actions(s, k):
        if k == 0:
            s.set_dt(0.005)
            s.set_viscosity(0.01)
            s.set_density(1.0)
            s.set_u(u0)
            s.initialize_history()
            s.set_precond_type(1)
        elif k == 2:
            s.set_scheme(1)
            s.set_dt(0.004)  # dt_old keeps the previous dt (solver.rs:36-44)
        elif k == 3:
            s.set_time_scheme(1)
            s.set_precond_type(0)  # Jacobi; the frozen AMG hierarchy stays built
        elif k == 4:
            s.set_precond_type(1)
            c = s.constants
            c.alpha_u = 0.8
            c.inlet_velocity = 1.5
            s.constants = c
        elif k == 5:
            s.set_p(0.1 * a["cell_cx"])  # clobbers u, d_p, grad_p too (solver.rs:23-34)
        elif k == 6:
            s.set_u(np.column_stack([0.5 + 0.0 * a["cell_cx"], 0.0 * a["cell_cx"]]))
            s.set_scheme(2)
        s.update_constants()

    for k in range(8):
        for s in (g, o):
            actions(s, k)
        g.step()
        o.step()
        _assert_same_fields(g, o, f"mid-run step {k}")
        _assert_same_info(g, o, f"mid-run step {k}")


@pytest.mark.parametrize("inlet", [0.0, 1.0])
def test_fixed_schedule_early_exits(inlet):
    """Fixed schedule with the solve's early exits (coupled_solver_fgmres.rs
    rhs / initial-residual checks, kept under the fixed schedule): with a zero
    state and no inflow every solve exits early (rhs = 0); with inflow the
    t = 0 step exits early and the rest run.  GPU == oracle bit-exact, step
    statistics included."""
    mesh = channel_obstacle(h=0.04)
    g, o = _pair(mesh, fixed_outer=2, fixed_inner=8)
    for s in (g, o):
        s.set_dt(1e-3)
        s.set_viscosity(0.01)
        s.set_density(1.0)
        s.set_inlet_velocity(inlet)
        s.set_precond_type(1)
        s.initialize_history()
    for k in range(3):
        g.step()
        o.step()
        _assert_same_fields(g, o, f"inlet={inlet} step {k}")
        _assert_same_info(g, o, f"inlet={inlet} step {k}")


@pytest.mark.parametrize("mesh_name", ["amg_test", "graded", "channel_012"])
@pytest.mark.parametrize("pair", ["2", "0"])
def test_amg_resrestrict_pair_parity(mesh_name, pair, monkeypatch, capfd):
    """k_amg_resrestrict_pair / k_amg_prolong_smooth_pair: two adjacent
    down-leg levels, and two adjacent up-leg post-smoothers, in one launch
    (CFD_AMG_FUSED_PAIR; production: C1's levels 4+5 where the ring adds
    under 50 % rows).  With the tail off every level pair of these meshes is a
    candidate and mode 2 pairs them all; GPU == oracle bit-exact with the
    pairs on and off, and the setup line names the pairs."""
    monkeypatch.setenv("CFD_AMG_TAIL_ROWS", "0")
    monkeypatch.setenv("CFD_AMG_FUSED_PAIR", pair)
    if mesh_name == "amg_test":
        mesh = backwards_step()
    elif mesh_name == "graded":
        from cfd2_amd.mesh import ChannelWithObstacle, generate_cut_cell_mesh
        geo = ChannelWithObstacle(length=3.0, height=1.0, obstacle_center=(1.0, 0.5), obstacle_radius=0.15)
        mesh = generate_cut_cell_mesh(geo, 0.02, 0.08, 1.2, (3.0, 1.0))
    else:
        mesh = channel_obstacle(h=0.012)
    cfg = dict(fixed_outer=2, fixed_inner=8)
    g = GpuSolver(mesh, config=default_config(log_level=2, **cfg))
    o = OracleSolver(mesh, config=default_config(**cfg))
    for s in (g, o):
        _setup_amg_test(s, mesh, 1)
    capfd.readouterr()
    for k in range(2):
        g.step()
        o.step()
        _assert_same_fields(g, o, f"pair={pair} {mesh_name} step {k}")
        _assert_same_info(g, o, f"pair={pair} {mesh_name} step {k}")
    import re
    m = re.search(r"down-leg pairs:(.*), up-leg pairs:(.*)\n", capfd.readouterr().err)
    assert m, "no AMG setup line"
    for grp in (1, 2):  # 2: every candidate pair of either leg, whatever its redundancy
        pairs = [] if m.group(grp).strip() == "none" else m.group(grp).split()
        assert (len(pairs) > 0) == (pair == "2"), (grp, pairs)
    g.close()
