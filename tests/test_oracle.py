"""CPU oracle: the reference tests' assertions, independent cross-checks
(numpy restatement of the face sweeps, scipy AMG Galerkin product, numpy
residuals) and the committed golden fixtures (tests/golden, made by
tests/golden/make_golden.py)."""
import os

import numpy as np
import pytest

from cfd2_amd import default_config
from tests import numpy_ref
from tests.meshes import backwards_step, channel_obstacle
from tests.oracle_py import OracleSolver

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def setup_amg_test(s, mesh, precond):
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


def setup_schemes_test(s, mesh, scheme, time_scheme):
    """tests/coupled_schemes_test.rs:28-49."""
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


@pytest.mark.parametrize("scheme,time_scheme", [(0, 0), (1, 0), (2, 0), (0, 1)])
def test_coupled_schemes_finite(scheme, time_scheme):
    """tests/coupled_schemes_test.rs:84-103: every field finite after 2 steps."""
    mesh = backwards_step()
    s = OracleSolver(mesh)
    setup_schemes_test(s, mesh, scheme, time_scheme)
    for _ in range(2):
        s.step()
        assert not (s.should_stop and s.degenerate_count > 10)
    assert np.all(np.isfinite(s.get_u())) and np.all(np.isfinite(s.get_p()))


@pytest.mark.parametrize("precond", [0, 1])
def test_amg_test_bounds(precond):
    """tests/amg_test.rs:84-86: 0 < max|p| < 1000 after 5 steps."""
    mesh = backwards_step()
    s = OracleSolver(mesh)
    setup_amg_test(s, mesh, precond)
    for _ in range(5):
        s.step()
    max_p = np.abs(s.get_p()).max()
    assert 0.0 < max_p < 1000.0


def test_reproduce_divergence_short():
    """tests/reproduce_divergence.rs (water, alpha 0.7/0.3, dt 1e-3; 8 steps instead of 50
    on the h=0.05 mesh): outer residuals finite and < 1e10."""
    mesh = backwards_step()
    s = OracleSolver(mesh)
    s.set_density(1000.0)
    s.set_viscosity(0.001)
    s.set_scheme(0)
    s.set_alpha_u(0.7)
    s.set_alpha_p(0.3)
    n = mesh.num_cells()
    s.set_u(np.zeros((n, 2)))
    s.set_p(np.zeros(n))
    s.set_dt(0.001)
    for _ in range(8):
        s.step()
        i = s.step_info()
        for r in (i.outer_residual_u, i.outer_residual_p):
            assert np.isfinite(r) and r < 1e10


def test_prepare_assemble_vs_numpy_restatement():
    """The oracle's literal WGSL restatement agrees with an independently written
    face-wise numpy restatement (tolerance: different summation order)."""
    mesh = channel_obstacle()
    a = mesh.arrays()
    s = OracleSolver(mesh)
    rng = np.random.default_rng(7)
    u0 = rng.uniform(-1, 1, size=(mesh.num_cells(), 2))
    s.set_u(u0)
    s.initialize_history()
    s.set_dt(0.002)
    c = s.constants
    c.time = 0.05
    s.constants = c
    s.debug_prepare_assemble(False)
    dp0 = s.get_d_p().astype(np.float32)
    gp0 = s.debug_buffer(10).reshape(-1, 2)
    s.debug_prepare_assemble(True)
    m = numpy_ref.mesh_f32(a)
    u32 = u0.astype(np.float32)
    p32 = np.zeros(mesh.num_cells(), np.float32)
    flux, d_p, gp, gu, gv = numpy_ref.prepare(m, u32, p32, dp0, gp0, s.constants)
    scale = lambda x: max(np.abs(x).max(), 1e-30)  # noqa: E731
    np.testing.assert_allclose(s.debug_buffer(0), flux, rtol=0, atol=2e-5 * scale(flux))
    np.testing.assert_allclose(s.get_d_p(), d_p, rtol=1e-4, atol=0)
    np.testing.assert_allclose(s.debug_buffer(10).reshape(-1, 2), gp, rtol=0, atol=2e-4 * scale(gp))
    np.testing.assert_allclose(s.debug_buffer(1).reshape(-1, 2), gu, rtol=0, atol=2e-4 * scale(gu))
    np.testing.assert_allclose(s.debug_buffer(2).reshape(-1, 2), gv, rtol=0, atol=2e-4 * scale(gv))
    srow, scol = numpy_ref.scalar_csr(a)
    mv, rhs, sv = numpy_ref.assemble(m, srow, scol, s.debug_buffer(0), u32,
                                     s.get_d_p(), s.constants)
    np.testing.assert_allclose(s.debug_buffer(9), mv, rtol=0, atol=1e-5 * scale(mv))
    np.testing.assert_allclose(s.debug_buffer(3), rhs, rtol=0, atol=1e-5 * scale(rhs))
    np.testing.assert_allclose(s.debug_buffer(8), sv, rtol=0, atol=1e-5 * scale(sv))


def test_amg_hierarchy_vs_scipy():
    """amg.rs:84-235 aggregation + Galerkin RAP, rebuilt with scipy.sparse from the
    oracle's scalar matrix: same level sizes and sparsity."""
    sp = pytest.importorskip("scipy.sparse")
    mesh = backwards_step()
    a = mesh.arrays()
    s = OracleSolver(mesh)
    setup_amg_test(s, mesh, 1)
    s.step()  # first AMG solve builds the hierarchy from the live scalar matrix
    srow, scol = numpy_ref.scalar_csr(a)
    levels = s.amg_levels()  # aggregation depends only on the sparsity pattern
    n = len(srow) - 1
    A = sp.csr_matrix((np.ones(len(scol)), scol, srow), shape=(n, n))
    sizes = [(n, A.nnz)]
    cur = A
    while cur.shape[0] > 100 and len(sizes) < 20:
        indptr, indices = cur.indptr, cur.indices
        agg = -np.ones(cur.shape[0], dtype=np.int64)
        na = 0
        for i in range(cur.shape[0]):
            if agg[i] >= 0:
                continue
            agg[i] = na
            for j in indices[indptr[i]:indptr[i + 1]]:
                if j != i and agg[j] < 0:
                    agg[j] = na
            na += 1
        if na >= cur.shape[0]:
            break
        P = sp.csr_matrix((np.ones(cur.shape[0]), agg, np.arange(cur.shape[0] + 1)),
                          shape=(cur.shape[0], na))
        cur = (P.T @ cur @ P).tocsr()
        cur.sum_duplicates()
        sizes.append((cur.shape[0], cur.nnz))
    assert levels == sizes


def test_fgmres_residual_consistent_with_numpy():
    """After one step the stored coupled system satisfies ||b - A x|| (numpy, f64)
    close to the solver's reported residual (true-residual path, lag 0)."""
    sp = pytest.importorskip("scipy.sparse")
    mesh = backwards_step()
    a = mesh.arrays()
    s = OracleSolver(mesh, config=default_config(convergence_lag=0, fixed_outer=1))
    setup_amg_test(s, mesh, 1)
    s.step()
    s.step()
    srow, scol = numpy_ref.scalar_csr(a)
    n = len(srow) - 1
    rows, cols = [], []
    for i in range(n):
        nb = scol[srow[i]:srow[i + 1]]
        for sub in range(3):
            for j in nb:
                rows += [3 * i + sub] * 3
                cols += [3 * j, 3 * j + 1, 3 * j + 2]
    A = sp.csr_matrix((s.debug_buffer(9).astype(np.float64), (rows, cols)), shape=(3 * n, 3 * n))
    b = s.debug_buffer(3).astype(np.float64)
    x = s.debug_buffer(4).astype(np.float64)
    r = np.linalg.norm(b - A @ x)
    info = s.step_info().stats_p
    assert np.isfinite(r)
    assert r <= max(10 * info.residual, 1e-5 * np.linalg.norm(b)), (r, info.residual)


def test_csr_structure_and_diagonal():
    """init/mesh.rs:27-53,201-212: scalar CSR rows sorted, diagonal present, symmetric."""
    a = backwards_step().arrays()
    srow, scol = numpy_ref.scalar_csr(a)
    n = len(srow) - 1
    for i in range(n):
        r = scol[srow[i]:srow[i + 1]]
        assert np.all(np.diff(r) > 0) and i in r
    s = OracleSolver(backwards_step())
    assert len(s.debug_buffer(8)) == len(scol)
    assert len(s.debug_buffer(9)) == 9 * len(scol)


@pytest.mark.parametrize("name", ["schemes", "amg"])
def test_golden_fixtures(name):
    """Oracle reproduces the committed golden vectors bit-for-bit (regression pin;
    generated by tests/golden/make_golden.py from this oracle)."""
    from tests.golden.make_golden import run_case
    path = os.path.join(GOLDEN, f"{name}.npz")
    ref = np.load(path, allow_pickle=False)
    got = run_case(name, OracleSolver)
    assert set(ref.files) == set(got)
    for k in ref.files:
        assert np.array_equal(ref[k], got[k]), k


def test_amg_rebuild_interval_changes_only_later_steps():
    """amg_rebuild_interval (opt-in): later steps rebuild
    the hierarchy from the current matrix and depart from the reference's
    frozen one."""
    mesh = backwards_step()
    runs = {}
    for k in (0, 1):
        o = OracleSolver(mesh, config=default_config(amg_rebuild_interval=k, fixed_outer=3, fixed_inner=10))
        setup_amg_test(o, mesh, 1)
        out = []
        for _ in range(5):
            o.step()
            out.append(o.get_u())
        runs[k] = out
        assert np.all(np.isfinite(out[-1]))
    # steps 1-3 start from the same (stale ring, §0.1-1) state, so their first
    # assembled matrices -- the AMG sources -- coincide; step 4 reads step 1's
    assert all(np.array_equal(runs[0][j], runs[1][j]) for j in range(3))
    assert not np.array_equal(runs[0][4], runs[1][4])


def _partition(n, nranks):
    """csrc/host/dist.cpp partition_starts: whole reduction segments per rank."""
    g = 0
    while g < 8 and (n >> (g + 1)) >= 16384:
        g += 1
    seg = 256 << g
    nseg = ((n + 255) // 256 + (1 << g) - 1) >> g
    s = [min(n, seg * (nseg * r // nranks)) for r in range(nranks + 1)]
    s[-1] = n
    return s


@pytest.mark.parametrize("nranks", [2, 3])
def test_oracle_local_aggregation(nranks, monkeypatch):
    """Partition-aware AMG mode of the oracle (cfd_config.amg_local_aggregation):
    level 1 has exactly the aggregates of the greedy index-order pass run on
    each rank's own rows with the cross-rank entries dropped (restated here on
    the mesh's face list, init/mesh.rs:27-53 + amg.rs:84-116); the run stays
    finite; one rank, or the mode off, gives the global hierarchy."""
    monkeypatch.setenv("CFD_AMG_REPLICATE_ROWS", "50")
    mesh = backwards_step()
    n = mesh.num_cells()
    a = mesh.arrays()
    own, nb = a["face_owner"].astype(np.int64), a["face_neighbor"].astype(np.int64)
    inner = (nb < n) & (nb != own)
    adj = [set([i]) for i in range(n)]
    for p, q in zip(own[inner], nb[inner]):
        adj[p].add(q)
        adj[q].add(p)
    starts = _partition(n, nranks)
    nagg = 0
    for r in range(nranks):
        lo, hi = starts[r], starts[r + 1]
        agg = {}
        for i in range(lo, hi):
            if i in agg:
                continue
            agg[i] = nagg
            for j in sorted(adj[i]):
                if lo <= j < hi and j not in agg:
                    agg[j] = nagg
            nagg += 1
    sols = {}
    for key, cfg, R in (("local", 1, nranks), ("global", 0, nranks), ("local1", 1, 1)):
        s = OracleSolver(mesh, config=default_config(amg_local_aggregation=cfg), nranks=R)
        setup_amg_test(s, mesh, 1)
        for _ in range(3):
            s.step()
        p = s.get_p()
        assert np.all(np.isfinite(p))
        sols[key] = (s.amg_levels(), p)
    assert sols["local"][0][1][0] == nagg, (sols["local"][0][:2], nagg)
    assert sols["local"][0] != sols["global"][0]
    assert sols["local1"][0] == sols["global"][0] and np.array_equal(sols["local1"][1], sols["global"][1])
