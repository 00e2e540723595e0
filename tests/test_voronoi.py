"""Polygonal (seeded Voronoi) meshes: 4-9 faces per cell, ragged ELL widths.
CPU: geometric closure + oracle runs.  GPU: bit-exact parity, one GPU and
distributed (in-process ranks)."""
import numpy as np
import pytest

from cfd2_amd import default_config
from tests.oracle_py import OracleSolver
from tests.voronoi import voronoi_channel


def _setup(s, scheme=0, precond=1):
    s.set_dt(0.01)
    s.set_viscosity(0.01)
    s.set_density(1.0)
    s.set_scheme(scheme)
    s.set_precond_type(precond)
    s.initialize_history()
    c = s.constants
    c.time = 0.1
    s.constants = c


def test_voronoi_mesh_is_closed_and_ragged():
    m = voronoi_channel(seed=7)
    a = m.arrays()
    n = m.num_cells()
    nf = np.diff(a["cell_face_offsets"].astype(np.int64))
    assert nf.min() >= 3 and nf.max() >= 7
    assert abs(a["cell_vol"].sum() - 3.0) < 1e-9
    own = a["face_owner"].astype(np.int64)
    nb = a["face_neighbor"].astype(np.int64)
    s = np.zeros((n, 2))
    an = np.stack([a["face_area"] * a["face_nx"], a["face_area"] * a["face_ny"]], 1)
    np.add.at(s, own, an)
    internal = nb != 0xFFFFFFFF
    np.add.at(s, nb[internal], -an[internal])
    assert np.abs(s).max() < 1e-12


@pytest.mark.parametrize("precond", [0, 1])
def test_voronoi_oracle_runs(precond):
    m = voronoi_channel()
    o = OracleSolver(m)
    _setup(o, precond=precond)
    for _ in range(3):
        o.step()
    u = o.get_u()
    assert np.all(np.isfinite(u)) and u[:, 0].max() > 0.1


@pytest.mark.gpu
@pytest.mark.parametrize("scheme,precond", [(0, 1), (1, 1), (2, 0)])
def test_voronoi_gpu_parity(scheme, precond):
    from cfd2_amd import GpuSolver
    from tests.test_gpu_parity import _assert_same_fields, _assert_same_info
    m = voronoi_channel(n_points=3000, seed=99)
    g, o = GpuSolver(m), OracleSolver(m)
    for s in (g, o):
        _setup(s, scheme, precond)
    for k in range(3):
        g.step()
        o.step()
        _assert_same_fields(g, o, f"voronoi step {k}")
        _assert_same_info(g, o, f"voronoi step {k}")


@pytest.mark.gpu
@pytest.mark.parametrize("nranks", [2, 3])
def test_voronoi_group_parity(nranks):
    import os
    from cfd2_amd import GpuGroup
    from tests.test_gpu_parity import _assert_same_fields
    os.environ["CFD_AMG_REPLICATE_ROWS"] = "200"
    try:
        m = voronoi_channel(n_points=3000, seed=5)
        cfg = dict(fixed_outer=3, fixed_inner=10)
        g = GpuGroup(m, nranks, config=default_config(**cfg))
        o = OracleSolver(m, config=default_config(**cfg), nranks=nranks)
        for s in (g, o):
            _setup(s, 1, 1)
        for k in range(3):
            g.step()
            o.step()
            _assert_same_fields(g, o, f"voronoi R={nranks} step {k}")
        g.close()
    finally:
        os.environ.pop("CFD_AMG_REPLICATE_ROWS", None)


@pytest.mark.gpu
@pytest.mark.parametrize("precond", [1, 0])
def test_c0_voronoi_bench_mesh_gpu_parity(precond):
    """BASELINE configs[0] as named: the ~10 k-cell seeded Voronoi channel +
    obstacle (bench.py --config c0), bench physics from t = 0.05; AMG under
    the bench's 5 x 30 schedule, Jacobi under the reference's natural
    schedule; two steps each, GPU == oracle bit-exact."""
    from cfd2_amd import GpuSolver
    from cfd2_amd.mesh import bench_voronoi_channel
    from tests.test_gpu_configs import _bench_setup
    from tests.test_gpu_parity import _assert_same_fields, _assert_same_info
    m = bench_voronoi_channel()
    assert 9000 < m.num_cells() < 11000
    cfg = dict(fixed_outer=5, fixed_inner=30) if precond == 1 else {}
    g = GpuSolver(m, config=default_config(**cfg))
    o = OracleSolver(m, config=default_config(**cfg))
    for s in (g, o):
        _bench_setup(s, 0.05)
        s.set_precond_type(precond)
    for k in range(2):
        g.step()
        o.step()
        _assert_same_fields(g, o, f"C0 voronoi precond {precond} step {k}")
        _assert_same_info(g, o, f"C0 voronoi precond {precond} step {k}")
    assert np.abs(g.get_u()).max() > 0.01
    g.close()
