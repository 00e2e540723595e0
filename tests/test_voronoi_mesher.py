"""Native seeded Voronoi mesher (cfd_mesh_generate_voronoi; SURVEY §8(f)
rank 4, a behavioural restatement of voronoi.rs / delaunay.rs, whose RNG is
unseeded).  CPU: the reference's own mesher tests (src/solver/mesh/tests.rs
test_voronoi_generation, tests/reproduce_voronoi_quality.rs) plus FV validity
(closed cells, positive CCW polygons, oriented faces), determinism and oracle
runs.  GPU: bit-exact parity on these meshes, one GPU and distributed."""
import numpy as np
import pytest

from cfd2_amd import default_config
from cfd2_amd.mesh import (BackwardsStep, ChannelWithObstacle, CircleObstacle, RectangularChannel,
                           generate_delaunay_mesh, generate_voronoi_mesh)
from tests.oracle_py import OracleSolver

NONE = 0xFFFFFFFF
STEP = BackwardsStep(length=2.0, height_inlet=0.5, height_outlet=1.0, step_x=0.5)
CHANNEL = ChannelWithObstacle(length=3.0, height=1.0, obstacle_center=(1.0, 0.5), obstacle_radius=0.2)

CASES = {
    "step": (STEP, 0.05, 0.05, 1.2, (2.0, 1.0)),
    "channel": (CHANNEL, 0.03, 0.1, 1.2, (3.0, 1.0)),
    "rect": (RectangularChannel(length=2.0, height=1.0), 0.04, 0.04, 1.2, (2.0, 1.0)),
    "circle": (CircleObstacle((0.5, 0.5), 0.1, (0.0, 0.0), (1.0, 1.0)), 0.05, 0.15, 1.2, (1.0, 1.0)),
}


def _mesh(name, seed=12345):
    geo, mn, mx, gr, dom = CASES[name]
    return generate_voronoi_mesh(geo, mn, mx, gr, dom, seed=seed)


def test_voronoi_generation():
    """src/solver/mesh/tests.rs:256-318: CircleObstacle (0.1, 0.2, 1.2): total
    volume within 0.05 of the fluid area, >= 3 faces per cell, CCW polygons."""
    geo = CircleObstacle((0.5, 0.5), 0.1, (0.0, 0.0), (1.0, 1.0))
    m = generate_voronoi_mesh(geo, 0.1, 0.2, 1.2, (1.0, 1.0))
    a, t = m.arrays(), m.topology()
    vx, vy, _ = m.vertices()
    assert m.num_cells() > 0
    assert abs(a["cell_vol"].sum() - (1.0 - np.pi * 0.01)) < 0.05
    assert np.diff(a["cell_face_offsets"].astype(np.int64)).min() >= 3
    off, cv = t["cell_vertex_offsets"], t["cell_vertices"]
    for i in range(m.num_cells()):
        p = cv[off[i]:off[i + 1]]
        x, y = vx[p], vy[p]
        assert (x * np.roll(y, -1) - np.roll(x, -1) * y).sum() > 0.0, f"cell {i} not CCW"


def test_voronoi_boundary_fidelity():
    """tests/reproduce_voronoi_quality.rs: BackwardsStep, h = 0.05, smoothed
    (0.3, 10): every vertex of every boundary face stays on the geometry."""
    m = _mesh("step")
    m.smooth(STEP, 0.3, 10)
    a, t = m.arrays(), m.topology()
    vx, vy, _ = m.vertices()
    bad = 0
    for f in np.nonzero(a["face_boundary"] != 0)[0]:
        for v in (t["face_v1"][f], t["face_v2"][f]):
            bad += abs(_sdf_step(vx[v], vy[v])) > 1e-3
    assert bad == 0


def _sdf_step(x, y, L=2.0, h_in=0.5, h_out=1.0, sx=0.5):
    def box(dx, dy):
        return min(max(dx, dy), 0.0) + np.hypot(max(dx, 0.0), max(dy, 0.0))
    outer = box(abs(x - L / 2) - L / 2, abs(y - h_out / 2) - h_out / 2)
    sh = h_out - h_in
    block = box(abs(x - sx / 2) - sx / 2, abs(y - sh / 2) - sh / 2)
    return max(outer, -block)


def test_voronoi_cell_connectivity():
    """tests/reproduce_voronoi_quality.rs: a boundary generator V appears in
    its cell's polygon between two boundary midpoints, never next to an
    interior dual point."""
    m = _mesh("step")
    t = m.topology()
    vx, vy, vfix = m.vertices()
    off, cv = t["cell_vertex_offsets"], t["cell_vertices"]
    checked = 0
    for i in range(m.num_cells()):
        p = cv[off[i]:off[i + 1]]
        on = [k for k, v in enumerate(p) if vfix[v] and abs(_sdf_step(vx[v], vy[v])) < 1e-9]
        if len(on) < 3:
            continue
        # the generator: the fixed vertex whose both polygon neighbours are fixed too
        for k in on:
            prev, nxt = p[k - 1], p[(k + 1) % len(p)]
            if vfix[prev] and vfix[nxt]:
                checked += 1
                assert abs(_sdf_step(vx[prev], vy[prev])) < 1e-9 and abs(_sdf_step(vx[nxt], vy[nxt])) < 1e-9
    assert checked > 0


@pytest.mark.parametrize("name", sorted(CASES))
def test_fv_validity(name):
    m = _mesh(name)
    a = m.arrays()
    n = m.num_cells()
    assert a["cell_vol"].min() > 0.0
    own = a["face_owner"].astype(np.int64)
    nb = a["face_neighbor"].astype(np.int64)
    internal = nb != NONE
    assert np.all(own[internal] < nb[internal])
    # closed cells: sum of outward area vectors vanishes
    an = np.stack([a["face_area"] * a["face_nx"], a["face_area"] * a["face_ny"]], 1)
    s = np.zeros((n, 2))
    np.add.at(s, own, an)
    np.add.at(s, nb[internal], -an[internal])
    assert np.abs(s).max() < 1e-12
    # interior normals point owner -> neighbour, boundary normals out of the owner
    d = np.stack([a["cell_cx"][nb[internal]] - a["cell_cx"][own[internal]],
                  a["cell_cy"][nb[internal]] - a["cell_cy"][own[internal]]], 1)
    assert np.all((d * an[internal]).sum(1) > 0.0)
    db = np.stack([a["face_cx"][~internal] - a["cell_cx"][own[~internal]],
                   a["face_cy"][~internal] - a["cell_cy"][own[~internal]]], 1)
    assert np.all((db * an[~internal]).sum(1) > 0.0)
    nf = np.diff(a["cell_face_offsets"].astype(np.int64))
    assert nf.min() >= 3 and nf.max() >= 7 and 5.5 < nf.mean() < 6.5  # polygonal
    kinds = set(np.unique(a["face_boundary"]).tolist())
    assert {1, 2, 3} <= kinds or name == "circle"


def test_seeded_determinism():
    m1, m2, m3 = _mesh("channel", 7), _mesh("channel", 7), _mesh("channel", 8)  # arrays() are views: keep alive
    a1, a2, b = m1.arrays(), m2.arrays(), m3.arrays()
    for k in a1:
        assert np.array_equal(a1[k], a2[k]), k
    assert a1["cell_cx"].shape != b["cell_cx"].shape or not np.array_equal(a1["cell_cx"], b["cell_cx"])


def test_bad_arguments_rejected():
    with pytest.raises(RuntimeError, match="status 1"):
        generate_voronoi_mesh(CHANNEL, 0.1, 0.05, 1.2, (3.0, 1.0))


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


@pytest.mark.parametrize("name", ["step", "channel"])
def test_oracle_runs_on_voronoi(name):
    m = _mesh(name)
    o = OracleSolver(m)
    _setup(o)
    for _ in range(3):
        o.step()
    u = o.get_u()
    assert np.all(np.isfinite(u)) and u[:, 0].max() > 0.1


@pytest.mark.gpu
@pytest.mark.parametrize("name,scheme,precond", [("step", 0, 1), ("channel", 1, 1), ("channel", 2, 0),
                                                 ("circle", 0, 1)])
def test_native_voronoi_gpu_parity(name, scheme, precond):
    from cfd2_amd import GpuSolver
    from tests.test_gpu_parity import _assert_same_fields, _assert_same_info
    m = _mesh(name)
    g, o = GpuSolver(m), OracleSolver(m)
    for s in (g, o):
        _setup(s, scheme, precond)
    for k in range(3):
        g.step()
        o.step()
        _assert_same_fields(g, o, f"{name} step {k}")
        _assert_same_info(g, o, f"{name} step {k}")


@pytest.mark.gpu
@pytest.mark.parametrize("nranks", [2, 3])
def test_native_voronoi_group_parity(nranks, monkeypatch):
    from cfd2_amd import GpuGroup
    from tests.test_gpu_parity import _assert_same_fields
    monkeypatch.setenv("CFD_AMG_REPLICATE_ROWS", "200")
    m = generate_voronoi_mesh(CHANNEL, 0.02, 0.06, 1.2, (3.0, 1.0), seed=3)
    cfg = dict(fixed_outer=3, fixed_inner=10)
    g = GpuGroup(m, nranks, config=default_config(**cfg))
    o = OracleSolver(m, config=default_config(**cfg), nranks=nranks)
    for s in (g, o):
        _setup(s, 1, 1)
    for k in range(3):
        g.step()
        o.step()
        _assert_same_fields(g, o, f"native voronoi R={nranks} step {k}")
    g.close()


@pytest.mark.parametrize("name", ["step", "channel"])
def test_delaunay_mesh_validity(name):
    """generate_delaunay_mesh (delaunay.rs:732): triangle cells, closed, fluid area."""
    geo, mn, mx, gr, dom = CASES[name]
    m = generate_delaunay_mesh(geo, mn, mx, gr, dom, seed=5)
    a = m.arrays()
    n = m.num_cells()
    assert np.all(np.diff(a["cell_face_offsets"].astype(np.int64)) == 3)
    assert a["cell_vol"].min() > 0.0
    area = {"step": 1.75, "channel": 3.0 - np.pi * 0.04}[name]
    assert abs(a["cell_vol"].sum() - area) < 0.02
    own = a["face_owner"].astype(np.int64)
    nb = a["face_neighbor"].astype(np.int64)
    internal = nb != NONE
    an = np.stack([a["face_area"] * a["face_nx"], a["face_area"] * a["face_ny"]], 1)
    s = np.zeros((n, 2))
    np.add.at(s, own, an)
    np.add.at(s, nb[internal], -an[internal])
    assert np.abs(s).max() < 1e-12
    assert {1, 2, 3} <= set(np.unique(a["face_boundary"]).tolist())


@pytest.mark.gpu
def test_delaunay_mesh_gpu_parity():
    from cfd2_amd import GpuSolver
    from tests.test_gpu_parity import _assert_same_fields, _assert_same_info
    m = generate_delaunay_mesh(CHANNEL, 0.03, 0.1, 1.2, (3.0, 1.0), seed=5)
    g, o = GpuSolver(m), OracleSolver(m)
    for s in (g, o):
        _setup(s, 1, 1)
    for k in range(3):
        g.step()
        o.step()
        _assert_same_fields(g, o, f"delaunay step {k}")
        _assert_same_info(g, o, f"delaunay step {k}")
