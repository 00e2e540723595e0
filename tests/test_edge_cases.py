"""Edge cases the reference's solver tests do not reach but a drop-in must
survive: degenerate sizes (1 cell, 1-D strips), broken meshes rejected with a
status instead of a crash, partition extremes (as many ranks as reduction segments)."""
import ctypes as C

import numpy as np
import pytest

from cfd2_amd import _ffi, default_config, dist_plan
from cfd2_amd.solver import _bind
from tests.oracle_py import OracleSolver
from tests.synthetic import broken, strip, wheel


def _create_status(mesh, **cfg):
    L = _bind()
    c = default_config(**cfg)
    h = C.c_void_p()
    st = L.cfd_solver_create(C.byref(mesh.view()), C.byref(c), 0, C.byref(h))
    if st == 0:
        L.cfd_solver_destroy(h)
    return st, L.cfd_last_error().decode()


@pytest.mark.parametrize("kind", ["owner_range", "neighbor_range", "cell_faces_range", "empty"])
def test_broken_meshes_rejected_before_device_use(kind):
    st, msg = _create_status(broken(kind))
    assert st == 1, (st, msg)
    assert msg


def test_row_width_limit():
    """A cell with 127 neighbours (scalar row width 128) exceeds the 7-bit
    slots-in-use field of the coupled-matrix ELL header: rejected with a
    status before any device use, never silently truncated.  126 neighbours
    (width 127) pass the topology check (the GPU parity of wide rows is
    tests/test_gpu_edge.py)."""
    st, msg = _create_status(wheel(127))
    assert st == 1 and "neighbours" in msg, (st, msg)
    st, msg = _create_status(wheel(126))
    assert "neighbours" not in msg, msg  # fails later, at device use, on a GPU-less host


@pytest.mark.parametrize("k", [5, 40, 100])
def test_oracle_wheel_mesh(k):
    """The wheel mesh is a valid FV mesh: closed cells, and the oracle steps it."""
    m = wheel(k)
    a = m.arrays()
    # every cell closed: sum of area * outward normal = 0
    for c in range(m.num_cells()):
        fs = a["cell_faces"][a["cell_face_offsets"][c]:a["cell_face_offsets"][c + 1]]
        sgn = np.where(a["face_owner"][fs] == c, 1.0, -1.0)
        sx = (sgn * a["face_area"][fs] * a["face_nx"][fs]).sum()
        sy = (sgn * a["face_area"][fs] * a["face_ny"][fs]).sum()
        assert abs(sx) < 1e-12 and abs(sy) < 1e-12, c
    s = OracleSolver(m)
    s.set_dt(0.01)
    s.set_viscosity(0.01)
    s.set_density(1.0)
    s.set_precond_type(1)
    s.initialize_history()
    c = s.constants
    c.time = 0.1
    s.constants = c
    for _ in range(2):
        s.step()
    assert np.all(np.isfinite(s.get_u())) and np.abs(s.get_u()).max() > 0


def test_bad_config_rejected():
    st, msg = _create_status(strip(4), max_restart=0)
    assert st == 1 and "max_restart" in msg


def test_more_ranks_than_cells_rejected():
    L = _bind()
    z = C.c_uint32()
    st = L.cfd_dist_plan(C.byref(strip(3).view()), 4, 0, C.byref(z), C.byref(z), C.byref(z), C.byref(z),
                         C.byref(z), None, None, None, None, None)
    assert st == 1


def test_more_ranks_than_segments_rejected():
    """Ranks own whole segments of the reduction tree (256 cells at this size):
    300 cells are 2 segments, so 3 ranks are refused with a status."""
    L = _bind()
    z = C.c_uint32()
    st = L.cfd_dist_plan(C.byref(strip(300).view()), 3, 0, C.byref(z), C.byref(z), C.byref(z), C.byref(z),
                         C.byref(z), None, None, None, None, None)
    assert st == 1 and "segments" in L.cfd_last_error().decode()


def test_one_segment_per_rank_plans():
    """As many ranks as reduction segments: each rank owns exactly one 256-cell
    segment of the strip and exchanges one ghost with each slab neighbour."""
    m = strip(6 * 256)
    plans = [dist_plan(m, 6, r) for r in range(6)]
    for r, P in enumerate(plans):
        assert (P["c0"], P["c1"]) == (256 * r, 256 * (r + 1))
        want = [q for q in (r - 1, r + 1) if 0 <= q < 6]
        assert P["peers"] == want
        assert list(P["ghost"]) == [g for g in (256 * r - 1, 256 * (r + 1)) if 0 <= g < 6 * 256]
        assert P["recv"] == [1] * len(want) and P["send"] == [1] * len(want)


@pytest.mark.parametrize("n", [1, 2, 7])
@pytest.mark.parametrize("precond", [0, 1])
def test_oracle_tiny_strips(n, precond):
    """1-D channel strips down to a single cell: steps stay finite, inflow moves fluid."""
    m = strip(n)
    s = OracleSolver(m)
    s.set_dt(0.01)
    s.set_viscosity(0.01)
    s.set_density(1.0)
    s.set_precond_type(precond)
    s.initialize_history()
    c = s.constants
    c.time = 0.1
    s.constants = c
    for _ in range(3):
        s.step()
    u, p = s.get_u(), s.get_p()
    assert np.all(np.isfinite(u)) and np.all(np.isfinite(p))
    assert u[:, 0].max() > 0.0
