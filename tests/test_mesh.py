"""Mesh input (restated cut-cell generator, src/solver/mesh): the reference's own
mesh tests (src/solver/mesh/tests.rs:63-145) plus structural invariants the
solver relies on."""
import math
import os
import tempfile

import numpy as np
import pytest

from cfd2_amd.mesh import (BackwardsStep, ChannelWithObstacle, CircleObstacle, Mesh,
                           bench_channel, generate_cut_cell_mesh)
from tests.meshes import backwards_step


def test_mesh_generation_circle_obstacle():
    """tests.rs:63-115: fixed vertices stay on the surface after smoothing; skew < 0.25."""
    geo = CircleObstacle(center=(0.5001, 0.5001), radius=0.2, domain_min=(0.0, 0.0),
                         domain_max=(1.0, 1.0))
    m = generate_cut_cell_mesh(geo, 0.1, 0.1, 1.2, (1.0, 1.0))
    assert m.num_cells() > 0
    vx, vy, vf = m.vertices()
    fixed = np.nonzero(vf)[0]
    assert len(fixed) > 0
    m.smooth(geo, 0.05, 50)
    vx, vy, _ = m.vertices()
    g = geo._geo()
    for i in fixed:  # sdf of the smoothed fixed vertices (re-evaluated with numpy)
        x, y = vx[i], vy[i]
        dx = abs(x - 0.5) - 0.5
        dy = abs(y - 0.5) - 0.5
        box = min(max(dx, dy), 0.0) + math.hypot(max(dx, 0.0), max(dy, 0.0))
        circ = math.hypot(x - 0.5001, y - 0.5001) - 0.2
        assert abs(max(box, -circ)) < 1e-4
    assert g.kind == 3
    assert m.calculate_max_skewness() < 0.25


def test_mesh_generation_backwards_step():
    """tests.rs:117-145: misaligned step (0.501) -> sliver cells; skew < 0.6 after smoothing."""
    geo = BackwardsStep(length=2.0, height_inlet=0.501, height_outlet=1.0, step_x=0.501)
    m = generate_cut_cell_mesh(geo, 0.1, 0.1, 1.2, (2.0, 1.0))
    assert m.num_cells() > 0
    m.smooth(geo, 0.1, 50)
    assert m.calculate_max_skewness() < 0.6


def _check_structure(m, domain_area, rtol=1e-9):
    a = m.arrays()
    n, f = m.num_cells(), m.num_faces()
    assert np.all(a["cell_vol"] > 0)
    assert abs(a["cell_vol"].sum() - domain_area) <= rtol * domain_area
    assert np.allclose(a["face_nx"] ** 2 + a["face_ny"] ** 2, 1.0)
    assert np.all(a["face_area"] > 0)
    internal = a["face_neighbor"] != 0xFFFFFFFF
    assert np.all(a["face_boundary"][internal] == 0)
    assert np.all(np.isin(a["face_boundary"][~internal], [1, 2, 3]))
    # every face is listed exactly by its owner (and its neighbour if internal)
    counts = np.bincount(a["cell_faces"], minlength=f)
    assert np.all(counts == np.where(internal, 2, 1))
    offs = a["cell_face_offsets"]
    assert offs[0] == 0 and offs[-1] == len(a["cell_faces"]) and np.all(np.diff(offs) >= 3)
    # stored normals point out of the owner for boundary faces (cut_cell.rs:455)
    b = ~internal
    ow = a["face_owner"][b]
    d = (a["face_cx"][b] - a["cell_cx"][ow]) * a["face_nx"][b] + \
        (a["face_cy"][b] - a["cell_cy"][ow]) * a["face_ny"][b]
    assert np.all(d > 0)
    # inlet faces at x = 0, outlet at x = L
    return a


def test_coupled_schemes_mesh():
    """The mesh of coupled_schemes_test.rs / amg_test.rs: ~1.3k cells."""
    m = backwards_step()
    assert m.num_cells() == 1300
    a = _check_structure(m, 3.5 * 1.0 - 0.5 * 0.5)
    inlet = a["face_boundary"] == 1
    assert np.all(np.abs(a["face_cx"][inlet]) < 1e-6)
    outlet = a["face_boundary"] == 2
    assert np.all(np.abs(a["face_cx"][outlet] - 3.5) < 1e-6)


def test_channel_obstacle_mesh_area_and_determinism():
    geo = ChannelWithObstacle(length=3.0, height=1.0, obstacle_center=(1.0, 0.51), obstacle_radius=0.1)
    m1 = generate_cut_cell_mesh(geo, 0.02, 0.02, 1.2, (3.0, 1.0))
    m1.smooth(geo, 0.3, 30)
    m2 = bench_channel(0.02, 30)
    _check_structure(m1, 3.0 - math.pi * 0.01, rtol=1e-4)  # polygonal circle
    a1, a2 = m1.arrays(), m2.arrays()
    for k in a1:
        assert np.array_equal(a1[k], a2[k]), k


def test_bench_cell_count_formula():
    """N ~ 2.9686 / h^2 for the benchmark geometry (partial edge cells: <3%)."""
    for h in (0.0172, 0.01):
        m = bench_channel(h, 0)
        assert abs(m.num_cells() - 2.9686 / h ** 2) / (2.9686 / h ** 2) < 0.03


def test_save_load_roundtrip():
    m = backwards_step()
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "m.bin")
        m.save(p)
        m2 = Mesh.load(p)
        a, b = m.arrays(), m2.arrays()
        for k in a:
            assert np.array_equal(a[k], b[k]), k
        assert m2.calculate_max_skewness() == m.calculate_max_skewness()


def test_shared_view_file_round_trip(tmp_path):
    """bench.py --gpus N: rank 0 writes the mesh view once, every rank maps it
    (cfd2_amd.mesh.save_view_file / MappedMesh); the mapped view must hold
    exactly the generated arrays."""
    import numpy as np
    from cfd2_amd.mesh import MappedMesh, bench_channel, save_view_file
    m = bench_channel(0.02, 20)
    p = str(tmp_path / "mesh.bin")
    save_view_file(m, p)
    mm = MappedMesh(p)
    assert (mm.num_cells(), mm.num_faces()) == (m.num_cells(), m.num_faces())
    a, b = m.arrays(), mm.arrays()
    for k in a:
        assert np.array_equal(a[k], b[k]), k
    v = mm.view()
    assert v.num_cells == m.num_cells() and v.num_faces == m.num_faces()
    assert v.cell_vol[0] == a["cell_vol"][0] and v.cell_faces[5] == a["cell_faces"][5]


def test_load_rejects_truncated_and_inconsistent_files(tmp_path):
    """cfd_mesh_load trusts nothing in the file: a truncated file, a count larger
    than the file, and arrays whose lengths disagree are all CFD_ERR_INVALID
    (no allocation from an unchecked count, no out-of-range reads later)."""
    import struct
    m = backwards_step()
    p = str(tmp_path / "m.bin")
    m.save(p)
    raw = open(p, "rb").read()
    # truncated
    bad = str(tmp_path / "trunc.bin")
    open(bad, "wb").write(raw[: len(raw) // 2])
    with pytest.raises(RuntimeError, match="status 1"):
        Mesh.load(bad)
    # first array count (vx) blown up to 2^60 entries
    bad2 = str(tmp_path / "count.bin")
    open(bad2, "wb").write(raw[:8] + struct.pack("<Q", 1 << 60) + raw[16:])
    with pytest.raises(RuntimeError, match="status 1"):
        Mesh.load(bad2)
    # a well-formed file whose cell arrays disagree in length: drop one cell_vol entry
    a = m.arrays()
    n = m.num_cells()
    # field order of MESH_FIELDS: vx vy v_fixed face_v1 face_v2 face_owner face_neighbor face_boundary
    # face_nx face_ny face_area face_cx face_cy cell_cx cell_cy cell_vol ...; walk to cell_vol
    off = 8
    sizes = {"vx": 8, "vy": 8, "v_fixed": 1, "face_v1": 4, "face_v2": 4, "face_owner": 4, "face_neighbor": 4,
             "face_boundary": 4, "face_nx": 8, "face_ny": 8, "face_area": 8, "face_cx": 8, "face_cy": 8,
             "cell_cx": 8, "cell_cy": 8}
    for name, sz in sizes.items():
        cnt = struct.unpack_from("<Q", raw, off)[0]
        off += 8 + cnt * sz
    cnt = struct.unpack_from("<Q", raw, off)[0]
    assert cnt == n == len(a["cell_vol"])
    body = raw[off + 8: off + 8 + (n - 1) * 8]
    rest = raw[off + 8 + n * 8:]
    bad3 = str(tmp_path / "len.bin")
    open(bad3, "wb").write(raw[:off] + struct.pack("<Q", n - 1) + body + rest)
    with pytest.raises(RuntimeError, match="inconsistent"):
        Mesh.load(bad3)
