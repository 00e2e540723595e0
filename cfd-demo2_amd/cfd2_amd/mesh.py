"""Mesh input of the hot path: mirror of ``cfd2::solver::mesh``.

``generate_cut_cell_mesh`` / ``Mesh.smooth`` run the native C++ restatement of
src/solver/mesh/cut_cell.rs:10-510 and structs.rs:159-292 (deterministic, f64).
Arrays are exposed as zero-copy numpy views of the native mesh.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

from . import _ffi


@dataclass
class BackwardsStep:  # geometry.rs:121-126
    length: float
    height_inlet: float
    height_outlet: float
    step_x: float

    def _geo(self) -> _ffi.Geometry:
        g = _ffi.Geometry(kind=0)
        g.p[:4] = [self.length, self.height_inlet, self.height_outlet, self.step_x]
        return g


@dataclass
class ChannelWithObstacle:  # geometry.rs:32-37
    length: float
    height: float
    obstacle_center: tuple
    obstacle_radius: float

    def _geo(self) -> _ffi.Geometry:
        g = _ffi.Geometry(kind=1)
        g.p[:5] = [self.length, self.height, self.obstacle_center[0], self.obstacle_center[1],
                   self.obstacle_radius]
        return g


@dataclass
class RectangularChannel:  # geometry.rs:216-219
    length: float
    height: float

    def _geo(self) -> _ffi.Geometry:
        g = _ffi.Geometry(kind=2)
        g.p[:2] = [self.length, self.height]
        return g


@dataclass
class CircleObstacle:  # src/solver/mesh/tests.rs:4-10
    center: tuple
    radius: float
    domain_min: tuple
    domain_max: tuple

    def _geo(self) -> _ffi.Geometry:
        g = _ffi.Geometry(kind=3)
        g.p[:7] = [self.center[0], self.center[1], self.radius, self.domain_min[0],
                   self.domain_min[1], self.domain_max[0], self.domain_max[1]]
        return g


def _np(ptr, n, dtype):
    if n == 0:
        return np.zeros(0, dtype=dtype)
    return np.ctypeslib.as_array(ptr, shape=(n,)).view(dtype)


class Mesh:
    """Owned native mesh (``cfd2::solver::mesh::Mesh``)."""

    def __init__(self, handle: int):
        self._h = C.c_void_p(handle)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            _ffi.lib().cfd_mesh_destroy(h)
            self._h = None

    @property
    def handle(self) -> C.c_void_p:
        return self._h

    def view(self) -> _ffi.MeshView:
        v = _ffi.MeshView()
        _ffi.check(_ffi.lib().cfd_mesh_get_view(self._h, C.byref(v)), "cfd_mesh_get_view")
        return v

    def num_cells(self) -> int:
        return int(self.view().num_cells)

    def num_faces(self) -> int:
        return int(self.view().num_faces)

    def arrays(self) -> dict:
        v = self.view()
        n, f = v.num_cells, v.num_faces
        offs = _np(v.cell_face_offsets, n + 1, np.uint32)
        s = int(offs[-1]) if n else 0
        return dict(
            face_owner=_np(v.face_owner, f, np.uint32),
            face_neighbor=_np(v.face_neighbor, f, np.uint32),
            face_boundary=_np(v.face_boundary, f, np.uint32),
            face_area=_np(v.face_area, f, np.float64),
            face_nx=_np(v.face_nx, f, np.float64),
            face_ny=_np(v.face_ny, f, np.float64),
            face_cx=_np(v.face_cx, f, np.float64),
            face_cy=_np(v.face_cy, f, np.float64),
            cell_cx=_np(v.cell_cx, n, np.float64),
            cell_cy=_np(v.cell_cy, n, np.float64),
            cell_vol=_np(v.cell_vol, n, np.float64),
            cell_face_offsets=offs,
            cell_faces=_np(v.cell_faces, s, np.uint32),
        )

    def vertices(self):
        nv = C.c_uint32()
        vx, vy = _ffi.f64p(), _ffi.f64p()
        vf = C.POINTER(C.c_uint8)()
        _ffi.check(_ffi.lib().cfd_mesh_get_vertices(self._h, C.byref(nv), C.byref(vx), C.byref(vy),
                                                      C.byref(vf)), "cfd_mesh_get_vertices")
        n = nv.value
        return _np(vx, n, np.float64), _np(vy, n, np.float64), _np(vf, n, np.uint8).astype(bool)

    def topology(self) -> dict:
        """face_v1, face_v2, cell_vertex_offsets, cell_vertices (CCW polygons)."""
        p = [C.POINTER(C.c_uint32)() for _ in range(4)]
        _ffi.check(_ffi.lib().cfd_mesh_get_topology(self._h, *[C.byref(q) for q in p]), "cfd_mesh_get_topology")
        nf, n = self.num_faces(), self.num_cells()
        offs = _np(p[2], n + 1, np.uint32)
        return dict(face_v1=_np(p[0], nf, np.uint32), face_v2=_np(p[1], nf, np.uint32), cell_vertex_offsets=offs,
                    cell_vertices=_np(p[3], int(offs[-1]) if n else 0, np.uint32))

    def smooth(self, geo, target_skew: float, max_iterations: int) -> int:
        it = C.c_int32()
        g = geo._geo()
        _ffi.check(_ffi.lib().cfd_mesh_smooth(self._h, C.byref(g), target_skew, max_iterations,
                                              C.byref(it)), "cfd_mesh_smooth")
        return it.value

    def calculate_max_skewness(self) -> float:
        return float(_ffi.lib().cfd_mesh_max_skewness(self._h))

    def save(self, path: str) -> None:
        _ffi.check(_ffi.lib().cfd_mesh_save(self._h, path.encode()), "cfd_mesh_save")

    @staticmethod
    def load(path: str) -> "Mesh":
        h = C.c_void_p()
        _ffi.check(_ffi.lib().cfd_mesh_load(path.encode(), C.byref(h)), "cfd_mesh_load")
        return Mesh(h.value)


def generate_cut_cell_mesh(geo, min_cell_size: float, max_cell_size: float, growth_rate: float,
                           domain_size) -> Mesh:
    """cut_cell.rs:10-16."""
    h = C.c_void_p()
    g = geo._geo()
    _ffi.check(_ffi.lib().cfd_mesh_generate_cut_cell(C.byref(g), min_cell_size, max_cell_size,
                                                     growth_rate, float(domain_size[0]),
                                                     float(domain_size[1]), C.byref(h)),
               "cfd_mesh_generate_cut_cell")
    return Mesh(h.value)


def generate_voronoi_mesh(geo, min_cell_size: float, max_cell_size: float, growth_rate: float,
                          domain_size, seed: int = 12345) -> Mesh:
    """voronoi.rs:23 (seeded restatement: same seed, same mesh)."""
    h = C.c_void_p()
    g = geo._geo()
    _ffi.check(_ffi.lib().cfd_mesh_generate_voronoi(C.byref(g), min_cell_size, max_cell_size, growth_rate,
                                                    float(domain_size[0]), float(domain_size[1]),
                                                    int(seed), C.byref(h)),
               "cfd_mesh_generate_voronoi")
    return Mesh(h.value)


def generate_delaunay_mesh(geo, min_cell_size: float, max_cell_size: float, growth_rate: float,
                           domain_size, seed: int = 12345) -> Mesh:
    """delaunay.rs:732 (seeded restatement; triangle cells)."""
    h = C.c_void_p()
    g = geo._geo()
    _ffi.check(_ffi.lib().cfd_mesh_generate_delaunay(C.byref(g), min_cell_size, max_cell_size, growth_rate,
                                                     float(domain_size[0]), float(domain_size[1]),
                                                     int(seed), C.byref(h)),
               "cfd_mesh_generate_delaunay")
    return Mesh(h.value)


def channel_obstacle_h(target_cells: float) -> float:
    """Cell size h for a ~target_cells channel+obstacle mesh (N ≈ 2.9686/h²)."""
    return float(np.sqrt(2.9686 / target_cells))


C0_VORONOI_H = 0.0138  # ~10.1 k cells (BASELINE configs[0]: "~10k Voronoi cells")


def bench_voronoi_channel(h: float = C0_VORONOI_H, seed: int = 12345) -> Mesh:
    """BASELINE configs[0]: the same ChannelWithObstacle{3x1, (1.0,0.51), r 0.1}
    meshed by the seeded Voronoi generator (voronoi.rs:23-721 restated,
    cfd_mesh_generate_voronoi) with min = max = h: 10,106 polygonal cells at
    the default h."""
    geo = ChannelWithObstacle(length=3.0, height=1.0, obstacle_center=(1.0, 0.51),
                              obstacle_radius=0.1)
    return generate_voronoi_mesh(geo, h, h, 1.2, (3.0, 1.0), seed=seed)


def bench_channel(h: float, smooth_iters: int = 100) -> Mesh:
    """SURVEY §8(d) synthetic input: ChannelWithObstacle{3x1, (1.0,0.51), r 0.1},
    cut-cell with min=max=h, growth 1.2, then smooth(0.3, 100)."""
    geo = ChannelWithObstacle(length=3.0, height=1.0, obstacle_center=(1.0, 0.51),
                              obstacle_radius=0.1)
    m = generate_cut_cell_mesh(geo, h, h, 1.2, (3.0, 1.0))
    if smooth_iters > 0:
        m.smooth(geo, 0.3, smooth_iters)
    return m


# ---------------------------------------------------------------------------
# Shared mesh file for one-process-per-GPU runs: rank 0 writes the SoA arrays
# of the mesh view once (page-aligned raw arrays + a JSON header) and every
# rank maps them read-only, so the ranks share ONE copy in the page cache
# instead of each holding (and generating) the whole mesh.  Only the fields
# of cfd_mesh_view are stored (what cfd_solver_create_dist reads).
_VIEW_FIELDS = [  # (name, dtype, length: "F" faces, "N" cells, "N1" cells + 1, "S" cell-face entries)
    ("face_owner", np.uint32, "F"), ("face_neighbor", np.uint32, "F"), ("face_boundary", np.uint32, "F"),
    ("face_area", np.float64, "F"), ("face_nx", np.float64, "F"), ("face_ny", np.float64, "F"),
    ("face_cx", np.float64, "F"), ("face_cy", np.float64, "F"),
    ("cell_cx", np.float64, "N"), ("cell_cy", np.float64, "N"), ("cell_vol", np.float64, "N"),
    ("cell_face_offsets", np.uint32, "N1"), ("cell_faces", np.uint32, "S"),
]
_PAGE = 4096


def save_view_file(mesh: "Mesh", path: str) -> None:
    import json
    a = mesh.arrays()
    n, f = mesh.num_cells(), mesh.num_faces()
    s = int(a["cell_face_offsets"][-1])
    lens = {"F": f, "N": n, "N1": n + 1, "S": s}
    hdr, off = {"num_cells": n, "num_faces": f, "arrays": {}}, _PAGE
    for name, dt, ln in _VIEW_FIELDS:
        nbytes = lens[ln] * np.dtype(dt).itemsize
        hdr["arrays"][name] = [off, lens[ln], np.dtype(dt).str]
        off += (nbytes + _PAGE - 1) // _PAGE * _PAGE
    raw = json.dumps(hdr).encode()
    assert len(raw) < _PAGE
    with open(path + ".tmp", "wb") as fh:
        fh.write(raw)
        for name, _, _ in _VIEW_FIELDS:
            fh.seek(hdr["arrays"][name][0])
            np.ascontiguousarray(a[name]).tofile(fh)
        fh.truncate(off)
    os.replace(path + ".tmp", path)  # readers never see a partial file


class MappedMesh:
    """A mesh view backed by a file of save_view_file (read-only memory map):
    what GpuSolver.create_dist / create_dist_host need (view, sizes)."""

    def __init__(self, path: str):
        import json
        with open(path, "rb") as fh:
            hdr = json.loads(fh.read(_PAGE).split(b"\0", 1)[0].decode())
        self._n, self._f = int(hdr["num_cells"]), int(hdr["num_faces"])
        self._a = {name: np.memmap(path, dtype=np.dtype(dt), mode="r", offset=off, shape=(ln,))
                   for name, (off, ln, dt) in hdr["arrays"].items()}

    def num_cells(self) -> int:
        return self._n

    def num_faces(self) -> int:
        return self._f

    def arrays(self) -> dict:
        return dict(self._a)

    def view(self) -> _ffi.MeshView:
        v = _ffi.MeshView()
        v.num_cells, v.num_faces = self._n, self._f
        for name, dt, _ in _VIEW_FIELDS:
            ct = C.c_uint32 if dt == np.uint32 else C.c_double
            setattr(v, name, self._a[name].ctypes.data_as(C.POINTER(ct)))
        return v
