"""Hand-built meshes for edge cases (a Mesh-like object over numpy arrays):
single cell, a 1-D strip of cells, and deliberately broken meshes."""
import ctypes as C

import numpy as np

from cfd2_amd import _ffi

NONE = 0xFFFFFFFF


class ArrayMesh:
    """Same surface as cfd2_amd.Mesh (view / num_cells / num_faces / arrays)."""

    def __init__(self, **arrays):
        self._a = {k: np.ascontiguousarray(v) for k, v in arrays.items()}

    def arrays(self):
        return self._a

    def num_cells(self):
        return len(self._a["cell_cx"])

    def num_faces(self):
        return len(self._a["face_cx"])

    def view(self):
        a = self._a
        u32 = lambda k: a[k].ctypes.data_as(C.POINTER(C.c_uint32))  # noqa: E731
        f64 = lambda k: a[k].ctypes.data_as(C.POINTER(C.c_double))  # noqa: E731
        return _ffi.MeshView(self.num_cells(), self.num_faces(), u32("face_owner"), u32("face_neighbor"),
                             u32("face_boundary"), f64("face_area"), f64("face_nx"), f64("face_ny"),
                             f64("face_cx"), f64("face_cy"), f64("cell_cx"), f64("cell_cy"),
                             f64("cell_vol"), u32("cell_face_offsets"), u32("cell_faces"))


def strip(n, h=0.1):
    """n unit cells in a row along x: inlet on the left, outlet on the right,
    walls top and bottom (cell faces listed owner-side first)."""
    owner, nb, bt, area, nx, ny, fx, fy = [], [], [], [], [], [], [], []
    cell_faces = [[] for _ in range(n)]

    def face(o, ngh, b, a, nxx, nyy, cx, cy):
        f = len(owner)
        owner.append(o), nb.append(ngh), bt.append(b), area.append(a)
        nx.append(nxx), ny.append(nyy), fx.append(cx), fy.append(cy)
        cell_faces[o].append(f)
        if ngh != NONE:
            cell_faces[ngh].append(f)

    for i in range(n):
        x0 = i * h
        if i == 0:
            face(i, NONE, 1, h, -1.0, 0.0, x0, 0.5 * h)  # inlet
        face(i, NONE, 3, h, 0.0, -1.0, x0 + 0.5 * h, 0.0)  # bottom wall
        face(i, NONE, 3, h, 0.0, 1.0, x0 + 0.5 * h, h)  # top wall
        if i + 1 < n:
            face(i, i + 1, 0, h, 1.0, 0.0, x0 + h, 0.5 * h)
        else:
            face(i, NONE, 2, h, 1.0, 0.0, x0 + h, 0.5 * h)  # outlet
    offs = np.zeros(n + 1, dtype=np.uint32)
    for i in range(n):
        offs[i + 1] = offs[i] + len(cell_faces[i])
    return ArrayMesh(
        face_owner=np.array(owner, np.uint32), face_neighbor=np.array(nb, np.uint32),
        face_boundary=np.array(bt, np.uint32), face_area=np.array(area), face_nx=np.array(nx),
        face_ny=np.array(ny), face_cx=np.array(fx), face_cy=np.array(fy),
        cell_cx=np.array([(i + 0.5) * h for i in range(n)]), cell_cy=np.full(n, 0.5 * h),
        cell_vol=np.full(n, h * h), cell_face_offsets=offs,
        cell_faces=np.array([f for cf in cell_faces for f in cf], np.uint32))


def broken(kind):
    m = strip(4)
    a = {k: v.copy() for k, v in m.arrays().items()}
    if kind == "owner_range":
        a["face_owner"][0] = 99
    elif kind == "neighbor_range":
        i = int(np.nonzero(a["face_neighbor"] != NONE)[0][0])
        a["face_neighbor"][i] = 77
    elif kind == "cell_faces_range":
        a["cell_faces"][0] = 1000
    elif kind == "empty":
        for k in a:
            a[k] = a[k][:0] if k != "cell_face_offsets" else np.zeros(1, np.uint32)
    return ArrayMesh(**a)


def max_ranks(n):
    """Most ranks a mesh of n cells can take: one segment of the canonical
    reduction tree each (kernels.hpp red_geom)."""
    g = 0
    while g < 8 and (n >> (g + 1)) >= 16384:
        g += 1
    nch = -(-n // 256)
    return -(-nch // (1 << g))
