"""Seeded polygonal (Voronoi) test meshes -- SURVEY §8(f) rank 4 as TEST INPUT:
the reference's Delaunay/Voronoi generator uses an unseeded RNG, so its meshes
cannot be reproduced; this builds a seeded bounded Voronoi mesh of a
rectangular channel with scipy (mirror points across the four walls so every
cell of an original point is clipped exactly by the box) to exercise the
solver on 4-9-face polygonal cells.  Boundary types: x = 0 inlet, x = L
outlet, y = 0 / H walls (as the reference channel)."""
import numpy as np

from tests.synthetic import NONE, ArrayMesh


def voronoi_channel(n_points=600, length=3.0, height=1.0, seed=12345, jitter=0.35):
    from scipy.spatial import Voronoi
    rng = np.random.default_rng(seed)
    # jittered lattice (bounded cell quality), sorted x-major like the cut-cell mesher
    nx = max(2, int(round(np.sqrt(n_points * length / height))))
    ny = max(2, int(round(n_points / nx)))
    hx, hy = length / nx, height / ny
    gx, gy = np.meshgrid((np.arange(nx) + 0.5) * hx, (np.arange(ny) + 0.5) * hy, indexing="ij")
    pts = np.stack([gx.ravel(), gy.ravel()], 1)
    pts += rng.uniform(-jitter, jitter, pts.shape) * np.array([hx, hy])
    n = len(pts)
    mir = [pts * [-1, 1], pts * [1, -1], np.stack([2 * length - pts[:, 0], pts[:, 1]], 1),
           np.stack([pts[:, 0], 2 * height - pts[:, 1]], 1)]
    allp = np.concatenate([pts] + mir)
    vor = Voronoi(allp)
    V = vor.vertices
    owner, nb, bt, area, fnx, fny, fcx, fcy = [], [], [], [], [], [], [], []
    cell_faces = [[] for _ in range(n)]
    for (a, b), rv in zip(vor.ridge_points, vor.ridge_vertices):
        if a >= n and b >= n:
            continue
        if -1 in rv:
            continue
        if a >= n:
            a, b = b, a  # a is an original point
        p0, p1 = V[rv[0]], V[rv[1]]
        ln = float(np.hypot(*(p1 - p0)))
        if ln < 1e-12:
            continue
        d = allp[b] - allp[a]
        nrm = d / np.linalg.norm(d)  # out of the owner a
        c = 0.5 * (p0 + p1)
        f = len(owner)
        if b < n:
            o, g = (a, b) if a < b else (b, a)
            if o != a:
                nrm = -nrm
            owner.append(o), nb.append(g), bt.append(0)
            cell_faces[o].append(f), cell_faces[g].append(f)
        else:
            side = (b - n) // n  # mirror block: 0 x=0, 1 y=0, 2 x=L, 3 y=H
            owner.append(a), nb.append(NONE), bt.append({0: 1, 1: 3, 2: 2, 3: 3}[side])
            cell_faces[a].append(f)
        area.append(ln), fnx.append(nrm[0]), fny.append(nrm[1]), fcx.append(c[0]), fcy.append(c[1])
    # cell geometry: polygon area / centroid of the clipped region
    cx, cy, vol = np.zeros(n), np.zeros(n), np.zeros(n)
    for i in range(n):
        reg = vor.regions[vor.point_region[i]]
        P = V[reg]
        ang = np.arctan2(P[:, 1] - pts[i, 1], P[:, 0] - pts[i, 0])
        P = P[np.argsort(ang)]
        x, y = P[:, 0], P[:, 1]
        xs, ys = np.roll(x, -1), np.roll(y, -1)
        cr = x * ys - xs * y
        A = 0.5 * cr.sum()
        vol[i] = A
        cx[i] = ((x + xs) * cr).sum() / (6 * A)
        cy[i] = ((y + ys) * cr).sum() / (6 * A)
    offs = np.zeros(n + 1, dtype=np.uint32)
    for i in range(n):
        offs[i + 1] = offs[i] + len(cell_faces[i])
    return ArrayMesh(
        face_owner=np.array(owner, np.uint32), face_neighbor=np.array(nb, np.uint32),
        face_boundary=np.array(bt, np.uint32), face_area=np.array(area), face_nx=np.array(fnx),
        face_ny=np.array(fny), face_cx=np.array(fcx), face_cy=np.array(fcy), cell_cx=cx, cell_cy=cy,
        cell_vol=vol, cell_face_offsets=offs,
        cell_faces=np.array([f for cf in cell_faces for f in cf], np.uint32))
