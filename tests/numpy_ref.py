"""Independent vectorised numpy restatement of prepare_coupled.wgsl:63-348 and
coupled_assembly_merged.wgsl:70-463 (Upwind + Euler), written face-wise
rather than cell-wise.  TEST INFRASTRUCTURE ONLY: a second, independently
written restatement used to cross-check the oracle (summation order differs,
so agreement is checked with a tolerance, not bit-for-bit)."""
import numpy as np

f32 = np.float32


def _dist(ax, ay, bx, by):
    dx, dy = ax - bx, ay - by
    return np.sqrt(dx * dx + dy * dy)


def mesh_f32(a):
    return dict(
        own=a["face_owner"].astype(np.int64),
        nb=np.where(a["face_neighbor"].astype(np.int64) == 0xFFFFFFFF, -1,
                    a["face_neighbor"].astype(np.int64)),
        bt=a["face_boundary"].astype(np.int64),
        A=a["face_area"].astype(f32), nx=a["face_nx"].astype(f32), ny=a["face_ny"].astype(f32),
        fx=a["face_cx"].astype(f32), fy=a["face_cy"].astype(f32),
        cx=a["cell_cx"].astype(f32), cy=a["cell_cy"].astype(f32), vol=a["cell_vol"].astype(f32),
    )


def prepare(m, u, p, dp, gp, c):
    """Returns fluxes[F], d_p[N], grad_p[N,2], grad_u[N,2], grad_v[N,2]."""
    own, nb, bt = m["own"], m["nb"], m["bt"]
    A, nx, ny, fx, fy, cx, cy, vol = (m[k] for k in ("A", "nx", "ny", "fx", "fy", "cx", "cy", "vol"))
    N = len(vol)
    internal = nb >= 0
    nbi = np.where(internal, nb, own)
    cox, coy = cx[own], cy[own]
    flip = ((fx - cox) * nx + (fy - coy) * ny) < 0
    nfx, nfy = np.where(flip, -nx, nx), np.where(flip, -ny, ny)
    d_own = _dist(cox, coy, fx, fy)
    d_ngh = _dist(cx[nbi], cy[nbi], fx, fy)
    tot = d_own + d_ngh
    lam = np.where(tot > f32(1e-6), d_ngh / np.where(tot > 0, tot, 1), f32(0.5)).astype(f32)
    om = f32(1) - lam
    ufx = lam * u[own, 0] + om * u[nbi, 0]
    ufy = lam * u[own, 1] + om * u[nbi, 1]
    dpf = lam * dp[own] + om * dp[nbi]
    gfx = lam * gp[own, 0] + om * gp[nbi, 0]
    gfy = lam * gp[own, 1] + om * gp[nbi, 1]
    dist = np.maximum(np.abs((cx[nbi] - cox) * nfx + (cy[nbi] - coy) * nfy), f32(1e-6))
    rc = dpf * A * ((gfx * nfx + gfy * nfy) - (p[nbi] - p[own]) / dist)
    flux_int = f32(c.density) * ((ufx * nfx + ufy * nfy) * A + rc)
    t = np.clip((f32(c.time) - 0) / f32(c.ramp_time), 0, 1).astype(f32)
    ramp = t * t * (f32(3) - f32(2) * t)
    ub = f32(c.inlet_velocity) * ramp
    flux_in = f32(c.density) * (ub * nfx) * A
    flux_out = np.maximum(f32(0), f32(c.density) * (u[own, 0] * nfx + u[own, 1] * nfy) * A)
    flux = np.where(internal, flux_int, np.where(bt == 1, flux_in, np.where(bt == 2, flux_out, f32(0))))
    flux = flux.astype(f32)

    diag = (vol * f32(c.density) / f32(c.dt)).astype(np.float64)
    gp_acc = np.zeros((N, 2))
    gu_acc = np.zeros((N, 2))
    gv_acc = np.zeros((N, 2))
    for side in (0, 1):  # owner side, neighbour side
        cell = own if side == 0 else nb
        mask = np.ones_like(internal) if side == 0 else internal
        cell = np.where(mask, cell, 0)
        other = np.where(side == 0, nbi, own)
        sgn = f32(1) if side == 0 else f32(-1)
        fo = sgn * flux
        ocx = np.where(internal, cx[other], fx)
        ocy = np.where(internal, cy[other], fy)
        dist_e = np.sqrt((ocx - cx[cell]) ** 2 + (ocy - cy[cell]) ** 2)
        diff = f32(c.viscosity) * A / dist_e
        conv = np.maximum(fo, 0)
        contrib = np.where(internal, diff + conv,
                           np.where((bt == 1) | (bt == 3), diff + conv, np.where(bt == 2, conv, 0)))
        np.add.at(diag, cell[mask], contrib[mask])
        d_c = _dist(cx[cell], cy[cell], fx, fy)
        d_o = _dist(ocx, ocy, fx, fy)
        lp = np.where(d_c + d_o > 1e-6, d_o / np.maximum(d_c + d_o, 1e-30), 0.5)
        vp = np.where(internal, lp * p[cell] + (1 - lp) * p[other], np.where(bt == 2, 0, p[cell]))
        vu = np.where(internal, lp * u[cell, 0] + (1 - lp) * u[other, 0],
                      np.where(bt == 1, ub, np.where(bt == 3, 0, u[cell, 0])))
        vv = np.where(internal, lp * u[cell, 1] + (1 - lp) * u[other, 1],
                      np.where(bt == 1, 0, np.where(bt == 3, 0, u[cell, 1])))
        snx, sny = sgn * nx, sgn * ny
        for acc, val in ((gp_acc, vp), (gu_acc, vu), (gv_acc, vv)):
            np.add.at(acc[:, 0], cell[mask], (val * snx * A)[mask])
            np.add.at(acc[:, 1], cell[mask], (val * sny * A)[mask])
    d_p = np.where(np.abs(diag) > 1e-20, vol / diag, 0)
    return flux, d_p, gp_acc / vol[:, None], gu_acc / vol[:, None], gv_acc / vol[:, None]


def assemble(m, srow, scol, flux, u_old, dp, c):
    """Coupled CSR values [9 nnz_s], rhs [3N], scalar values [nnz_s] (Upwind, Euler).
    Off-diagonal entries are last-write-wins per (cell, neighbour) in face order."""
    own, nb, bt = m["own"], m["nb"], m["bt"]
    A, nx, ny, fx, fy, cx, cy, vol = (m[k] for k in ("A", "nx", "ny", "fx", "fy", "cx", "cy", "vol"))
    N = len(vol)
    internal = nb >= 0
    nbi = np.where(internal, nb, own)
    nnz = len(scol)
    mv = np.zeros(9 * nnz)
    sv = np.zeros(nnz)
    rhs = np.zeros(3 * N)
    dg = np.zeros(N)
    sup, svp, spu, spv, spp, sdiag = (np.zeros(N) for _ in range(6))
    ct = vol * f32(c.density) / f32(c.dt)
    dg += ct
    rhs[0::3] += ct * u_old[:, 0]
    rhs[1::3] += ct * u_old[:, 1]
    t = np.clip(f32(c.time) / f32(c.ramp_time), 0, 1)
    ub = c.inlet_velocity * t * t * (3 - 2 * t)

    def slot(i, j):
        a, b = srow[i], srow[i + 1]
        return a + np.searchsorted(scol[a:b], j), b - a

    F = len(A)
    for f in range(F):  # face order == last-write-wins order per cell
        for side in ((0,) if nb[f] < 0 else (0, 1)):
            i = own[f] if side == 0 else nb[f]
            s = 1.0 if side == 0 else -1.0
            nX, nY = s * nx[f], s * ny[f]
            fl = s * flux[f]
            if nb[f] >= 0:
                o = nb[f] if side == 0 else own[f]
                ox, oy = cx[o], cy[o]
            else:
                ox, oy = fx[f], fy[f]
            dist = max(abs((ox - cx[i]) * nX + (oy - cy[i]) * nY), 1e-6)
            diff = c.viscosity * A[f] / dist
            cd, co = (fl, 0.0) if fl > 0 else (0.0, fl)
            if nb[f] >= 0:
                k, nbr = slot(i, o)
                r = k - srow[i]
                base = 9 * srow[i]
                d_o = np.hypot(ox - fx[f], oy - fy[f])
                d_c = np.hypot(cx[i] - fx[f], cy[i] - fy[f])
                lam = d_o / (d_c + d_o) if d_c + d_o > 1e-6 else 0.5
                mv[base + 3 * r + 0] = -diff + co
                mv[base + 3 * r + 1] = 0
                mv[base + 3 * nbr + 3 * r + 0] = 0
                mv[base + 3 * nbr + 3 * r + 1] = -diff + co
                dg[i] += diff + cd
                mv[base + 3 * r + 2] = (1 - lam) * A[f] * nX
                mv[base + 3 * nbr + 3 * r + 2] = (1 - lam) * A[f] * nY
                mv[base + 6 * nbr + 3 * r + 0] = (1 - lam) * A[f] * nX
                mv[base + 6 * nbr + 3 * r + 1] = (1 - lam) * A[f] * nY
                sup[i] += lam * A[f] * nX
                svp[i] += lam * A[f] * nY
                spu[i] += lam * A[f] * nX
                spv[i] += lam * A[f] * nY
                dpf = lam * dp[i] + (1 - lam) * dp[o]
                lap = dpf * A[f] / dist
                mv[base + 6 * nbr + 3 * r + 2] = -lap
                spp[i] += lap
                sv[k] = -c.density * dpf * A[f] / dist
                sdiag[i] += c.density * dpf * A[f] / dist
            elif bt[f] == 1:
                dg[i] += diff
                rhs[3 * i] += diff * ub
                if fl > 0:
                    dg[i] += fl
                else:
                    rhs[3 * i] -= fl * ub
                sup[i] += A[f] * nX
                svp[i] += A[f] * nY
                rhs[3 * i + 2] -= ub * nX * A[f]
            elif bt[f] == 3:
                dg[i] += diff
                sup[i] += A[f] * nX
                svp[i] += A[f] * nY
            elif bt[f] == 2:
                if fl > 0:
                    dg[i] += fl
                spu[i] += nX * A[f]
                spv[i] += nY * A[f]
                spp[i] += dp[i] * A[f] / dist
                sdiag[i] += c.density * dp[i] * A[f] / dist
    for i in range(N):
        k, nbr = slot(i, i)
        r = k - srow[i]
        base = 9 * srow[i]
        mv[base + 3 * r + 0] = dg[i]
        mv[base + 3 * r + 2] = sup[i]
        mv[base + 3 * nbr + 3 * r + 1] = dg[i]
        mv[base + 3 * nbr + 3 * r + 2] = svp[i]
        mv[base + 6 * nbr + 3 * r + 0] = spu[i]
        mv[base + 6 * nbr + 3 * r + 1] = spv[i]
        mv[base + 6 * nbr + 3 * r + 2] = spp[i]
        sv[k] = sdiag[i]
    return mv, rhs, sv


def scalar_csr(a):
    """init/mesh.rs:27-53."""
    N = len(a["cell_cx"])
    own = a["face_owner"].astype(np.int64)
    nb = a["face_neighbor"].astype(np.int64)
    internal = nb != 0xFFFFFFFF
    rows = [set([i]) for i in range(N)]
    for o, n in zip(own[internal], nb[internal]):
        rows[o].add(n)
        rows[n].add(o)
    srow = np.zeros(N + 1, dtype=np.int64)
    cols = []
    for i in range(N):
        r = sorted(rows[i])
        srow[i + 1] = srow[i] + len(r)
        cols.extend(r)
    return srow, np.asarray(cols, dtype=np.int64)
