"""The reference's own WGSL kernels, run on the CPU -- TEST INFRASTRUCTURE ONLY.

`WgslRefSolver` executes the reference's hot-path shaders
(src/solver/gpu/shaders/{prepare_coupled, coupled_assembly_merged,
update_fields_from_coupled, schur_precond, amg, gmres_ops, gmres_cgs,
gmres_logic}.wgsl, read from /root/reference) with oracle/wgsl/wgsl_exec.py,
and restates only the Rust host around them: the buffers and bind groups of
init/mesh.rs, init/fields.rs, init/linear_solver/mod.rs and
coupled_solver_fgmres.rs:212-1284, the dispatch sequence of step_coupled
(coupled_solver.rs:33-499) and solve_coupled_fgmres
(coupled_solver_fgmres.rs:1728-2448, with gpu_norm :1444-1588 and
compute_residual_into :1637-1667), the AMG V-cycle encoding (amg.rs:666-770)
and check_evolution (coupled_solver.rs:501-580).  The AMG hierarchy (amg.rs
host setup) and the mesh upload tables come from tests/refpy.py, whose
agreement with the oracle test_refpy.py establishes.

So every floating-point operation of a step happens inside the reference's
shader text, under the schedule oracle/wgsl/wgsl_exec.py describes
(workgroups in dispatch order, a workgroup's lanes in lockstep, wgpu's
Restrict bounds policy).  The oracle reproduces that schedule with its
reference-semantics flags 15 (in-place AMG smoother, racy prepare reads,
the reference's reduction order, restrict_residual's clamped rows --
oracle.cpp kSem*), so `oracle(flags 15) == WgslRefSolver` bit for bit pins
the oracle to the reference's kernels; the canonical mode (flags 0, what the
HIP path reproduces) differs from it only by those four documented
resolutions.

The async readbacks follow the oracle's deterministic lag model
(convergence_lag 0 / 1); fixed_outer / fixed_inner give the bench's fixed
schedule, as in refpy.RefSolver.
"""
from __future__ import annotations

import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
from wgsl.wgsl_exec import Binding, Dispatcher, Mem, buffer  # noqa: E402

from tests import refpy  # noqa: E402

REF_SHADERS = "/root/reference/src/solver/gpu/shaders"
F = np.float32
U = np.uint32
MAXU = 0xFFFFFFFF
WG = 64
_SHADERS = {}


def shader(name):
    """the reference shader `name`.wgsl, parsed once"""
    if name not in _SHADERS:
        path = os.path.join(REF_SHADERS, name + ".wgsl")
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path}: the reference is only present in the build container")
        with open(path) as f:
            _SHADERS[name] = Dispatcher(f.read())
    return _SHADERS[name]


def available():
    return os.path.isdir(REF_SHADERS)


def _f32bits(x):
    return int(np.array(x, F).view(U))


def _words(*vals):
    """uniform struct words: Python floats -> f32 bits, ints -> u32"""
    out = np.zeros(len(vals), U)
    for k, v in enumerate(vals):
        out[k] = _f32bits(v) if isinstance(v, (float, np.floating)) else (int(v) & MAXU)
    return out


def _wg(n):
    return -(-n // WG)


class WgslRefSolver(refpy.RefSolver):
    """refpy.RefSolver's surface; step() runs the reference's WGSL."""

    def __init__(self, mesh, fixed_outer=0, fixed_inner=0, convergence_lag=1, schedule="workgroups",
                 bounds="restrict", amg=None):
        """schedule / bounds: oracle/wgsl/wgsl_exec.py Dispatcher.dispatch --
        ("workgroups", "restrict") is the schedule of oracle flags 15,
        ("dispatch", "zero") the one of oracle flags 4 (reference reduction
        order, every other resolution canonical).  amg: (schedule, bounds) of
        the V-cycle's dispatches alone (every dispatch may run under its own
        schedule): ("workgroups", "restrict") with the rest ("dispatch",
        "zero") is oracle flags 13 (in-place smoother, restrict clamp,
        reference reductions; prepare's reads the snapshot)."""
        super().__init__(mesh, fixed_outer=fixed_outer, fixed_inner=fixed_inner, convergence_lag=convergence_lag)
        self.schedule, self.bounds = schedule, bounds
        self.amg_sched = amg or (schedule, bounds)
        M = self.M
        N, nf = M.N, len(M.area)
        self.N = N
        # --- init/mesh.rs: mesh buffers (f32), face_neighbor as u32 with u32::MAX
        offs = np.asarray(mesh.arrays()["cell_face_offsets"], np.int64)
        cfaces = np.asarray(mesh.arrays()["cell_faces"], np.int64)
        cfmi = np.full(len(cfaces), MAXU, U)
        for i in range(N):
            for k in range(offs[i + 1] - offs[i]):
                sm = M.slot_mat[i, k]
                if sm >= 0:
                    cfmi[offs[i] + k] = sm
        nb = np.where(M.nb < 0, MAXU, M.nb).astype(U)
        vec2 = lambda a, b: np.stack([a, b], 1).astype(F)  # noqa: E731
        self.mesh_b = {
            (0, 0): buffer(M.own.astype(U)), (0, 1): buffer(nb), (0, 2): buffer(M.area),
            (0, 3): buffer(vec2(M.nx, M.ny)), (0, 4): buffer(vec2(M.cx, M.cy)), (0, 5): buffer(M.vol),
            (0, 6): buffer(offs.astype(U)), (0, 7): buffer(cfaces.astype(U)), (0, 10): buffer(cfmi),
            (0, 11): buffer(M.diag_idx.astype(U)), (0, 12): buffer(M.bt.astype(U)),
            (0, 13): buffer(vec2(M.fx, M.fy)),
        }
        # --- init/fields.rs: three FluidState buffers (8 f32 per cell), fluxes, constants
        self.states = [Mem(8 * N) for _ in range(3)]
        self.state_step_index = 0
        self.fluxes = Mem(max(nf, 1))
        self.constants_b = Mem(14)
        # --- init/linear_solver/mod.rs: scalar CSR + values, coupled CSR + values, rhs, x, ...
        nnz_s = len(M.scol)
        self.s_row = buffer(M.srow.astype(U))
        self.s_col = buffer(M.scol.astype(U))
        self.s_val = Mem(nnz_s)
        self.c_row = buffer(M.crow.astype(U))
        self.c_col = buffer(M.ccol.astype(U))
        self.c_val = Mem(9 * nnz_s)
        self.rhs_b = Mem(3 * N)
        self.x_b = Mem(3 * N)
        self.grad_u = Mem(2 * N)
        self.grad_v = Mem(2 * N)
        self.diag_u = Mem(N)
        self.diag_v = Mem(N)
        self.diag_p = Mem(N)
        self.max_diff = Mem(2)
        # --- coupled_solver_fgmres.rs:212-1284 (max_restart 50)
        m = self.m
        n = 3 * N
        self.n = n
        self.ndg = _wg(n)  # num_dot_groups
        self.bstride = ((n * 4 + 255) & ~255) // 4
        self.basis = Mem(self.bstride * (m + 1))
        self.z = [Mem(n) for _ in range(m)]
        self.w = Mem(n)
        self.temp = Mem(n)
        self.dot_partial = Mem(self.ndg * (m + 1))
        self.scalars = Mem(16)
        self.temp_p = Mem(N)
        self.p_sol = Mem(N)
        self.params = Mem(8)
        self.precond_params = Mem(4)
        self.hess = Mem((m + 1) * m)
        self.givens = Mem(2 * m)
        self.g = Mem(m + 1)
        self.y = Mem(m)
        self.iter_params = Mem(4)
        self.amg_levels = None
        self._write_params_restore()

    # ------------------------------------------------------------ host API
    def _state_mem(self, which):
        idx = {0: (0, 1, 2), 1: (2, 0, 1), 2: (1, 2, 0)}[self.state_step_index]
        return self.states[idx[which]]

    def set_u(self, u):  # solver.rs:9-21: the whole FluidState buffer rewritten
        a = np.zeros((self.N, 8), F)
        a[:, 0:2] = np.asarray(u, np.float64).reshape(-1, 2).astype(F)
        self._state_mem(0).f[:] = a.reshape(-1)

    def set_p(self, p):  # solver.rs:23-34
        a = np.zeros((self.N, 8), F)
        a[:, 2] = np.asarray(p, np.float64).astype(F)
        self._state_mem(0).f[:] = a.reshape(-1)

    def initialize_history(self):  # solver.rs:276-294
        s = self._state_mem(0).u
        self._state_mem(1).u[:] = s
        self._state_mem(2).u[:] = s

    def _fields(self):
        """the current FluidState buffer as [N, 8] f32 (u, v, p, d_p, grad_p, grad_component)"""
        return self._state_mem(0).f.reshape(-1, 8)

    def get_u(self):
        return self._fields()[:, 0:2].astype(np.float64)

    def get_p(self):
        return self._fields()[:, 2].astype(np.float64)

    def get_d_p(self):
        return self._fields()[:, 3].astype(np.float64)

    # ------------------------------------------------------------ plumbing
    def _run(self, D, entry, bindings, groups):
        # wgpu refuses a dispatch dimension above 65,535 workgroups (the
        # reference's mesh-size ceiling): so does this driver
        if max(groups) > 65535:
            raise ValueError(f"{entry}: {groups} workgroups exceed wgpu's 65,535 per dimension")
        if D is _SHADERS.get("amg"):
            D.dispatch(entry, bindings, groups, schedule=self.amg_sched[0], bounds=self.amg_sched[1])
        else:
            D.dispatch(entry, bindings, groups, schedule=self.schedule, bounds=self.bounds)

    def _write_constants(self):
        c = self.c
        self.constants_b.u[:] = _words(F(c.dt), F(c.dt_old), F(c.time), F(c.viscosity), F(c.density), 0,
                                       F(c.alpha_p), int(c.scheme), F(c.alpha_u), 0, int(c.time_scheme),
                                       F(c.inlet_velocity), F(c.ramp_time), int(c.precond_type))

    def _write_params(self, n, num_cells, num_iters, omega, dispatch_x, max_restart):
        self.params.u[:] = _words(n, num_cells, num_iters, F(omega), dispatch_x, max_restart, 0, 0)

    def _write_params_restore(self):  # RawFgmresParams as restored after each special use
        self._write_params(self.n, self.N, 2, 1.0, _wg(self.n) * WG, self.m)

    def _iter_params(self, idx):
        self.iter_params.u[:] = _words(idx, self.m, 0, 0)

    def _bg_mesh_fields_solver(self):
        b = {k: Binding(v) for k, v in self.mesh_b.items()}
        b.update({(1, 0): Binding(self._state_mem(0)), (1, 1): Binding(self._state_mem(1)),
                  (1, 2): Binding(self._state_mem(2)), (1, 3): Binding(self.fluxes),
                  (1, 4): Binding(self.constants_b),
                  (2, 0): Binding(self.c_val), (2, 1): Binding(self.rhs_b), (2, 2): Binding(self.s_row),
                  (2, 3): Binding(self.grad_u), (2, 4): Binding(self.grad_v), (2, 5): Binding(self.s_val),
                  (2, 6): Binding(self.diag_u), (2, 7): Binding(self.diag_v), (2, 8): Binding(self.diag_p)})
        return b

    def _basis(self, j):  # basis_binding: offset j * stride, size of w
        return Binding(self.basis, j * self.bstride, self.n)

    def _vec_groups(self, x, y, z, group3="params"):
        b = {(0, 0): x, (0, 1): y, (0, 2): z,
             (1, 0): Binding(self.c_row), (1, 1): Binding(self.c_col), (1, 2): Binding(self.c_val),
             (2, 0): Binding(self.diag_u), (2, 1): Binding(self.diag_v), (2, 2): Binding(self.diag_p),
             (2, 3): Binding(self.precond_params)}
        if group3 == "params":  # bg_params
            b.update({(3, 0): Binding(self.params), (3, 1): Binding(self.scalars), (3, 2): Binding(self.iter_params),
                      (3, 3): Binding(self.hess), (3, 4): Binding(self.y)})
        else:  # bg_pressure_matrix (the live scalar matrix)
            b.update({(3, 0): Binding(self.s_row), (3, 1): Binding(self.s_col), (3, 2): Binding(self.s_val)})
        return b

    def _ops(self, entry, x, y, z, groups):
        self._run(shader("gmres_ops"), entry, self._vec_groups(x, y, z), (groups,))

    def _gpu_norm(self, x, n):  # coupled_solver_fgmres.rs:1444-1588
        wgs = _wg(n)
        self._write_params(n, self.N, 2, 1.0, wgs * WG, self.m)
        self._ops("norm_sq_partial", x, Binding(self.temp), Binding(self.dot_partial), wgs)
        self._write_params(self.ndg, 0, 0, 0.0, WG, 0)
        self._ops("reduce_final", Binding(self.dot_partial), Binding(self.temp), Binding(self.temp), 1)
        self._write_params(n, self.N, 2, 1.0, wgs * WG, self.m)
        return F(math.sqrt(F(self.scalars.f[0])))  # f32::sqrt on the host

    def _compute_residual_into(self):  # :1637-1667 (target = basis vector 0)
        wgs = _wg(self.n)
        self._ops("spmv", Binding(self.x_b), Binding(self.w), Binding(self.temp), wgs)
        self.scalars.f[0:2] = [F(1.0), F(-1.0)]
        self._ops("axpby", Binding(self.rhs_b), Binding(self.w), self._basis(0), wgs)
        return self._gpu_norm(self._basis(0), self.n)

    def _scale_in_place(self, target):
        self._ops("scale_in_place", Binding(self.temp), target, Binding(self.dot_partial), _wg(self.n))

    # ------------------------------------------------------------ AMG (amg.rs)
    def _build_amg(self):  # ensure_amg_resources: the scalar matrix at this moment, frozen
        self.amg = refpy.Amg(self.M.srow, self.M.scol, self.s_val.f.copy())
        lv = []
        for k, L in enumerate(self.amg.levels):
            n = L["n"]
            d = dict(n=n, row=buffer(L["row"].astype(U)), col=buffer(L["col"].astype(U)),
                     val=buffer(L["val"].astype(F)), x=Mem(n), b=Mem(n), params=buffer(_words(n, F(0.8), 0, 0)))
            if "agg" in L:
                nc = L["nc"]
                d["p_row"] = buffer(np.arange(n + 1, dtype=U))  # build_prolongation (amg.rs:118-139)
                d["p_col"] = buffer(L["agg"].astype(U))
                d["p_val"] = buffer(np.ones(n, F))
                mem = L["members"]  # transpose (amg.rs:141-185): fine indices ascending
                rr = np.zeros(nc + 1, U)
                rr[1:] = np.cumsum([len(x) for x in mem])
                d["r_row"] = buffer(rr)
                d["r_col"] = buffer(np.concatenate([np.asarray(x, U) for x in mem]))
                d["r_val"] = buffer(np.ones(n, F))
            lv.append(d)
        self.amg_levels = lv

    def _v_cycle(self):  # amg.rs:666-770, level 0 state = (p_sol, temp_p, level-0 params)
        lv = self.amg_levels
        A = shader("amg")

        def mat(i):
            return {(0, 0): Binding(lv[i]["row"]), (0, 1): Binding(lv[i]["col"]), (0, 2): Binding(lv[i]["val"])}

        def state(i):
            if i == 0:
                return {(1, 0): Binding(self.p_sol), (1, 1): Binding(self.temp_p), (1, 2): Binding(lv[0]["params"])}
            return {(1, 0): Binding(lv[i]["x"]), (1, 1): Binding(lv[i]["b"]), (1, 2): Binding(lv[i]["params"])}
        nl = len(lv)
        for i in range(nl - 1):
            fine, coarse = lv[i], lv[i + 1]
            self._run(A, "smooth_op", {**mat(i), **state(i)}, (_wg(fine["n"]),))
            if "r_row" in fine:
                self._run(A, "restrict_residual",
                           {**mat(i), **state(i), (2, 0): Binding(fine["r_row"]), (2, 1): Binding(fine["r_col"]),
                            (2, 2): Binding(fine["r_val"]), (3, 0): Binding(coarse["b"])}, (_wg(coarse["n"]),))
            self._run(A, "clear", {**mat(i + 1), **state(i + 1)}, (_wg(coarse["n"]),))
        for _ in range(10):
            self._run(A, "smooth_op", {**mat(nl - 1), **state(nl - 1)}, (_wg(lv[nl - 1]["n"]),))
        for i in range(nl - 2, -1, -1):
            fine = lv[i]
            if "p_row" in fine:
                self._run(A, "prolongate_op",
                           {**mat(i), **state(i), (2, 0): Binding(fine["p_row"]), (2, 1): Binding(fine["p_col"]),
                            (2, 2): Binding(fine["p_val"]), (3, 0): Binding(lv[i + 1]["x"])}, (_wg(fine["n"]),))
            self._run(A, "smooth_op", {**mat(i), **state(i)}, (_wg(fine["n"]),))

    # ------------------------------------------------------------ FGMRES
    def solve(self):
        N, n, m = self.N, self.n, self.m
        tol, abstol, max_outer = F(1e-5), F(1e-7), 20
        if self.c.precond_type == 1 and self.amg_levels is None:
            self._build_amg()
        wg_dofs, wg_cells = _wg(n), _wg(N)
        self._iter_params(0)
        self.precond_params.u[:] = _words(0, N, F(1.2), int(self.c.precond_type))
        rhs_norm = self._gpu_norm(Binding(self.rhs_b), n)
        if rhs_norm < abstol or not np.isfinite(rhs_norm):
            return dict(iterations=0, residual=rhs_norm, converged=bool(rhs_norm < abstol))

        def h_idx(r, c):
            return c * (m + 1) + r
        residual_norm = self._compute_residual_into()
        target = max(F(tol * rhs_norm), abstol)
        if residual_norm < target:
            return dict(iterations=0, residual=residual_norm, converged=True)
        self.scalars.f[0] = F(F(1.0) / residual_norm)
        self._scale_in_place(self._basis(0))
        self.g.f[:] = 0
        self.g.f[0] = residual_norm
        fixed = self.fixed_inner > 0
        inner_max = min(self.fixed_inner, m) if fixed else m
        outer_max = 1 if fixed else max_outer
        total, final, converged, stag, prev = 0, residual_norm, False, 0, residual_norm
        tol_abs = F(tol * rhs_norm)
        S, C, L = shader("schur_precond"), shader("gmres_cgs"), shader("gmres_logic")
        for outer in range(outer_max):
            size = 0
            for j in range(inner_max):
                size = j + 1
                total += 1
                cur = {(0, 0): self._basis(j), (0, 1): Binding(self.z[j]), (0, 2): Binding(self.temp_p),
                       (0, 3): Binding(self.p_sol), (0, 4): Binding(self.temp)}
                swp = dict(cur)
                swp[(0, 3)], swp[(0, 4)] = Binding(self.temp), Binding(self.p_sol)

                def sch(bg):
                    b = self._vec_groups(None, None, None, group3="pressure")
                    b.update(bg)
                    return b
                self._run(S, "predict_and_form_schur", sch(cur), (wg_cells,))
                in_sol = True
                if self.c.precond_type == 1:
                    self._v_cycle()
                else:
                    p_iters = max(min(20 + int(math.sqrt(F(N))) // 2, 200) - 1, 0)
                    for _ in range(p_iters):
                        self._run(S, "relax_pressure", sch(cur if in_sol else swp), (wg_cells,))
                        in_sol = not in_sol
                self._run(S, "correct_velocity", sch(cur if in_sol else swp), (wg_cells,))
                self._ops("spmv", Binding(self.z[j]), Binding(self.w), Binding(self.temp), wg_dofs)
                self._write_params(n, N, j, 0.0, self.ndg, m)
                cg = {(0, 0): Binding(self.params), (0, 1): Binding(self.basis), (0, 2): Binding(self.w),
                      (0, 3): Binding(self.dot_partial), (0, 4): Binding(self.hess)}
                self._run(C, "calc_dots_cgs", cg, (self.ndg,))
                self._run(C, "reduce_dots_cgs", cg, (j + 1,))
                self._run(C, "update_w_cgs", cg, (self.ndg,))
                self._write_params_restore()
                self._iter_params(h_idx(j + 1, j))
                self._ops("norm_sq_partial", Binding(self.w), Binding(self.temp), Binding(self.dot_partial), self.ndg)
                self._write_params(self.ndg, 0, 0, 0.0, WG, 0)
                self._ops("reduce_final_and_finish_norm", Binding(self.dot_partial), Binding(self.temp),
                          Binding(self.temp), 1)
                self._write_params_restore()
                self._ops("scale", Binding(self.w), self._basis(j + 1), Binding(self.temp), wg_dofs)
                self._iter_params(j)
                lg = {(0, 0): Binding(self.hess), (0, 1): Binding(self.givens), (0, 2): Binding(self.g),
                      (0, 3): Binding(self.y), (1, 0): Binding(self.iter_params), (1, 1): Binding(self.scalars)}
                self._run(L, "update_hessenberg_givens", lg, (1,))
                resid = F(self.scalars.f[0])
                if fixed:
                    continue
                # async_buffer.rs under the deterministic lag model; the reader is never reset
                have = (self.lag == 0) or (self.inner_last is not None)
                check = resid if self.lag == 0 else self.inner_last
                self.inner_last = resid
                if have and check < tol_abs:
                    converged = True
                    break
            self._iter_params(size)
            self._run(L, "solve_triangular", lg, (1,))
            for i in range(size):
                self._iter_params(i)
                self._ops("axpy_from_y", Binding(self.z[i]), Binding(self.x_b), Binding(self.temp), wg_dofs)
            if converged:
                final = self.inner_last
                break
            residual_norm = self._compute_residual_into()
            final = residual_norm
            if fixed:
                converged = bool(residual_norm < tol_abs)
                break
            if residual_norm < tol_abs:
                converged = True
                break
            self.g.f[:] = 0
            self.g.f[0] = residual_norm
            if residual_norm <= F(0):
                converged = True
                break
            self.scalars.f[0] = F(F(1.0) / residual_norm)
            self._scale_in_place(self._basis(0))
            improvement = (prev - residual_norm) / prev
            if improvement < F(1e-3):
                stag += 1
                if stag >= 3:
                    converged = True
                    break
            else:
                stag = 0
            prev = residual_norm
        return dict(iterations=total, residual=final, converged=converged)

    # ------------------------------------------------------------ step (coupled_solver.rs:33-499)
    def step(self):
        c = self.c
        N = self.N
        self.state_step_index = (self.state_step_index + 1) % 3
        P, A, Uf = shader("prepare_coupled"), shader("coupled_assembly_merged"), shader("update_fields_from_coupled")
        self._write_constants()
        self._run(P, "main", self._bg_mesh_fields_solver(), (_wg(N),))
        fixed = self.fixed_outer > 0
        max_iters = self.fixed_outer if fixed else max(20, 10)
        prev_u = prev_p = float("inf")
        last = None  # outer async reader, reset per step
        self.info["total_iterations"] = 0
        for it in range(max_iters):
            self._write_constants()
            if it > 0 or c.scheme != 0:
                self._run(P, "main", self._bg_mesh_fields_solver(), (_wg(N),))
            self._run(A, "main", self._bg_mesh_fields_solver(), (_wg(N),))
            ls = self.solve()
            self.info["iterations"], self.info["residual"] = ls["iterations"], ls["residual"]
            self.info["total_iterations"] += ls["iterations"]
            if np.isnan(ls["residual"]):
                raise FloatingPointError("Coupled Linear Solver Diverged: NaN detected in linear residual")
            if it > 0:
                self.max_diff.u[:] = 0
            b = self._bg_mesh_fields_solver()
            ub = {(0, 0): b[(1, 0)], (0, 1): b[(1, 1)], (0, 2): b[(1, 2)], (0, 3): b[(1, 3)], (0, 4): b[(1, 4)],
                  (1, 0): Binding(self.x_b), (1, 1): Binding(self.max_diff)}
            self._run(Uf, "main", ub, (_wg(N),))
            if it == 0:
                self.info.update(res_u=float(np.finfo(F).max), res_p=float(np.finfo(F).max), outer_iterations=1)
                continue
            du, dp = F(self.max_diff.f[0]), F(self.max_diff.f[1])
            if self.lag == 0:
                cu, cp, have = du, dp, True
            else:
                have = last is not None
                cu, cp = last if have else (F(0), F(0))
                last = (du, dp)
            if not have:
                continue
            if np.isnan(cu) or np.isnan(cp):
                raise FloatingPointError("Coupled Solver Diverged: NaN detected in outer residuals")
            self.info.update(res_u=float(cu), res_p=float(cp), outer_iterations=it + 1)
            if not fixed:
                if cu < 1e-5 and cp < 1e-4:
                    break
                rel_u = abs((float(cu) - prev_u) / prev_u) if np.isfinite(prev_u) and abs(prev_u) > 1e-14 else np.inf
                rel_p = abs((float(cp) - prev_p) / prev_p) if np.isfinite(prev_p) and abs(prev_p) > 1e-14 else np.inf
                if rel_u < 1e-2 and rel_p < 1e-2 and it > 2:
                    break
            prev_u, prev_p = float(cu), float(cp)
        c.time = F(c.time + c.dt)
        self._check_evolution()

    def _check_evolution(self):
        """coupled_solver.rs:501-580, literally: serial f64 sums, the f32
        squared differences, and the stride bug (2i, 2i+1 of the 8N floats)."""
        u = self._state_mem(0).f.copy()
        N = self.N
        n = float(N)
        s_u = s_v = sq_u = sq_v = 0.0
        for i in range(N):
            a, b = float(u[2 * i]), float(u[2 * i + 1])
            s_u += a
            s_v += b
            sq_u += a * a
            sq_v += b * b
        mu, mv = s_u / n, s_v / n
        var_u = max(sq_u / n - mu * mu, 0.0)
        var_v = max(sq_v / n - mv * mv, 0.0)
        self.variance = (self.variance + [(var_u, var_v)])[-10:]
        if self.prev is not None and len(self.prev) == len(u):
            d = (u - self.prev).astype(F)
            sq = (d * d).astype(F)
            evo = 0.0
            for x in sq:
                evo += float(x)
            evo = math.sqrt(evo / n)
        else:
            evo = float(np.finfo(np.float64).max)
        self.prev = u
        inf = self.info
        if evo < 1e-6:
            if var_u < 1e-10 and var_v < 1e-10:
                inf["degenerate"] += 1
                inf["steady"] = 0
            else:
                inf["steady"] += 1
                inf["degenerate"] = 0
        else:
            inf["degenerate"] = inf["steady"] = 0
        if inf["degenerate"] > 10 or inf["steady"] > 10:
            inf["should_stop"] = True
