"""Generates tests/golden/wgsl_ref.npz: outputs of the REFERENCE'S OWN WGSL
kernels, executed on the CPU (oracle/wgsl/wgsl_exec.py) under the Rust host
sequence restated in tests/wgsl_ref.py, on the meshes and setups of the
reference's own solver tests (amg_test.rs, coupled_schemes_test.rs), the
bench's fixed schedule and BASELINE configs[0] (the seeded Voronoi channel).

Needs /root/reference (the build container only); the fixtures travel, the
shader text does not: the file holds inputs' descriptions (case names) and
outputs (fields, per-step SHA-256 digests of the fields' f32 bytes, step
statistics) -- no reference source.

Two legal executions of the reference per case (wgsl_exec.py):
  A  workgroups in dispatch order, lanes in lockstep, Restrict bounds policy
     -> checked against the oracle with reference-semantics flags 15;
  B  the whole dispatch resident and in lockstep, ReadZeroSkipWrite policy
     -> checked against the oracle with flags 4 (the reference's reduction
        order; every other resolution the canonical one the HIP path uses).
Plus the kernel-level case: prepare_coupled + coupled_assembly_merged under
B on a random state, every output buffer (no reduction inside: equal to the
oracle's canonical mode, flags 0).

Run:  python -m tests.golden.make_wgsl_golden        (≈ 20 min)
      python -m tests.golden.make_wgsl_golden --only=C   (one mode, the rest kept)
      python -m tests.golden.make_wgsl_golden --c1   (BASELINE configs[1]: wgsl_ref_c1.npz)
"""
import hashlib
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "cfd-demo2_amd"))
sys.path.insert(0, os.path.join(HERE, "..", ".."))

F = np.float32


def digest(s):
    h = hashlib.sha256()
    for a in (s.get_u(), s.get_p(), s.get_d_p()):
        h.update(np.ascontiguousarray(np.asarray(a, np.float64).astype(F)).tobytes())
    return h.hexdigest()


def info_vec(s):
    """step statistics in a fixed order (float64)"""
    if hasattr(s, "step_info"):
        i = s.step_info()
        return np.array([i.total_linear_iterations, i.outer_iterations, F(i.outer_residual_u),
                         F(i.outer_residual_p), F(i.stats_p.residual), i.degenerate_count,
                         i.steady_state_count, int(bool(i.should_stop))], np.float64)
    d = s.info
    return np.array([d["total_iterations"], d["outer_iterations"], F(d["res_u"]), F(d["res_p"]),
                     F(d["residual"]), d["degenerate"], d["steady"], int(bool(d["should_stop"]))], np.float64)


def cases():
    """(name, mesh factory, setup(solver, mesh), solver kwargs, steps, modes)"""
    from tests.meshes import backwards_step
    from tests.test_oracle import setup_amg_test, setup_schemes_test

    def c0_setup(s, mesh):  # tests/test_refpy.py::test_c0_channel_fixed_schedule
        s.set_dt(1e-3)
        s.set_viscosity(0.01)
        s.set_density(1.0)
        s.set_alpha_u(0.7)
        s.set_alpha_p(0.3)
        s.set_precond_type(1)
        s.initialize_history()
        c = s.constants
        c.time = 0.05
        s.constants = c

    def c0_mesh():
        from cfd2_amd.mesh import bench_voronoi_channel
        return bench_voronoi_channel()
    out = []
    for pc, tag in ((1, "amg"), (0, "jacobi")):
        out.append((f"amg_test_{tag}", backwards_step, lambda s, m, pc=pc: setup_amg_test(s, m, pc), {}, 5,
                    "ABC" if pc else "AB"))
    for sc, ts in ((0, 0), (1, 0), (2, 0), (0, 1)):
        out.append((f"schemes_s{sc}t{ts}", backwards_step,
                    lambda s, m, sc=sc, ts=ts: setup_schemes_test(s, m, sc, ts), {}, 2, "AB"))
    fixed = dict(convergence_lag=0, fixed_outer=3, fixed_inner=10)
    for pc, tag in ((1, "amg"), (0, "jacobi")):
        out.append((f"fixed_{tag}", backwards_step, lambda s, m, pc=pc: setup_amg_test(s, m, pc), fixed, 3,
                    "ABC" if pc else "AB"))
    out.append(("c0_voronoi", c0_mesh, c0_setup, dict(convergence_lag=0, fixed_outer=2, fixed_inner=8), 2, "ABC"))
    return out


# mode: (schedule, bounds, oracle flags, the V-cycle's own (schedule, bounds) or None)
#   C: B for every dispatch but the V-cycle's, which run as in A -- the
#      reference's in-place smoother and clamped restriction rows, the rest
#      resident (oracle flags 13; the HIP path's reference-semantics mode 13)
MODES = {"A": ("workgroups", "restrict", 15, None), "B": ("dispatch", "zero", 4, None),
         "C": ("dispatch", "zero", 13, ("workgroups", "restrict"))}


def run_wgsl(name, mk, setup, kw, steps, mode):
    from tests.wgsl_ref import WgslRefSolver
    sched, bounds, _, amg = MODES[mode]
    mesh = mk()
    s = WgslRefSolver(mesh, schedule=sched, bounds=bounds, amg=amg, **kw)
    setup(s, mesh)
    res = {}
    digs, infos = [], []
    for _ in range(steps):
        s.step()
        digs.append(digest(s))
        infos.append(info_vec(s))
    res["digests"] = np.array(digs)
    res["info"] = np.stack(infos)
    if mesh.num_cells() <= 2000:
        res["u"] = s.get_u().astype(F)
        res["p"] = s.get_p().astype(F)
        res["d_p"] = s.get_d_p().astype(F)
    return res


def kernel_case(scheme, time_scheme):
    """prepare + assemble on a random state (tests/test_refpy.py's setup):
    the WGSL buffers after B (dispatch-resident prepare == snapshot reads)."""
    from tests.meshes import channel_obstacle
    from tests.wgsl_ref import WgslRefSolver, shader, _wg
    mesh = channel_obstacle()
    r = WgslRefSolver(mesh, schedule="dispatch", bounds="zero")
    rng = np.random.default_rng(11 + scheme + 3 * time_scheme)
    u0 = rng.uniform(-1, 1, size=(mesh.num_cells(), 2))
    u1 = rng.uniform(-1, 1, size=(mesh.num_cells(), 2))
    r.set_u(u1)
    r.initialize_history()
    r.set_u(u0)
    r.set_dt(0.002)
    r.set_dt(0.003)
    r.set_scheme(scheme)
    r.set_time_scheme(time_scheme)
    r.c.time = F(0.05)
    r._write_constants()
    b = r._bg_mesh_fields_solver()
    r._run(shader("prepare_coupled"), "main", b, (_wg(r.N),))  # d_p / grad_p from the zero state
    r._run(shader("prepare_coupled"), "main", b, (_wg(r.N),))  # Rhie-Chow with them
    r._run(shader("coupled_assembly_merged"), "main", b, (_wg(r.N),))
    st = r._state_mem(0).f.reshape(-1, 8)
    return dict(fluxes=r.fluxes.f.copy(), grad_u=r.grad_u.f.copy(), grad_v=r.grad_v.f.copy(),
                grad_p=st[:, 4:6].reshape(-1).copy(), d_p=st[:, 3].copy(), matrix=r.c_val.f.copy(),
                rhs=r.rhs_b.f.copy(), scalar_matrix=r.s_val.f.copy(), diag_u_inv=r.diag_u.f.copy(),
                diag_v_inv=r.diag_v.f.copy(), diag_p_inv=r.diag_p.f.copy())


def c1_setup(s, mesh):  # tests/test_gpu_parity.py::test_c1_scale_parity_and_true_residual
    s.set_dt(1e-3)
    s.set_viscosity(0.01)
    s.set_density(1.0)
    s.set_alpha_u(0.7)
    s.set_alpha_p(0.3)
    s.set_precond_type(1)
    s.initialize_history()


def c1_mesh():
    from tests.meshes import bench_mesh
    return bench_mesh(0.001723, 100)


# BASELINE configs[1] (1.0 M cells, the bench geometry and physics), schedule B
# only, 3 steps of 2 Picard x 6 FGMRES: every C1-only kernel form of the HIP
# path (paired AMG levels, the blob tail, 16-bit ELL levels) against the
# reference's kernels.  Digests and statistics only (the fields are 16 MB).
C1 = ("c1", c1_mesh, c1_setup, dict(convergence_lag=0, fixed_outer=2, fixed_inner=6), 3)


def main_c1():
    from tests import wgsl_ref
    if not wgsl_ref.available():
        raise SystemExit("the reference (/root/reference) is not present: fixtures cannot be regenerated here")
    name, mk, setup, kw, steps = C1
    t = time.time()
    res = run_wgsl(name, mk, setup, kw, steps, "B")
    print(f"{name} B: {time.time() - t:.1f} s, info {res['info'][-1].tolist()}", flush=True)
    np.savez_compressed(os.path.join(HERE, "wgsl_ref_c1.npz"), **{f"{name}/B/{k}": v for k, v in res.items()})


def main(only=None):
    """only: regenerate just these modes, keeping the file's other arrays"""
    from tests import wgsl_ref
    if not wgsl_ref.available():
        raise SystemExit("the reference (/root/reference) is not present: fixtures cannot be regenerated here")
    out = {}
    path = os.path.join(HERE, "wgsl_ref.npz")
    if only and os.path.exists(path):
        with np.load(path) as z:
            out = {k: z[k] for k in z.files}
    for name, mk, setup, kw, steps, modes in cases():
        for mode in modes:
            if only and mode not in only:
                continue
            t = time.time()
            res = run_wgsl(name, mk, setup, kw, steps, mode)
            for k, v in res.items():
                out[f"{name}/{mode}/{k}"] = v
            print(f"{name} {mode}: {time.time() - t:.1f} s, info {res['info'][-1].tolist()}", flush=True)
    if not only:
        for sc, ts in ((0, 0), (1, 0), (2, 0), (0, 1)):
            for k, v in kernel_case(sc, ts).items():
                out[f"kernels_s{sc}t{ts}/{k}"] = v
    np.savez_compressed(path, **out)
    print("wrote", path, len(out), "arrays")


if __name__ == "__main__":
    if "--c1" in sys.argv:
        main_c1()
    else:
        main(only=[a[len("--only="):] for a in sys.argv if a.startswith("--only=")] or None)
