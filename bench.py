#!/usr/bin/env python3
"""Benchmark of the coupled FV step (BASELINE.json metric: cell-updates/sec +
AMG smoother HBM GB/s on the channel+obstacle mesh).

One "step" = one GpuSolver.step() (reference coupled_solver.rs:33-499) on the
SURVEY §8(d) workload under its fixed schedule: 5 Picard iterations x 30
FGMRES(Schur + 1 AMG V-cycle) iterations, Upwind/Euler, rho=1, nu=0.01,
dt=1e-3, alpha_u=0.7, alpha_p=0.3, U_in=1 ramped over 0.1.  Synthetic input:
the deterministic cut-cell mesh of ChannelWithObstacle{3x1, (1.0,0.51), r 0.1}
(h=5.449e-4 -> ~10M cells per GPU), smoothed (0.3, 100); initial u = p = 0.

Launch: ``python bench.py`` (N=1) or, for N GPUs, under torch.distributed.run
with one process per GPU; rank 0 prints ONE JSON line.  ``python bench.py
--gpus N`` started WITHOUT a launcher (no WORLD_SIZE in the env) starts
torch.distributed.run itself, as a child process, before anything touches
the GPU, and exits with its status; under a launcher --gpus must equal
WORLD_SIZE (else exit 2).  N > 1 is weak
scaling (BASELINE configs[3..4]): the mesh is refined to
~10M x N cells (h / sqrt(N)), every rank owns one vertical slab of ~10M
cells, halos and reductions go over RCCL (xGMI); torch.distributed (gloo)
only bootstraps the RCCL unique id and the barrier / max-time reduction.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "cfd-demo2_amd"))
sys.path.insert(0, ROOT)

CONFIGS = {
    # name: (h, target cells per GPU, BASELINE.json configs[] index)
    # the reference-test scale (CPU-runnable; launch-bound on a GPU): the seeded
    # Voronoi channel (BASELINE configs[0] names Voronoi cells), h of the Voronoi mesher
    "c0": (0.0138, 1.0e4, 0),
    "c1": (0.001723, 1.0e6, 1),
    "c2": (5.449e-4, 1.0e7, 2),
}
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def setup_solver(solver, ramp_time=0.1):
    solver.set_dt(1e-3)
    solver.set_viscosity(0.01)
    solver.set_density(1.0)
    solver.set_alpha_u(0.7)
    solver.set_alpha_p(0.3)
    solver.set_scheme(0)
    solver.set_time_scheme(0)
    solver.set_inlet_velocity(1.0)
    solver.set_ramp_time(ramp_time)
    solver.set_precond_type(1)  # AMG
    solver.initialize_history()


def host_cores():
    """(nproc-equivalent CPUs of the machine, CPUs this process may run on)."""
    total = os.cpu_count() or 1
    try:
        allowed = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        allowed = total
    return total, allowed


def cgroup_cpus():
    """CPUs of this process's cgroup CPU quota (cpu.max / cfs quota), or None."""
    for path, parse in (("/sys/fs/cgroup/cpu.max", lambda t: t.split()),
                        ("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", None)):
        try:
            with open(path) as f:
                txt = f.read().strip()
        except OSError:
            continue
        if parse:
            q, per = parse(txt)[:2]
            if q != "max":
                return max(1, int(int(q) / int(per)))
            return None
        q = int(txt)
        if q > 0:
            with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                return max(1, int(q / int(f.read())))
        return None
    return None


def cpu_baseline(mesh, n_cells, outer_fixed, inner_fixed, step_ref_bytes=None, step_layout_bytes=None):
    """Oracle (C++ CPU restatement, OpenMP) on a bounded sample of the workload:
    the same mesh, physics and fixed schedule; the trivial t=0 step untimed (it
    also builds the AMG hierarchy), then ONE whole step (all `outer_fixed`
    Picard iterations x `inner_fixed` FGMRES iterations) timed.
    value = cells / seconds of that step, in cell-updates/sec.  Threads: every
    CPU this process can use -- the affinity set, capped by the cgroup CPU
    quota (a thread beyond the quota only time-slices) -- whatever
    OMP_NUM_THREADS says; when OMP_NUM_THREADS names a different count, that
    is timed too and the faster run is the value (both are reported)."""
    from tests.oracle_py import OracleSolver, set_threads
    from cfd2_amd import default_config

    total, allowed = host_cores()
    quota = cgroup_cpus()
    usable = min(allowed, quota) if quota else allowed
    counts = [usable]
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and 0 < int(env) != usable:
        counts.append(min(int(env), allowed))
    o = OracleSolver(mesh, config=default_config(fixed_outer=outer_fixed, fixed_inner=inner_fixed))
    setup_solver(o)
    set_threads(usable)
    o.step()  # t = 0: b == 0 -> early exits; builds the AMG hierarchy
    runs = []
    for threads in counts:
        set_threads(threads)
        if runs:  # the same state again: a fresh oracle through the t = 0 step
            o = OracleSolver(mesh, config=default_config(fixed_outer=outer_fixed, fixed_inner=inner_fixed))
            setup_solver(o)
            o.step()
        t0 = time.perf_counter()
        o.step()
        runs.append((threads, time.perf_counter() - t0))
    threads, dt = min(runs, key=lambda r: r[1])
    # BASELINE.md section 2 "Reported": the CPU's achieved GB/s from the same
    # algorithmic byte counts as the GPU line -- the reference-format count
    # (the oracle's own CSR layout is that format) and the GPU
    # library's layout-true bytes -- over the oracle's step time
    gbs = {
        "reference_format_gbs": (step_ref_bytes / dt / 1e9) if step_ref_bytes else None,
        "layout_true_gbs": (step_layout_bytes / dt / 1e9) if step_layout_bytes else None,
        "step_reference_format_bytes_count": step_ref_bytes,
        "step_layout_bytes": step_layout_bytes,
        "seconds_per_step": dt,
    }
    return {
        "value": n_cells / dt,
        "unit": "cell-updates/sec",
        "gbs": gbs,
        "cores": threads,
        "kind": "port",
        "host_cpus": total,
        "affinity_cpus": allowed,
        "cgroup_quota_cpus": quota,
        "runs": [{"threads": t, "seconds": d, "value": n_cells / d} for t, d in runs],
        "sample": (f"oracle/oracle.cpp (f32, OpenMP {threads} threads; the process may use {usable} CPUs: "
                   f"affinity {allowed}, cgroup quota {quota or 'none'}; machine: {total}), same {n_cells}-cell "
                   f"mesh, one whole step ({outer_fixed} Picard x {inner_fixed} FGMRES iterations, step 2) in "
                   f"{dt:.2f} s"),
    }


def load_traffic(round_tag, config, world):
    """HBM bytes per level-0 smoother launch from the committed rocprofv3 PMC
    summary (profiles/<round>/smoother_pmc.json) when it was measured on this
    workload (its config, one GPU), else None; returns (bytes, source)."""
    p = os.path.join(ROOT, "profiles", round_tag, "smoother_pmc.json")
    try:
        with open(p) as f:
            d = json.load(f)
        if world != 1 or not d["kernel"].endswith(f"config {config}"):
            return None, None
        return float(d["hbm_bytes_per_launch"]), os.path.relpath(p, ROOT)
    except (OSError, KeyError, ValueError):
        return None, None


def load_step_traffic(round_tag, config, world):
    """Counter-measured HBM bytes of one whole step (sum over every kernel of
    the step of FETCH_SIZE x 2 + WRITE_SIZE, tools/step_traffic.py) from the
    committed summary profiles/<round>/<config>_step_traffic.json, else None."""
    p = os.path.join(ROOT, "profiles", round_tag, f"{config}_step_traffic.json")
    try:
        with open(p) as f:
            d = json.load(f)
        if world != 1 or d.get("config") != config:
            return None
        d["source"] = os.path.relpath(p, ROOT)
        return d
    except (OSError, ValueError):
        return None


def reference_workloads(max_seconds=60.0, only=None):
    """The reference's own criterion benchmarks, run under THEIR schedule
    (natural convergence: lagged FGMRES/outer tests, up to 20 Picard x 20
    restarts x 50), as extra keys beside the headline (not the headline:
    their step cost is set by how many iterations the lagged tests admit):
      solver_step   benches/gpu_solver_benchmark.rs:6-46  BackwardsStep h=0.02,
                    smooth(0.3,50), water (rho 1000, nu 1e-3), dt 0.01,
                    alpha_p 1.0, Jacobi (default), no initialize_history
      fine_mesh     benches/gpu_dispatch_benchmark.rs:198-227 (+ setup_solver
                    :13-46)  BackwardsStep h=0.00175 (~1.06 M cells),
                    smooth(0.3,50), dt 1e-3, nu 1e-3, rho 1, alpha_p 0.3,
                    alpha_u 0.7, Upwind, AMG, one untimed step first
    Each is timed step by step (device-synchronised) until `steps` steps or
    `max_seconds`; ms/step and cell-updates/sec over the timed steps."""
    import numpy as np
    from cfd2_amd import GpuSolver, default_config
    from cfd2_amd.mesh import BackwardsStep, generate_cut_cell_mesh

    geo = BackwardsStep(length=3.5, height_inlet=0.5, height_outlet=1.0, step_x=0.5)

    def mesh_for(h):
        m = generate_cut_cell_mesh(geo, h, h, 1.2, (3.5, 1.0))
        m.smooth(geo, 0.3, 50)
        return m

    def inlet(m):
        a = m.arrays()
        u = np.zeros((m.num_cells(), 2))
        u[(np.asarray(a["cell_cx"]) < 0.05) & (np.asarray(a["cell_cy"]) > 0.5), 0] = 1.0
        return u

    def run(s, n_cells, warm, steps):
        for _ in range(warm):
            s.step()
        s.synchronize()
        times, iters = [], []
        t_all = time.perf_counter()
        for _ in range(steps):
            t0 = time.perf_counter()
            s.step()
            s.synchronize()
            times.append(time.perf_counter() - t0)
            iters.append(int(s.step_info().total_linear_iterations))
            if time.perf_counter() - t_all > max_seconds:
                break
        tot = sum(times)
        return {"cells": n_cells, "steps_timed": len(times), "ms_per_step": 1e3 * tot / len(times),
                "cell_updates_per_sec": n_cells * len(times) / tot,
                "fgmres_iterations_per_step": iters}

    out = {}
    if only in (None, "solver_step"):
        m = mesh_for(0.02)
        s = GpuSolver(m, config=default_config())
        s.set_dt(0.01)
        s.set_viscosity(0.001)
        s.set_density(1000.0)
        s.set_alpha_p(1.0)
        s.set_u(inlet(m))
        r = run(s, m.num_cells(), 0, 10)
        r["source"] = "benches/gpu_solver_benchmark.rs:6-46 (criterion sample_size 10)"
        out["solver_step"] = r
        s.close()
    if only in (None, "fine_mesh"):
        m = mesh_for(0.00175)
        s = GpuSolver(m, config=default_config())
        s.set_dt(0.001)
        s.set_viscosity(0.001)
        s.set_density(1.0)
        s.set_alpha_p(0.3)
        s.set_alpha_u(0.7)
        s.set_scheme(0)
        s.set_u(inlet(m))
        s.initialize_history()
        s.set_precond_type(1)
        r = run(s, m.num_cells(), 1, 10)
        r["source"] = "benches/gpu_dispatch_benchmark.rs:198-227 (criterion sample_size 10, one untimed step)"
        out["fine_mesh"] = r
        s.close()
    return out


def comm_timing_summary(t):
    """Per-FGMRES-iteration communication times of the extra timed step
    (cfd_comm_timing), by category: max and mean over ranks of the compute
    stream's exposed wait and of the transport's own time, in us; AMG halos
    per level.  `exposed_us_per_iteration` (max over ranks of the summed
    waits) against `iteration_us` (the step time with timing on / its
    iterations) gives the predicted parallel efficiency 1 - exposed / iteration
    (DESIGN.md section 7.1)."""
    its = t["iterations"]
    cats = {}
    for r, entries in enumerate(t["ranks"]):
        for e in entries:
            key = e["category"] + (f"_l{e['level']}" if e["level"] >= 0 else "")
            c = cats.setdefault(key, {"calls": [], "wait_us": [], "comm_us": [], "bytes": []})
            c["calls"].append(e["calls"] / its)
            c["wait_us"].append(e["wait_us"] / its)
            c["comm_us"].append(e["comm_us"] / its)
            c["bytes"].append(e["bytes"] / its)
    out = {}
    for k, c in sorted(cats.items()):
        out[k] = {"calls": max(c["calls"]), "bytes": max(c["bytes"]),
                  "wait_us_max": max(c["wait_us"]), "wait_us_mean": sum(c["wait_us"]) / len(c["wait_us"]),
                  "comm_us_max": max(c["comm_us"]), "comm_us_mean": sum(c["comm_us"]) / len(c["comm_us"])}
    exposed = max(sum(e["wait_us"] for e in entries) / its for entries in t["ranks"]) if t["ranks"] else 0.0
    it_us = 1e3 * t["step_ms_with_timing"] / its
    return {"per_iteration": out, "exposed_us_per_iteration": exposed, "iteration_us": it_us,
            "predicted_efficiency": 1.0 - exposed / it_us if it_us > 0 else None,
            "note": "one extra step after the timed ones, halos / all-gathers bracketed by timing events; "
                    "wait = compute-stream stall, comm = transport time (RCCL: includes peer skew)"}


def rank_launch_cmd(n, argv, port):
    """torch.distributed.run command that runs this script as n local ranks
    (the driver's own launch line, 127.0.0.1 rendezvous)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *argv]


def launch_ranks(n, argv):
    """--gpus N > 1 without a launcher: run the N ranks through
    torch.distributed.run in a CHILD process and return its exit status.  This
    process never touches the GPU (no torch import, no HIP call) and never
    re-execs; the ranks' stdout is this process's stdout, so rank 0's JSON line
    is the one line printed."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = rank_launch_cmd(n, argv, port)
    log(f"bench.py: --gpus {n} without a launcher: starting {n} ranks via torch.distributed.run (port {port})")
    sys.stdout.flush()
    return subprocess.call(cmd, env=dict(os.environ, MASTER_ADDR="127.0.0.1"))


def check_world(gpus, env):
    """(world size, error message or None): --gpus against the launcher's WORLD_SIZE."""
    ws = env.get("WORLD_SIZE")
    world = int(ws) if ws else 1
    if gpus < 1:
        return world, f"--gpus must be >= 1 (got {gpus})"
    if ws and gpus != world:
        return world, (f"--gpus {gpus} but the launcher started WORLD_SIZE={world} ranks: "
                       f"run with --gpus {world}, or start bench.py --gpus {gpus} without a launcher")
    return world, None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)  # 10 timed steps after 2 warm-up steps
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--outer", type=int, default=5)
    ap.add_argument("--inner", type=int, default=30)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--round", default="r06")
    ap.add_argument("--ref-workloads", type=int, default=1,
                    help="1: also time the reference's own criterion workloads (natural convergence) as extra keys")
    ap.add_argument("--inproc-ranks", type=int, default=0,
                    help="test mode: run the distributed solver as R in-process ranks on GPU 0 "
                         "(not a bench line; exercises the multi-GPU code path at scale on one GPU)")
    ap.add_argument("--amg-rebuild", type=int, default=0,
                    help="rebuild the AMG hierarchy every K steps (opt-in deviation from the reference's "
                         "frozen hierarchy; not the headline configuration)")
    ap.add_argument("--amg-local", type=int, default=0,
                    help="1: partition-aware AMG aggregation on the distributed levels (cfd_config."
                         "amg_local_aggregation; opt-in, no restriction / prolongation halos)")
    ap.add_argument("--mesh-cache", default=None,
                    help="binary mesh file: loaded if present, else generated and saved (A/B runs)")
    args = ap.parse_args()

    if args.gpus > 1 and not os.environ.get("WORLD_SIZE"):
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world, err = check_world(args.gpus, os.environ)
    if err:
        log("bench.py:", err)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        # gloo announces its connections on fd 1; keep stdout for the JSON line
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            dist.init_process_group("gloo")
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)

    import numpy as np  # noqa: F401
    from cfd2_amd import GpuSolver, default_config, dist_unique_id
    from cfd2_amd.mesh import bench_channel

    h, _, cfg_idx = CONFIGS[args.config]
    h_run = h / (world ** 0.5)  # weak scaling: ~N x the 1-GPU cell count
    if args.inproc_ranks > 1:
        h_run = h / (args.inproc_ranks ** 0.5)
    t0 = time.perf_counter()

    def make_mesh():
        if args.mesh_cache and os.path.exists(args.mesh_cache):
            from cfd2_amd.mesh import Mesh
            return Mesh.load(args.mesh_cache)
        if args.config == "c0":
            from cfd2_amd.mesh import bench_voronoi_channel
            m = bench_voronoi_channel(h_run)
        else:
            m = bench_channel(h_run, 100)
        if args.mesh_cache and rank == 0:
            m.save(args.mesh_cache)
        return m

    shared = None
    if world > 1:
        # one process per GPU: rank 0 generates the mesh once and writes its view
        # arrays to a file every rank maps read-only (one shared page-cache copy
        # instead of N generated meshes: ~12 GB each at 80 M cells)
        from cfd2_amd.mesh import MappedMesh, save_view_file
        est = 160 * 2.9686 / h_run ** 2  # bytes of the view arrays (~148 B per cell)
        base = "/dev/shm"
        try:
            st = os.statvfs(base)
            if st.f_bavail * st.f_frsize < 2 * est:
                base = tempfile.gettempdir()
        except OSError:
            base = tempfile.gettempdir()
        shared = os.path.join(base, f"cfd2_bench_mesh_{os.environ.get('MASTER_PORT', '0')}_{args.config}_{world}.bin")
        ok = [True]
        if rank == 0:
            import atexit

            def _drop_shared(path=shared):  # a failed run must not leave GBs in /dev/shm
                for junk in (path, path + ".tmp"):
                    try:
                        os.unlink(junk)
                    except OSError:
                        pass
            atexit.register(_drop_shared)
            m0 = make_mesh()
            try:
                save_view_file(m0, shared)
            except OSError as e:  # no room for the shared file: every rank generates its own mesh
                log(f"[rank 0] shared mesh file {shared} failed ({e}); generating per rank")
                ok[0] = False
                for junk in (shared, shared + ".tmp"):
                    if os.path.exists(junk):
                        os.unlink(junk)
            del m0
        dist.broadcast_object_list(ok, src=0)
        if ok[0]:
            mesh = MappedMesh(shared)
        else:
            shared = None
            mesh = make_mesh()
    else:
        mesh = make_mesh()
    n_global = mesh.num_cells()
    setup_s = {"mesh": time.perf_counter() - t0}
    log(f"[rank {rank}] mesh {n_global} cells / {mesh.num_faces()} faces in {setup_s['mesh']:.1f}s")

    cfg = default_config(fixed_outer=args.outer, fixed_inner=args.inner, amg_rebuild_interval=args.amg_rebuild,
                         amg_local_aggregation=args.amg_local)
    t0 = time.perf_counter()
    # test / rehearsal mode: CFD_DIST_TRANSPORT=host stages every exchange through
    # the gloo process group (several ranks may then share one GPU: CFD_BENCH_DEVICE)
    transport = os.environ.get("CFD_DIST_TRANSPORT", "rccl")
    device = int(os.environ.get("CFD_BENCH_DEVICE", local_rank))
    if world > 1 and transport == "host":
        solver = GpuSolver.create_dist_host(mesh, world, rank, device=device, config=cfg)
    elif world > 1:
        uid = [dist_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        solver = GpuSolver.create_dist(mesh, world, rank, uid[0], device=device, config=cfg)
    elif args.inproc_ranks > 1:
        from cfd2_amd import GpuGroup
        solver = GpuGroup(mesh, args.inproc_ranks, config=cfg)
        solver.num_cells = solver.ranks[0].num_cells
        solver.profile_smoother = solver.ranks[0].profile_smoother
        solver.smoother_layout_bytes = solver.ranks[0].smoother_layout_bytes
        solver.step_layout_bytes = solver.ranks[0].step_layout_bytes
        solver.step_algorithmic_bytes = solver.ranks[0].step_algorithmic_bytes
    else:
        solver = GpuSolver(mesh, config=cfg, device=0)
    n_cells = solver.num_cells  # cells this rank owns
    setup_solver(solver)
    if shared is not None:
        dist.barrier()  # every rank has built its slab: the shared file can go
        if rank == 0 and os.path.exists(shared):
            os.unlink(shared)
    if world > 1 or args.inproc_ranks > 1:
        del mesh  # the solver keeps what it needs; free the global mesh
        import gc
        gc.collect()
        mesh = None
    setup_s["create"] = time.perf_counter() - t0
    log(f"[rank {rank}] solver created in {setup_s['create']:.1f}s (owns {n_cells} cells)")

    def barrier_sync():
        # device fence (the torch.cuda.synchronize() of the contract: the
        # solver's own HIP device sync; torch never touches the GPU here), then
        # the barrier lines the ranks up
        solver.synchronize()
        if dist is not None:
            dist.barrier()

    # timing on from the warm-up steps: the FGMRES iteration graphs (one GPU,
    # small meshes) are captured there with the smoother's timing nodes, not
    # inside the timed region (profile_reset below drops the warm-up times)
    solver.profile_enable(True)
    for k in range(args.warmup):
        t0 = time.perf_counter()
        solver.step()
        setup_s.setdefault("first_step", time.perf_counter() - t0)  # t = 0 step: includes the AMG setup
        log(f"[rank {rank}] warmup step {k}: {time.perf_counter() - t0:.3f}s")
    barrier_sync()
    solver.profile_reset()
    graph0 = solver.graph_stats() if hasattr(solver, "graph_stats") else None
    handles = solver.ranks if args.inproc_ranks > 1 else [solver]
    for hnd in handles:
        hnd.comm_stats(reset=True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        solver.step()
    # step() returns after its blocking check_evolution read: the stream is idle
    barrier_sync()
    elapsed = time.perf_counter() - t0
    sm_ms, sm_n, sm_bytes = solver.profile_smoother()
    solver.profile_enable(False)
    graph1 = solver.graph_stats() if graph0 is not None else None
    info = solver.step_info()
    if dist is not None:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    # every rank's cells (in-process ranks included): the whole job's work
    total_cells = float(n_global)
    # transport of every rank and its collective traffic over the timed steps
    comm = [hnd.comm_stats() for hnd in handles]
    if dist is not None:
        allc = [None] * world
        dist.all_gather_object(allc, comm[0])
        comm = allc
    comm_line = None
    timing = None
    if len(comm) > 1:
        # one more step, outside the timed region, with every halo / all-gather
        # bracketed by timing events: exposed (compute-stream) wait and transport
        # time per category, per FGMRES iteration, on every rank
        for hnd in handles:
            hnd.comm_timing_enable(True)
        t1 = time.perf_counter()
        solver.step()
        solver.synchronize()
        timed_step_ms = 1e3 * (time.perf_counter() - t1)
        its = max(1, int(solver.step_info().total_linear_iterations))
        mine = [hnd.comm_timing() for hnd in handles]
        for hnd in handles:
            hnd.comm_timing_enable(False)
        if dist is not None:
            allt = [None] * world
            dist.all_gather_object(allt, mine[0])
            mine = allt
            ts = [None] * world
            dist.all_gather_object(ts, timed_step_ms)
            timed_step_ms = max(ts)
        timing = {"iterations": its, "step_ms_with_timing": timed_step_ms, "ranks": mine}
        iters = max(1, args.steps * int(info.total_linear_iterations))
        comm_line = {
            "transport": comm[0]["transport"],
            "comm_count": [c["comm_count"] for c in comm],
            "rank_device": [c["device"] for c in comm],
            "comm_rank": [c["comm_rank"] for c in comm],
            "fgmres_iterations_timed": iters,
            # per FGMRES iteration (everything of the timed steps / their iterations), max over ranks
            "exchanges_per_iteration": max(c["exchanges"] for c in comm) / iters,
            "allgathers_per_iteration": max(c["allgathers"] for c in comm) / iters,
            "halo_bytes_per_iteration": max(c["bytes_sent"] for c in comm) / iters,
            "allgather_bytes_per_iteration": max(c["bytes_gathered"] for c in comm) / iters,
        }
        comm_line["timing"] = comm_timing_summary(timing)
        comm_line["setup_s_rank0"] = setup_s

    ms_per_step = 1e3 * elapsed / args.steps
    inproc = args.inproc_ranks > 1
    if inproc:
        cfg_label = f"configs[{cfg_idx}] weak-scaled x{args.inproc_ranks} as {args.inproc_ranks} in-process ranks on ONE GPU (test mode)"
    elif world == 1:
        cfg_label = f"configs[{cfg_idx}]"
    elif args.config == "c2" and world in (4, 8):
        cfg_label = f"configs[{3 if world == 4 else 4}]"
    else:
        cfg_label = f"configs[{cfg_idx}] weak-scaled x{world}"
    value = total_cells * args.steps / elapsed
    sm_avg_s = (sm_ms / 1e3) / max(sm_n, 1)
    layout_bytes = solver.smoother_layout_bytes()
    achieved = layout_bytes / sm_avg_s / 1e9 if sm_n else 0.0
    achieved_ref = sm_bytes / sm_avg_s / 1e9 if sm_n else 0.0
    step_bytes = solver.step_algorithmic_bytes()
    step_layout = solver.step_layout_bytes()
    traffic, traffic_src = load_traffic(args.round, args.config, world if not inproc else args.inproc_ranks)
    counter_gbs = traffic / sm_avg_s / 1e9 if (traffic and sm_n) else None
    if world > 1:
        par = (f"slab{world} (RCCL halo + all-gather)" if transport != "host" else
               f"slab{world} (host-staged gloo transport: test mode, not a bench line)")
    elif inproc:
        par = f"inproc{args.inproc_ranks} (in-process ranks sharing one GPU, peer-copy transport: test mode)"
    else:
        par = "single"
    try:
        import __graft_entry__ as ge
        src_hash = ge.source_hash()
    except Exception:  # the hash is provenance, never the measurement
        src_hash = None
    from cfd2_amd import build_id
    bid = build_id()
    out = {
        "metric": "cell-updates/sec + AMG smoother HBM GB/s, channel+obstacle",
        "value": value,
        "unit": "cell-updates/sec",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": ("synthetic: seeded Voronoi channel+obstacle mesh (voronoi.rs restated, seed 12345)"
                 if args.config == "c0" else
                 "synthetic: deterministic cut-cell channel+obstacle mesh (reference generator restated)"),
        "config": {
            "workload": (f"BASELINE {cfg_label}: channel+obstacle {n_global} cells on {world} GPU(s) (~{n_cells} per rank), "
                         f"fixed schedule {args.outer} Picard x {args.inner} FGMRES/AMG per step"
                         + (f", AMG hierarchy rebuilt every {args.amg_rebuild} step(s) (opt-in deviation)"
                            if args.amg_rebuild else "")
                         + (", partition-aware AMG aggregation (opt-in)" if args.amg_local and world > 1 else "")),
            "cells_total": n_global,
            "cells_per_gpu": n_cells if not inproc else n_global,
            "cells_per_rank": n_cells,
            "h": h_run,
            "parallelism": par,
        },
        "build_id": bid,
        "source_hash": src_hash,
        "build_matches_sources": (bid == src_hash) if src_hash else None,
        # roofline of record: the level-0 AMG smoother.
        # achieved/frac: LAYOUT-TRUE algorithmic bytes per launch (what the
        # kernel must move in this library's level image: u8 lengths, ELL
        # values + 16-bit column deltas, b, x, diagonal, x_out; 41 B/row at C2)
        # / the live HIP-event launch time.  achieved_counter/frac_counter: HBM
        # bytes the counters measured per launch (FETCH_SIZE x 2 + WRITE_SIZE,
        # traffic_source) / the same time.  reference_format_*: SURVEY §8(d)'s
        # count in the reference's CSR format (56 B/row) -- a count of bytes
        # this layout does not move, kept for comparison, not an HBM rate.
        "roofline": {
            "bound": "hbm",
            "kernel": "k_amg_smooth (level 0, this rank's rows)",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": traffic,
            "traffic_source": (f"{traffic_src} (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes, committed; "
                               "not measured in this run)") if traffic_src else None,
            "achieved_counter": counter_gbs,
            "frac_counter": (counter_gbs / HBM_PEAK_GBS) if counter_gbs else None,
            "bytes_per_launch": layout_bytes,
            "bytes_model": "layout-true (cfd_smoother_layout_bytes)",
            # counts, not HBM rates: bytes in the reference's CSR format that
            # this layout does not move, and that count / the launch time
            "reference_format_bytes_count": sm_bytes,
            "reference_format_effective_gbs": achieved_ref,
            "avg_launch_us": sm_avg_s * 1e6,
            "launches": sm_n,  # timed sweeps: every sample_stride-th level-0 sweep of the timed steps
            "sample_stride": 1,  # every level-0 sweep of the timed steps
        },
        "comm": comm_line,
        # hipGraph replay of the FGMRES iteration: captures / replays inside the timed steps
        "graph": ({"enabled": graph1[0], "captures_timed": graph1[1] - graph0[1],
                   "replays_timed": graph1[2] - graph0[2]} if graph1 else None),
        # whole-step byte COUNT in the reference's CSR format (SURVEY §8(d)
        # sum): this layout moves ~45 % less (step_counter_traffic below is the
        # measured traffic), so count / step time is not an HBM rate
        "step_reference_format_bytes_count": step_bytes,
        # layout-true bytes of one step (this rank): each kernel's minimum
        # traffic at kernel level in this library's layouts x its launches (not
        # a bound on HBM traffic: some lines come from the Infinity Cache)
        "step_layout_bytes": {
            "bytes_per_step": step_layout,
            "gbs": step_layout / (ms_per_step / 1e3) / 1e9,
            "frac": step_layout / (ms_per_step / 1e3) / 1e9 / HBM_PEAK_GBS,
        },
        "linear_iterations_last_step": int(info.total_linear_iterations),
    }
    st = load_step_traffic(args.round, args.config, world if not inproc else args.inproc_ranks)
    if st:
        gbs = st["bytes_per_step"] / (ms_per_step / 1e3) / 1e9
        out["step_counter_traffic"] = {
            "bytes_per_step": st["bytes_per_step"],
            "gbs": gbs,
            "frac": gbs / HBM_PEAK_GBS,
            "source": st["source"] + " (committed PMC passes over one whole step; rate = those bytes / this run's step time)",
        }
    if rank == 0 and world == 1 and not inproc and mesh is not None and args.outer > 0 and not args.no_cpu_baseline:
        try:
            out["cpu_baseline"] = cpu_baseline(mesh, n_cells, args.outer, args.inner, step_bytes, step_layout)
        except Exception as e:  # the baseline is reported, never the target
            log("cpu baseline failed:", e)
            out["cpu_baseline"] = None
    if rank == 0 and world == 1 and not inproc and args.ref_workloads:
        try:
            out["reference_workloads"] = reference_workloads()
        except Exception as e:
            log("reference workloads failed:", e)
            out["reference_workloads"] = None
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
