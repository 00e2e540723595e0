"""Every BASELINE.json config under parity on the HIP path (VERDICT r02 item 1,
r03 item 1).

- C2 (configs[2], 10 M cells): the bench's exact fixed schedule, 5 Picard x
  30 FGMRES iterations, the t = 0 step and the first real step (the bench's
  two warm-up steps), GPU == oracle bit-exact after each.
- C3 (configs[3], 40 M cells, 4 ranks): GpuGroup(4) == GpuSolver bit-exact
  under the bench's 5 x 30 schedule (one step at t = 0.05), and
  GpuGroup(4) == OracleSolver bit-exact under a short fixed schedule
  (1 Picard x 6 FGMRES iterations): 40 M-cell HIP output tied to the oracle.
- C4 (configs[4], 80 M cells, 8 ranks): GpuSolver == OracleSolver under
  1 x 6, and GpuGroup(8) == GpuSolver under the bench's 5 x 30 schedule;
  each solver is freed before the next is built (two 80 M-cell solvers do
  not both fit).

At 40 M / 80 M rows the coupled matrices hold more than 2^31 entries and the
AMG hierarchy is deeper than at C2, so these legs check the single-GPU path
(coupled_solver.rs:33-499, coupled_solver_fgmres.rs:1728-2448, amg.rs:374-595)
where nothing smaller does.  The oracle's Krylov basis is sized to the fixed
schedule (oracle.cpp ensure_fgmres: 7 vectors for 6 iterations; 64 GB of
host memory at 80 M cells instead of ~160 GB).

Each phase prints a progress line straight to the terminal (pytest's capture
disabled for that line) so a long test is never mistaken for a hung one.
"""
import gc
import os
import time

import numpy as np
import pytest

from cfd2_amd import GpuGroup, GpuSolver, default_config
from cfd2_amd.mesh import bench_channel
from tests.oracle_py import OracleSolver, olib
from tests.test_gpu_parity import _assert_same_fields, _assert_same_info

pytestmark = pytest.mark.gpu

BENCH_H = {"c2": 5.449e-4, "c3": 2.724e-4, "c4": 1.926e-4}


@pytest.fixture
def progress(capsys):
    t0 = time.perf_counter()

    def say(msg):
        with capsys.disabled():
            print(f"\n    [{time.perf_counter() - t0:6.1f}s] {msg}", flush=True)
    return say


def _bench_setup(s, t0=0.0):
    """bench.py setup_solver (SURVEY §8(d) physics)."""
    s.set_dt(1e-3)
    s.set_viscosity(0.01)
    s.set_density(1.0)
    s.set_alpha_u(0.7)
    s.set_alpha_p(0.3)
    s.set_scheme(0)
    s.set_time_scheme(0)
    s.set_inlet_velocity(1.0)
    s.set_ramp_time(0.1)
    s.set_precond_type(1)
    s.initialize_history()
    if t0:
        c = s.constants
        c.time = t0
        s.constants = c


@pytest.mark.skipif(os.environ.get("CFD_C2_PARITY") == "0", reason="CFD_C2_PARITY=0")
def test_c2_headline_schedule_bitexact(progress):
    """The timed work itself: configs[2] under the bench's 5 x 30 schedule, the
    t = 0 step (rhs = 0: early exits) and the first real step, bit-exact."""
    olib().oracle_set_threads(min(16, os.cpu_count() or 1))
    mesh = bench_channel(BENCH_H["c2"], 100)
    assert mesh.num_cells() > 9_000_000
    progress(f"C2 mesh {mesh.num_cells()} cells")
    cfg = dict(fixed_outer=5, fixed_inner=30)
    g = GpuSolver(mesh, config=default_config(**cfg))
    o = OracleSolver(mesh, config=default_config(**cfg))
    for s in (g, o):
        _bench_setup(s)
    for k in range(2):
        g.step()
        progress(f"C2 GPU step {k} done")
        o.step()
        progress(f"C2 oracle step {k} done")
        _assert_same_fields(g, o, f"C2 5x30 step {k}")
        _assert_same_info(g, o, f"C2 5x30 step {k}")
    assert g.step_info().total_linear_iterations == 150
    assert g.amg_levels() == o.amg_levels()
    assert np.abs(g.get_u()).max() > 0.01
    g.close()


def _leg(make, mesh, cfg, t0, progress, label):
    """Build one solver of the leg, run one step, keep the fields / statistics /
    hierarchy on the host, free the solver."""
    s = make(mesh, cfg)
    _bench_setup(s, t0)
    progress(f"{label} created")
    s.step()
    progress(f"{label} step done")
    out = {"fields": (s.get_u(), s.get_p(), s.get_d_p()), "info": s.step_info(), "levels": s.amg_levels(),
           "ranks": [r.amg_levels() for r in s.ranks] if hasattr(s, "ranks") else None,
           "comm": [r.comm_stats() for r in s.ranks] if hasattr(s, "ranks") else None}
    if hasattr(s, "close"):
        s.close()
    del s  # the oracle frees its state when collected
    gc.collect()
    return out


def _same(a, b, label):
    for x, y, name in zip(a["fields"], b["fields"], ("u", "p", "d_p")):
        assert np.all(np.isfinite(x)), f"{label} {name} not finite"
        assert np.array_equal(x, y), f"{label}: {name} differs (max {np.abs(x - y).max()})"
    ia, ib = a["info"], b["info"]
    for f in ("outer_iterations", "total_linear_iterations", "outer_residual_u", "outer_residual_p"):
        assert getattr(ia, f) == getattr(ib, f), f"{label}: {f}"
    assert ia.stats_p.residual == ib.stats_p.residual, label
    assert np.abs(a["fields"][0]).max() > 0.01, label


def _global_levels(per_rank):
    """The global hierarchy from every rank's levels: a replicated level is the
    same on every rank, a row-partitioned one sums over the ranks."""
    out = []
    for i in range(len(per_rank[0])):
        lv = [p[i] for p in per_rank]
        out.append(lv[0] if all(x == lv[0] for x in lv) else (sum(x[0] for x in lv), sum(x[1] for x in lv)))
    return out


def _group_hierarchy(g, one, nranks):
    """Row-partitioned levels sum to the one-GPU level; replicated levels are
    the one-GPU level on every rank; the transport reports every rank."""
    levels1 = one["levels"]
    per_rank = g["ranks"]
    assert all(len(lv) == len(levels1) for lv in per_rank)
    for i, (rows1, nnz1) in enumerate(levels1):
        lv = [p[i] for p in per_rank]
        if all(x == lv[0] for x in lv) and lv[0] == (rows1, nnz1):
            continue
        assert sum(x[0] for x in lv) == rows1 and sum(x[1] for x in lv) == nnz1, (i, lv, rows1, nnz1)
    for r, st in enumerate(g["comm"]):
        assert st["comm_count"] == nranks and st["comm_rank"] == r


def _gpu(mesh, cfg):
    return GpuSolver(mesh, config=default_config(**cfg))


def _group(nranks):
    return lambda mesh, cfg: GpuGroup(mesh, nranks, config=default_config(**cfg))


def _oracle(mesh, cfg):
    olib().oracle_set_threads(min(16, os.cpu_count() or 1))
    return OracleSolver(mesh, config=default_config(**cfg))


SHORT = dict(fixed_outer=1, fixed_inner=6)
BENCH = dict(fixed_outer=5, fixed_inner=30)


def test_c3_group4_bench_schedule_and_oracle(progress):
    """configs[3] (40 M cells, 4 ranks): GpuGroup(4) == GpuSolver under the
    bench's 5 x 30 schedule, and GpuGroup(4) == OracleSolver under 1 x 6."""
    mesh = bench_channel(BENCH_H["c3"], 100)
    assert mesh.num_cells() > 39_000_000
    progress(f"C3 mesh {mesh.num_cells()} cells")
    one = _leg(_gpu, mesh, BENCH, 0.05, progress, "C3 GpuSolver 5x30")
    grp = _leg(_group(4), mesh, BENCH, 0.05, progress, "C3 GpuGroup(4) 5x30")
    _same(grp, one, "C3 5x30 group vs one GPU")
    assert grp["info"].total_linear_iterations == 150
    _group_hierarchy(grp, one, 4)
    del one, grp
    gs = _leg(_group(4), mesh, SHORT, 0.05, progress, "C3 GpuGroup(4) 1x6")
    orc = _leg(_oracle, mesh, SHORT, 0.05, progress, "C3 oracle 1x6")
    _same(gs, orc, "C3 1x6 group vs oracle")
    assert _global_levels(gs["ranks"]) == orc["levels"]


def test_c4_group8_one_gpu_and_oracle(progress):
    """configs[4] (80 M cells, 8 ranks): GpuSolver == OracleSolver under 1 x 6,
    and GpuGroup(8) == GpuSolver under the bench's own 5 x 30 schedule (the
    schedule `bench.py --gpus 8` times: distributed Krylov bases up to j = 29,
    all-gathered CGS dots), both from t = 0.05."""
    mesh = bench_channel(BENCH_H["c4"], 100)
    assert mesh.num_cells() > 79_000_000
    progress(f"C4 mesh {mesh.num_cells()} cells")
    one = _leg(_gpu, mesh, SHORT, 0.05, progress, "C4 GpuSolver 1x6")
    orc = _leg(_oracle, mesh, SHORT, 0.05, progress, "C4 oracle 1x6")
    _same(one, orc, "C4 one GPU vs oracle")
    assert one["levels"] == orc["levels"]
    del one, orc
    one = _leg(_gpu, mesh, BENCH, 0.05, progress, "C4 GpuSolver 5x30")
    grp = _leg(_group(8), mesh, BENCH, 0.05, progress, "C4 GpuGroup(8) 5x30")
    _same(grp, one, "C4 5x30 group vs one GPU")
    assert grp["info"].total_linear_iterations == 150
    _group_hierarchy(grp, one, 8)
