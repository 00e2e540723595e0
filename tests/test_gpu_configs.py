"""Every BASELINE.json config under parity on the HIP path.

- C2 (configs[2], 10 M cells): the bench's exact fixed schedule, 5 Picard x
  30 FGMRES iterations, the t = 0 step and the first real step (the bench's
  two warm-up steps), GPU == oracle bit-exact after each.
- C3 (configs[3], 40 M cells, 4 ranks): GpuGroup(4) == GpuSolver bit-exact on
  one GPU (the distributed algorithm the RCCL path runs; the oracle's
  equality with GpuSolver is established at C2 and on every smaller case).
- C4 (configs[4], 80 M cells, 8 ranks): the same with 8 in-process ranks; the
  single-GPU run goes first and is freed before the group is built (two
  80 M-cell solvers do not both fit).  ~4 min: CFD_C4_PARITY=1 enables it.

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


def _group_vs_one(config, nranks, progress, cfg=None, t0=0.05):
    """One GPU first (its fields kept on the host, the solver freed), then the
    in-process group of `nranks` ranks on the same GPU: bit-identical fields,
    step statistics and AMG hierarchy."""
    cfg = cfg or dict(fixed_outer=2, fixed_inner=10)
    mesh = bench_channel(BENCH_H[config], 100)
    n = mesh.num_cells()
    progress(f"{config} mesh {n} cells")
    one = GpuSolver(mesh, config=default_config(**cfg))
    _bench_setup(one, t0)
    progress(f"{config} GpuSolver created")
    one.step()
    progress(f"{config} GpuSolver step done")
    want = (one.get_u(), one.get_p(), one.get_d_p())
    info1 = one.step_info()
    levels1 = one.amg_levels()
    one.close()
    del one
    gc.collect()
    grp = GpuGroup(mesh, nranks, config=default_config(**cfg))
    del mesh
    gc.collect()
    _bench_setup(grp, t0)
    progress(f"{config} GpuGroup({nranks}) created")
    grp.step()
    progress(f"{config} GpuGroup({nranks}) step done")
    got = (grp.get_u(), grp.get_p(), grp.get_d_p())
    for a, b, name in zip(got, want, ("u", "p", "d_p")):
        assert np.all(np.isfinite(a)), name
        assert np.array_equal(a, b), f"{config} R={nranks} {name} differs (max {np.abs(a - b).max()})"
    ig = grp.step_info()
    for f in ("outer_iterations", "total_linear_iterations", "outer_residual_u", "outer_residual_p"):
        assert getattr(ig, f) == getattr(info1, f), f
    assert ig.stats_p.residual == info1.stats_p.residual
    # the same hierarchy: row-partitioned levels sum to the one-GPU level,
    # replicated levels are the one-GPU level on every rank
    per_rank = [r.amg_levels() for r in grp.ranks]
    assert all(len(lv) == len(levels1) for lv in per_rank)
    for i, (rows1, nnz1) in enumerate(levels1):
        lv = [p[i] for p in per_rank]
        if all(x == lv[0] for x in lv) and lv[0] == (rows1, nnz1):
            continue
        assert sum(x[0] for x in lv) == rows1 and sum(x[1] for x in lv) == nnz1, (i, lv, rows1, nnz1)
    assert np.abs(got[0]).max() > 0.01
    for r in range(nranks):
        st = grp.ranks[r].comm_stats()
        assert st["comm_count"] == nranks and st["comm_rank"] == r
    grp.close()


def test_c3_group4_equals_one_gpu(progress):
    """configs[3] (40 M cells, 4 ranks): GpuGroup(4) == GpuSolver bit-exact."""
    _group_vs_one("c3", 4, progress)


@pytest.mark.skipif(os.environ.get("CFD_C4_PARITY") != "1", reason="~4 min: CFD_C4_PARITY=1")
def test_c4_group8_equals_one_gpu(progress):
    """configs[4] (80 M cells, 8 ranks): GpuGroup(8) == GpuSolver bit-exact."""
    _group_vs_one("c4", 8, progress)
