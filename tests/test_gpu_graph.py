"""hipGraph replay of the FGMRES iteration (Solver::run_iteration).

Each iteration j is captured once into an executable graph and replayed by
every later solve; the launches inside are the eager path's, so graph replay
must give the eager path's bits -- and the oracle's -- under the fixed
schedule and the reference's natural one (lag 0 and 1: the per-iteration
residual lands in one of two pinned slots, one graph variant each), with the
AMG and the Jacobi preconditioner, across preconditioner switches (graphs
dropped and captured again) and AMG re-setups (numeric refresh: same pointers;
full rebuild: graphs dropped with the hierarchy).
"""
import numpy as np
import pytest

from cfd2_amd import GpuSolver, default_config
from tests.meshes import backwards_step, channel_obstacle
from tests.oracle_py import OracleSolver
from tests.test_gpu_parity import _assert_same_fields, _assert_same_info, _setup_amg_test

pytestmark = pytest.mark.gpu


def _three(mesh, **cfg):
    eager = GpuSolver(mesh, config=default_config(**cfg))
    eager.graph_enable(False)
    graph = GpuSolver(mesh, config=default_config(**cfg))
    graph.graph_enable(True)
    return eager, graph, OracleSolver(mesh, config=default_config(**cfg))


@pytest.mark.parametrize("precond,cfg", [
    (1, dict(fixed_outer=3, fixed_inner=10)),   # the bench's fixed schedule
    (1, dict()),                                # natural schedule, lag 1 (reference)
    (1, dict(convergence_lag=0)),               # natural schedule, blocking reads
    (0, dict()),                                # Jacobi preconditioner (fused sweeps)
    (0, dict(fixed_outer=2, fixed_inner=6)),
])
def test_graph_replay_parity(precond, cfg):
    """amg_test setup, 4 steps: graph replay == eager launches == oracle, bit-exact."""
    mesh = backwards_step()
    eager, graph, o = _three(mesh, **cfg)
    for s in (eager, graph, o):
        _setup_amg_test(s, mesh, precond)
    for k in range(4):
        for s in (eager, graph, o):
            s.step()
        _assert_same_fields(graph, eager, f"graph vs eager step {k}")
        _assert_same_info(graph, eager, f"graph vs eager step {k}")
        _assert_same_fields(graph, o, f"graph vs oracle step {k}")
        _assert_same_info(graph, o, f"graph vs oracle step {k}")
    on, cap, rep = graph.graph_stats()
    iters = graph.step_info().total_linear_iterations
    assert on and cap > 0 and rep >= iters > 0, (on, cap, rep, iters)
    assert rep > cap, "graphs captured but never replayed"
    assert eager.graph_stats() == (False, 0, 0)


def test_graph_preconditioner_switch_and_rebuild(monkeypatch):
    """Jacobi <-> AMG switches and a full AMG rebuild every 2 steps (the
    graphs hold the hierarchy's pointers: dropped and captured again)."""
    monkeypatch.setenv("CFD_AMG_SETUP", "rebuild")  # every re-setup a full rebuild, new allocations
    mesh = channel_obstacle(h=0.04)
    eager, graph, o = _three(mesh, fixed_outer=2, fixed_inner=8, amg_rebuild_interval=2)
    for s in (eager, graph, o):
        _setup_amg_test(s, mesh, 1)
    caps = []
    for k in range(7):
        if k in (2, 4):
            for s in (eager, graph, o):
                s.set_precond_type(0 if k == 2 else 1)
        for s in (eager, graph, o):
            s.step()
        _assert_same_fields(graph, eager, f"step {k}")
        _assert_same_fields(graph, o, f"oracle step {k}")
        _assert_same_info(graph, o, f"oracle step {k}")
        caps.append(graph.graph_stats()[1])
    # captures grow after each switch / rebuild, not every step
    assert caps[-1] > caps[0] and caps[1] == caps[0], caps


def test_graph_profiled_smoother_matches_eager():
    """The level-0 smoother timing (bench roofline) inside replayed graphs:
    event nodes around the smoother launches, harvested per replay -- the same
    number of timed sweeps as the eager path and a time of the same order."""
    mesh = channel_obstacle(h=0.02)
    res = {}
    for on in (False, True):
        s = GpuSolver(mesh, config=default_config(fixed_outer=2, fixed_inner=10))
        s.graph_enable(on)
        _setup_amg_test(s, mesh, 1)
        s.profile_enable(True)
        s.step()
        s.profile_reset()
        for _ in range(3):
            s.step()
        ms, n, _ = s.profile_smoother()
        s.profile_enable(False)
        res[on] = (ms, n, s.get_p())
    (ms0, n0, p0), (ms1, n1, p1) = res[False], res[True]
    assert n0 == n1 and n0 > 0, (n0, n1)
    assert ms0 > 0 and ms1 > 0
    assert 0.2 < (ms1 / n1) / (ms0 / n0) < 5.0, (ms0 / n0, ms1 / n1)
    assert np.array_equal(p0, p1)
