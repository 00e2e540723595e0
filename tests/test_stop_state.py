"""Caller-writable stop state (the reference's public fields should_stop /
degenerate_count / steady_state_count, structs.rs:244-247).

The GUI clears ``should_stop`` before it resumes stepping
(src/ui/app.rs:852-857); check_evolution (coupled_solver.rs:553-578) then
counts again from the caller's values.  Scenario: a field frozen by zero
under-relaxation (alpha_u = alpha_p = 0: every step reproduces the same
non-uniform state) reaches the steady-state stop after 11 steps; the caller
clears the flag, turns the relaxation back on and raises the inlet velocity;
the field evolves again, so the counters reset and ``should_stop`` stays
false.  A second leg clears the flag WITHOUT a change: the next step stops
again (count 12 > 10), as in the reference.  A third leg is a zero flow
(u = 0, inlet 0): check_evolution's stride bug puts d_p,
which varies over the cells, into the "velocity" variance, so the reference
counts this as a steady state, not a degenerate one.

CPU: the oracle.  GPU: the HIP path, step_info equal to the oracle's after
every step, fields bit-exact.
"""
import numpy as np
import pytest

from cfd2_amd import GpuSolver, default_config
from tests.meshes import backwards_step, channel_obstacle
from tests.oracle_py import OracleSolver
from tests.test_oracle import setup_amg_test


def _frozen_setup(s, mesh):
    s.set_dt(0.01)
    s.set_viscosity(0.01)
    s.set_density(1.0)
    s.set_alpha_u(0.0)
    s.set_alpha_p(0.0)
    a = mesh.arrays()
    u = np.zeros((mesh.num_cells(), 2))
    u[:, 0] = 4.0 * a["cell_cy"] * (1.0 - a["cell_cy"])
    s.set_u(u)
    s.initialize_history()
    s.set_precond_type(1)


def _zero_flow_setup(s, mesh):
    s.set_dt(0.01)
    s.set_viscosity(0.01)
    s.set_inlet_velocity(0.0)
    s.initialize_history()
    s.set_precond_type(1)


def _info(s):
    i = s.step_info()
    return (int(i.should_stop), int(i.degenerate_count), int(i.steady_state_count))


def _run_resume(solvers, mesh, on_step):
    """Steps every solver in lock step through the stop / clear / resume script;
    ``on_step`` compares them after each step.  Returns solvers[0]'s info trail."""
    trail = []

    def step(tag):
        for s in solvers:
            s.step()
        on_step(tag)
        trail.append((tag, _info(solvers[0])))

    for k in range(12):
        step(f"frozen {k}")
    assert trail[-1][1] == (1, 0, 11), trail  # steady-state stop: count 11 > 10
    # clear the flag only (no change): the next step stops again
    for s in solvers:
        s.should_stop = False
        assert _info(s) == (0, 0, 11)
    step("cleared, unchanged")
    assert trail[-1][1] == (1, 0, 12), trail
    # the GUI's resume: clear the flag, change the flow; the field evolves
    for s in solvers:
        s.should_stop = False
        s.set_alpha_u(0.7)
        s.set_alpha_p(0.3)
        s.set_inlet_velocity(2.0)
    for k in range(3):
        step(f"resumed {k}")
        assert trail[-1][1] == (0, 0, 0), trail
    # the counters themselves are writable too (all three fields public)
    for s in solvers:
        s.set_stop_state(True, 3, 4)
        assert _info(s) == (1, 3, 4)
    step("after set_stop_state")
    assert trail[-1][1] == (1, 0, 0), trail  # evolving: counts reset, the flag stays set
    return trail


def test_stop_state_oracle_cpu():
    mesh = channel_obstacle(h=0.1)
    o = OracleSolver(mesh, fixed_outer=2, fixed_inner=5)
    _frozen_setup(o, mesh)
    _run_resume([o], mesh, lambda tag: None)


def test_zero_flow_stop_oracle_cpu():
    mesh = channel_obstacle(h=0.1)
    o = OracleSolver(mesh, fixed_outer=2, fixed_inner=5)
    _zero_flow_setup(o, mesh)
    for _ in range(12):
        o.step()
    assert _info(o) == (1, 0, 11)
    o.should_stop = False
    o.set_inlet_velocity(1.0)
    o.step()
    assert _info(o) == (0, 0, 0)


@pytest.mark.gpu
def test_stop_state_gpu_matches_oracle():
    mesh = channel_obstacle(h=0.1)
    cfg = dict(fixed_outer=2, fixed_inner=5)
    g = GpuSolver(mesh, config=default_config(**cfg))
    o = OracleSolver(mesh, config=default_config(**cfg))
    for s in (g, o):
        _frozen_setup(s, mesh)

    def compare(tag):
        ig, io = g.step_info(), o.step_info()
        for f in ("should_stop", "degenerate_count", "steady_state_count"):
            assert getattr(ig, f) == getattr(io, f), f"{tag}: {f} {getattr(ig, f)} vs {getattr(io, f)}"
        assert np.array_equal(g.get_u(), o.get_u()), tag
        assert np.array_equal(g.get_p(), o.get_p()), tag

    _run_resume([g, o], mesh, compare)
    g.close()


@pytest.mark.gpu
def test_zero_flow_stop_gpu():
    mesh = channel_obstacle(h=0.1)
    g = GpuSolver(mesh, config=default_config(fixed_outer=2, fixed_inner=5))
    _zero_flow_setup(g, mesh)
    for _ in range(12):
        g.step()
    assert _info(g) == (1, 0, 11)
    g.should_stop = False
    g.set_inlet_velocity(1.0)
    g.step()
    assert _info(g) == (0, 0, 0)
    g.close()


def test_n_outer_correctors_writable_oracle_cpu():
    """structs.rs:238: a public field, read by every step (coupled_solver.rs:111,
    at least 10): amg_test reaches the 20-iteration cap; written to 12 the next
    step stops at 12; written to 5 it still runs 10 (the max with 10)."""
    mesh = backwards_step()
    o = OracleSolver(mesh)
    setup_amg_test(o, mesh, 1)
    o.step()
    assert o.step_info().outer_iterations == 20
    o.n_outer_correctors = 12
    o.step()
    assert o.step_info().outer_iterations == 12
    o.n_outer_correctors = 5
    o.step()
    assert o.step_info().outer_iterations == 10


@pytest.mark.gpu
def test_n_outer_correctors_gpu_matches_oracle():
    mesh = backwards_step()
    g, o = GpuSolver(mesh), OracleSolver(mesh)
    for s in (g, o):
        setup_amg_test(s, mesh, 1)
    for k, n in enumerate((20, 12, 5, 25)):
        for s in (g, o):
            s.n_outer_correctors = n
            s.step()
        assert g.step_info().outer_iterations == o.step_info().outer_iterations, (k, n)
        assert np.array_equal(g.get_u(), o.get_u()) and np.array_equal(g.get_p(), o.get_p()), (k, n)
    assert g.n_outer_correctors == 25
