"""Layout limits and failure paths of the HIP solver (round-3 advisor items):

- the widest rows a mesh can give (a hub cell with 100 neighbours: untyped
  coupled ELL, width > 32) bit-exact against the oracle;
- FGMRES(1) under the natural schedule: the lagged residual read of the
  previous iteration is always the slot the next iteration would write
  (two pinned slots, Solver::solve), bit-exact against the oracle;
- an in-process group whose rank fails returns an error on every rank instead
  of hanging, and stays usable afterwards (LocalGroup::reset).
"""
import numpy as np
import pytest

from cfd2_amd import GpuGroup, GpuSolver, default_config
from tests.meshes import backwards_step
from tests.oracle_py import OracleSolver
from tests.synthetic import wheel
from tests.test_gpu_parity import _assert_same_fields, _assert_same_info, _setup_amg_test

pytestmark = pytest.mark.gpu


def _wheel_setup(s, precond):
    s.set_dt(0.01)
    s.set_viscosity(0.01)
    s.set_density(1.0)
    s.set_alpha_u(0.7)
    s.set_alpha_p(0.3)
    s.set_precond_type(precond)
    s.initialize_history()
    c = s.constants
    c.time = 0.1
    s.constants = c


@pytest.mark.parametrize("k,precond", [(100, 1), (100, 0), (40, 1)])
def test_wide_row_wheel_parity(k, precond):
    """Hub cell with k neighbours (scalar row width k + 1, face slots k):
    three steps, GPU == oracle bit-exact."""
    m = wheel(k)
    g, o = GpuSolver(m), OracleSolver(m)
    for s in (g, o):
        _wheel_setup(s, precond)
    for step in range(3):
        g.step()
        o.step()
        _assert_same_fields(g, o, f"wheel({k}) precond {precond} step {step}")
        _assert_same_info(g, o, f"wheel({k}) precond {precond} step {step}")
    assert np.abs(g.get_u()).max() > 0
    g.close()


@pytest.mark.parametrize("precond", [0, 1])
def test_fgmres_one_iteration_per_restart_lag_parity(precond):
    """max_restart = 1: every FGMRES iteration is a restart and the lagged
    reader's pending slot is the previous iteration's (the reader is never
    reset): GPU == oracle bit-exact under the natural lag-1 schedule."""
    mesh = backwards_step()
    cfg = dict(max_restart=1, max_outer_restarts=6)
    g = GpuSolver(mesh, config=default_config(**cfg))
    o = OracleSolver(mesh, config=default_config(**cfg))
    for s in (g, o):
        _setup_amg_test(s, mesh, precond)
    for step in range(3):
        g.step()
        o.step()
        _assert_same_fields(g, o, f"FGMRES(1) step {step}")
        _assert_same_info(g, o, f"FGMRES(1) step {step}")
    g.close()


def test_group_rank_failure_then_reuse():
    """One rank fails while the others wait in a collective: every rank
    returns (an error naming the failed rank, no hang), and the same group
    then steps bit-exactly like one GPU."""
    mesh = backwards_step()
    grp = GpuGroup(mesh, 3)
    one = GpuSolver(mesh)
    for s in (grp, one):
        _setup_amg_test(s, mesh, 1)
    for fail in (1, 0, 2):
        with pytest.raises(RuntimeError, match=f"rank {fail}: injected fault"):
            grp.debug_fault(fail)
    for step in range(2):
        grp.step()
        one.step()
        _assert_same_fields(grp, one, f"group after faults, step {step}")
        _assert_same_info(grp, one, f"group after faults, step {step}")
    st = grp.ranks[1].comm_stats()
    assert st["transport"] == "in-process" and st["comm_count"] == 3 and st["comm_rank"] == 1
    assert st["exchanges"] > 0 and st["allgathers"] > 0
    grp.close()
    one.close()


def test_group_midstep_failure_needs_restore(tmp_path):
    """A rank that fails in the middle of a group step (after its first
    prepare(), while the others run on to their next collective) leaves the
    ranks at different points of the step: the group refuses to step again
    until every rank loads a consistent state, and after the load it steps
    bit-exactly like one GPU from the same checkpoint."""
    mesh = backwards_step()
    grp = GpuGroup(mesh, 3)
    one = GpuSolver(mesh)
    for s in (grp, one):
        _setup_amg_test(s, mesh, 1)
    for _ in range(2):
        grp.step()
        one.step()
    path = str(tmp_path / "ckpt.bin")
    grp.save_state(path)
    assert not grp.needs_restore
    with pytest.raises(RuntimeError, match="rank 1: injected fault after prepare"):
        grp.debug_fault_midstep(1)
    assert grp.needs_restore
    with pytest.raises(RuntimeError, match="needs restore"):
        grp.step()
    # nor can the mid-step state be checkpointed (its load would clear the mark,
    # ADVICE r04): whole group and single rank alike
    with pytest.raises(RuntimeError, match="needs restore"):
        grp.save_state(str(tmp_path / "bad.bin"))
    with pytest.raises(RuntimeError, match="needs restore"):
        grp.ranks[1].save_state(str(tmp_path / "bad1.bin"))
    assert not (tmp_path / "bad.bin").exists() and not (tmp_path / "bad1.bin").exists()
    grp.load_state(path)
    assert not grp.needs_restore
    for step in range(2):
        grp.step()
        one.step()
        _assert_same_fields(grp, one, f"group after restore, step {step}")
        _assert_same_info(grp, one, f"group after restore, step {step}")
    with pytest.raises(RuntimeError, match="rank 0: injected fault after prepare"):
        grp.debug_fault_midstep(0)
    assert grp.needs_restore
    grp.reset()  # the caller accepts the state as is
    assert not grp.needs_restore
    grp.close()
    one.close()
