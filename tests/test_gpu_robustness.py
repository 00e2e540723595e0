"""Failure paths of the hot path on the GPU, against the oracle.

- Divergence: the reference panics on a NaN linear residual
  (coupled_solver.rs:344-346) and on NaN outer residuals (:421-426); the C ABI
  returns CFD_ERR_DIVERGED (status 3) instead.  A NaN injected through set_u
  must stop the GPU solver and the oracle at the same step with that status.
- Wide AMG rows: a level whose rows exceed the u8 row-length layout is built
  with 16-bit lengths and run by the one-workgroup tail kernels.
  CFD_AMG_WIDE_LIMIT lowers the layout limit so small meshes take that path;
  the results must stay bit-exact.
"""
import numpy as np
import pytest

from cfd2_amd import GpuSolver, default_config
from tests.meshes import backwards_step
from tests.oracle_py import OracleSolver
from tests.test_gpu_parity import _assert_same_fields, _assert_same_info, _setup_amg_test

pytestmark = pytest.mark.gpu


def _step_until_error(s, nsteps):
    for k in range(nsteps):
        try:
            s.step()
        except RuntimeError as e:
            return k, str(e)
    return None, ""


@pytest.mark.parametrize("precond", [0, 1])
@pytest.mark.parametrize("at_step", [0, 2])
def test_nan_state_diverges_like_reference(precond, at_step):
    """A NaN velocity (set_u clobbers the state, as solver.rs:9-21) reaches the
    linear residual: CFD_ERR_DIVERGED at the same step on GPU and oracle."""
    mesh = backwards_step()
    g = GpuSolver(mesh, config=default_config())
    o = OracleSolver(mesh, config=default_config())
    for s in (g, o):
        _setup_amg_test(s, mesh, precond)
    for _ in range(at_step):  # some healthy steps first (AMG hierarchy built)
        g.step()
        o.step()
    _assert_same_fields(g, o, "before the NaN")
    u = g.get_u().copy()
    u[len(u) // 3, 0] = np.nan
    g.set_u(u)
    o.set_u(u)
    kg, mg = _step_until_error(g, 3)
    ko, mo = _step_until_error(o, 3)
    assert kg == ko == 0, (kg, ko, mg, mo)
    assert "status 3" in mg and "Diverged" in mg, mg
    assert "Diverged" in mo, mo
    assert ("linear residual" in mg) == ("linear residual" in mo)


@pytest.mark.parametrize("tail", ["blob2", "global"])
def test_wide_amg_rows_take_the_16bit_path_bitexact(monkeypatch, tail):
    """Coarse levels wider than the (lowered) layout limit: host setup path,
    16-bit row lengths, the whole coarse cycle in the tail kernel (LDS-resident
    or global-memory); fields and step statistics bit-exact vs the oracle."""
    mesh = backwards_step()
    monkeypatch.setenv("CFD_AMG_WIDE_LIMIT", "5")  # level 0: 4, coarse levels: 6
    monkeypatch.setenv("CFD_AMG_TAIL", tail)
    g = GpuSolver(mesh, config=default_config())
    o = OracleSolver(mesh, config=default_config())
    for s in (g, o):
        _setup_amg_test(s, mesh, 1)
    for k in range(4):
        g.step()
        o.step()
        _assert_same_fields(g, o, f"wide step {k}")
        _assert_same_info(g, o, f"wide step {k}")
    path, _ = g.amg_setup_info()
    assert path == 1, "a wide level must send the setup to the host path"
    monkeypatch.delenv("CFD_AMG_WIDE_LIMIT")
    g2 = GpuSolver(mesh, config=default_config())
    _setup_amg_test(g2, mesh, 1)
    g2.step()
    assert g2.amg_setup_info()[0] == 2, "without wide rows the device setup runs"


def test_aligned_slot_ell_bitexact():
    """Coupled-matrix ELL with aligned slots (gaps where a wall removes a
    neighbour; Topology::tslot) on a quad mesh: the oracle's bits (amg_test
    setup, Jacobi and AMG preconditioners).  The positional layout of wider
    meshes (ws > 8) is the Voronoi meshes' own (tests/test_voronoi.py)."""
    mesh = backwards_step()
    for precond in (0, 1):
        g = GpuSolver(mesh, config=default_config())
        o = OracleSolver(mesh, config=default_config())
        for s in (g, o):
            _setup_amg_test(s, mesh, precond)
        for k in range(3):
            g.step()
            o.step()
            _assert_same_fields(g, o, f"precond={precond} step {k}")
            _assert_same_info(g, o, f"precond={precond} step {k}")
        g.close()
