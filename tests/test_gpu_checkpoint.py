"""Checkpoint / resume (cfd_state_save / cfd_state_load).

The bar: a solver resumed from a checkpoint steps BIT-IDENTICALLY to the one
that wrote it (fields, step_info, AMG hierarchy), and both to the oracle; the
file is rank-count independent (written by R ranks, re-written by R' ranks:
same bytes).  Schemes cover what a step reads from earlier steps: BDF2 reads
both old ring slots, the lagged convergence model carries the last FGMRES
residual read across steps, and the AMG hierarchy is built once from the
first step's matrix (the resumed solver must rebuild it from that matrix,
not its own first one).
"""
import numpy as np
import pytest

from cfd2_amd import GpuGroup, GpuSolver, default_config
from cfd2_amd.state import read_state, write_state
from tests.meshes import backwards_step, channel_obstacle
from tests.oracle_py import OracleSolver
from tests.test_gpu_parity import _assert_same_fields, _assert_same_info, _setup_amg_test

pytestmark = pytest.mark.gpu


def _setup(s, mesh, precond, time_scheme, scheme):
    _setup_amg_test(s, mesh, precond)
    s.set_time_scheme(time_scheme)
    s.set_scheme(scheme)
    s.update_constants()


def _snap(s):
    i = s.step_info()
    return (s.get_u(), s.get_p(), s.get_d_p(), i.outer_iterations, i.total_linear_iterations,
            i.outer_residual_u, i.outer_residual_p, i.degenerate_count, i.steady_state_count)


def _same(a, b, ctx):
    for k, (x, y) in enumerate(zip(a, b)):
        assert np.array_equal(x, y), f"{ctx}: item {k} differs"


@pytest.mark.parametrize("precond,time_scheme,scheme,lag,rebuild",
                         [(1, 1, 0, 1, 0), (1, 0, 1, 0, 0), (0, 1, 2, 1, 0), (1, 0, 0, 1, 2)])
def test_resume_is_bitexact(precond, time_scheme, scheme, lag, rebuild, tmp_path):
    mesh = backwards_step()
    cfg = default_config(convergence_lag=lag, amg_rebuild_interval=rebuild)
    a = GpuSolver(mesh, config=cfg)
    o = OracleSolver(mesh, config=default_config(convergence_lag=lag, amg_rebuild_interval=rebuild))
    for s in (a, o):
        _setup(s, mesh, precond, time_scheme, scheme)
    k0, k1 = 3, 3
    for _ in range(k0):
        a.step()
        o.step()
    path = str(tmp_path / "state.bin")
    a.save_state(path)
    ref = []
    for k in range(k1):
        a.step()
        o.step()
        _assert_same_fields(a, o, f"uninterrupted step {k0 + k}")
        _assert_same_info(a, o, f"uninterrupted step {k0 + k}")
        ref.append(_snap(a))
    b = GpuSolver(mesh, config=cfg)  # fresh: default constants, zero fields
    b.load_state(path)
    for k in range(k1):
        b.step()
        _same(_snap(b), ref[k], f"resumed step {k0 + k}")
    if precond == 1:
        assert b.amg_levels() == a.amg_levels()
        assert b.amg_setup_info()[1] == a.amg_setup_info()[1], "AMG level images differ"


def test_file_contents_and_python_round_trip(tmp_path):
    mesh = backwards_step()
    g = GpuSolver(mesh)
    _setup(g, mesh, 1, 1, 0)
    for _ in range(2):
        g.step()
    path = str(tmp_path / "s.bin")
    g.save_state(path)
    st = read_state(path)
    assert st.num_cells == mesh.num_cells() and st.step_index == 2
    assert np.array_equal(st.current["u"].astype(np.float64), g.get_u())
    assert np.array_equal(st.current["p"].astype(np.float64), g.get_p())
    assert np.array_equal(st.current["d_p"].astype(np.float64), g.get_d_p())
    assert st.amg_val is not None and st.amg_rowptr[-1] == st.amg_val.size
    assert st.have_prev and len(st.variance) == 2
    assert st.constants.time == g.constants.time and st.constants.precond_type == 1
    # the Python writer reproduces the native file byte for byte
    path2 = str(tmp_path / "s2.bin")
    write_state(path2, st)
    with open(path, "rb") as f1, open(path2, "rb") as f2:
        assert f1.read() == f2.read()


def test_rank_count_independent_file(tmp_path, monkeypatch):
    """R=2 writes; R=1, 3 and 6 (one 256-cell segment per rank) load and re-write
    the same bytes; the R=2 resume continues bit-exactly (and equals the
    oracle, which has no rank semantics of its own)."""
    monkeypatch.setenv("CFD_AMG_REPLICATE_ROWS", "50")
    mesh = backwards_step()
    g2 = GpuGroup(mesh, 2)
    o = OracleSolver(mesh, nranks=2)
    for s in (g2, o):
        _setup(s, mesh, 1, 1, 0)
    for _ in range(2):
        g2.step()
        o.step()
    p2 = str(tmp_path / "r2.bin")
    g2.save_state(p2)
    raw = open(p2, "rb").read()
    assert read_state(p2).nranks == 2 and read_state(p2).amg_local_aggregation == 0

    def masked(b):  # every byte but the header's record of the saving rank count (offset 344)
        return b[:344] + b[348:]
    for r in (1, 3, 6):
        h = GpuSolver(mesh) if r == 1 else GpuGroup(mesh, r)
        h.load_state(p2)
        pr = str(tmp_path / f"r{r}.bin")
        h.save_state(pr)
        assert read_state(pr).nranks == r
        assert masked(open(pr, "rb").read()) == masked(raw), f"R={r} re-save differs"
        h.close()
    g2.step()
    o.step()
    b = GpuGroup(mesh, 2)
    b.load_state(p2)
    b.step()
    _assert_same_fields(b, o, "R=2 resumed")
    _assert_same_info(b, o, "R=2 resumed")
    g2.close()
    b.close()


def test_load_errors(tmp_path):
    mesh = backwards_step()
    g = GpuSolver(mesh)
    _setup(g, mesh, 1, 0, 0)
    g.step()
    path = str(tmp_path / "s.bin")
    g.save_state(path)
    other = GpuSolver(channel_obstacle(h=0.03))
    with pytest.raises(RuntimeError, match="different mesh"):
        other.load_state(path)
    bad = str(tmp_path / "trunc.bin")
    with open(path, "rb") as f, open(bad, "wb") as t:
        t.write(f.read()[:-4])
    fresh = GpuSolver(mesh)
    with pytest.raises(RuntimeError, match="truncated"):
        fresh.load_state(bad)
    with pytest.raises(RuntimeError, match="cannot open"):
        fresh.load_state(str(tmp_path / "missing.bin"))
    fresh.load_state(path)  # a failed load leaves the solver usable
    fresh.step()
    assert np.all(np.isfinite(fresh.get_u()))


def test_load_into_a_running_solver(tmp_path):
    """Loading drops the solver's own hierarchy (built from a different matrix)
    and resumes bit-exactly: the same solver rewinds and replays."""
    mesh = backwards_step()
    g = GpuSolver(mesh)
    _setup(g, mesh, 1, 1, 0)
    g.step()
    path = str(tmp_path / "s.bin")
    g.save_state(path)
    ref = []
    for _ in range(3):
        g.step()
        ref.append(_snap(g))
    digests = g.amg_setup_info()[1]
    h = GpuSolver(mesh)
    _setup(h, mesh, 1, 0, 2)  # different scheme: its first hierarchy differs
    for _ in range(2):
        h.step()
    assert h.amg_setup_info()[1] != digests
    for s in (g, h):
        s.load_state(path)
        for k in range(3):
            s.step()
            _same(_snap(s), ref[k], f"replay step {k}")
        assert s.amg_setup_info()[1] == digests


def test_partition_aware_file_records_mode_and_rank_count(tmp_path, capfd):
    """A partition-aware run (amg_local_aggregation=1) records its mode and rank
    count; loading it under another rank count or mode warns (the hierarchy
    rebuilt from the saved matrix differs); the same count and mode load
    silently (include/cfd2_amd.h, cfd_state_file_header)."""
    import os
    old = os.environ.get("CFD_AMG_REPLICATE_ROWS")
    os.environ["CFD_AMG_REPLICATE_ROWS"] = "50"
    try:
        mesh = backwards_step()
        cfg = default_config(amg_local_aggregation=1, fixed_outer=1, fixed_inner=6)
        g = GpuGroup(mesh, 2, config=cfg)
        _setup(g, mesh, 1, 1, 0)
        g.step()
        p = str(tmp_path / "local2.bin")
        g.save_state(p)
        st = read_state(p)
        assert st.amg_local_aggregation == 1 and st.nranks == 2 and st.amg_val is not None
        capfd.readouterr()
        same = GpuGroup(mesh, 2, config=cfg)
        same.load_state(p)
        assert "cfd_state_load" not in capfd.readouterr().err
        other = GpuGroup(mesh, 3, config=cfg)
        other.load_state(p)
        assert "amg_local_aggregation=1 on 2 rank(s)" in capfd.readouterr().err
        glob = GpuGroup(mesh, 2, config=default_config(fixed_outer=1, fixed_inner=6))
        glob.load_state(p)
        assert "this solver runs amg_local_aggregation=0" in capfd.readouterr().err
        for h in (g, same, other, glob):
            h.close()
    finally:
        if old is None:
            os.environ.pop("CFD_AMG_REPLICATE_ROWS", None)
        else:
            os.environ["CFD_AMG_REPLICATE_ROWS"] = old
