"""Distributed solver: rank-count invariant.

The in-process group (cfd_group_*) runs R ranks on ONE GPU with the same
halo / all-gather / distributed-AMG code the RCCL path runs.  The distributed
solver builds the GLOBAL AMG hierarchy (the reference's index-order greedy
aggregation, amg.rs:84-116; aggregates may straddle ranks) and reduces in the
canonical tree order whose segments the ranks own whole (kernels.hpp), so R
ranks must give EXACTLY the bits of one GPU: every test here asserts
GpuGroup(R) == GpuSolver (one GPU) == OracleSolver bit-for-bit.  RCCL itself
refuses two ranks on one device; its transport is exercised by
bench.py --gpus N on a multi-GPU node.
"""
import os

import numpy as np
import pytest

from cfd2_amd import GpuGroup, GpuSolver, default_config
from tests.meshes import backwards_step, bench_mesh, channel_obstacle
from tests.oracle_py import OracleSolver
from tests.test_gpu_parity import _assert_same_fields, _assert_same_info, _setup_amg_test

pytestmark = pytest.mark.gpu


@pytest.fixture
def replicate_rows():
    """Force distributed coarse levels (and the all-gather into the replicated
    tail) even on small meshes."""
    old = os.environ.get("CFD_AMG_REPLICATE_ROWS")
    yield lambda v: os.environ.__setitem__("CFD_AMG_REPLICATE_ROWS", str(v))
    if old is None:
        os.environ.pop("CFD_AMG_REPLICATE_ROWS", None)
    else:
        os.environ["CFD_AMG_REPLICATE_ROWS"] = old


def _bench_physics(s, t0=0.0):
    s.set_dt(1e-3)
    s.set_viscosity(0.01)
    s.set_density(1.0)
    s.set_alpha_u(0.7)
    s.set_alpha_p(0.3)
    s.set_precond_type(1)
    s.initialize_history()
    if t0:
        c = s.constants
        c.time = t0
        s.constants = c


def _three_way(mesh, nranks, cfg, setup, steps, ctx, oracle=True):
    """R ranks, one GPU and (optionally) the oracle, stepped together: all
    bit-identical after every step."""
    g = GpuGroup(mesh, nranks, config=default_config(**cfg))
    one = GpuSolver(mesh, config=default_config(**cfg))
    o = OracleSolver(mesh, config=default_config(**cfg)) if oracle else None
    for s in (g, one) + ((o,) if o else ()):
        setup(s)
    for k in range(steps):
        g.step()
        one.step()
        _assert_same_fields(g, one, f"{ctx} R={nranks} vs 1 GPU, step {k}")
        _assert_same_info(g, one, f"{ctx} R={nranks} vs 1 GPU, step {k}")
        if o:
            o.step()
            _assert_same_fields(one, o, f"{ctx} 1 GPU vs oracle, step {k}")
            _assert_same_info(one, o, f"{ctx} 1 GPU vs oracle, step {k}")
    g.close()
    one.close()


@pytest.mark.parametrize("nranks,precond,rep", [(2, 1, 32768), (2, 1, 50), (3, 1, 50), (2, 0, 32768),
                                                (4, 1, 120), (6, 1, 50)])
def test_group_amg_test_parity(nranks, precond, rep, replicate_rows):
    """tests/amg_test.rs setup, 4 steps: R ranks == one GPU == oracle, bit-exact
    (rep 50: coarse levels distributed, aggregates straddling ranks)."""
    replicate_rows(rep)
    mesh = backwards_step()
    _three_way(mesh, nranks, {}, lambda s: _setup_amg_test(s, mesh, precond), 4, "amg_test")


@pytest.mark.parametrize("nranks", [2, 3])
def test_group_fixed_schedule_schemes(nranks, replicate_rows):
    """Fixed schedule, SOU scheme (neighbour gradients through the halo), BDF2."""
    replicate_rows(200)
    mesh = channel_obstacle(h=0.03)

    def setup(s):
        _setup_amg_test(s, mesh, 1)
        s.set_scheme(1)
        s.set_time_scheme(1)
    _three_way(mesh, nranks, dict(fixed_outer=3, fixed_inner=10), setup, 3, "SOU/BDF2")


@pytest.mark.parametrize("nranks,rep", [(2, 4096), (3, 4096), (4, 4096), (8, 4096), (8, 262144)])
def test_group_bench_geometry(nranks, rep, replicate_rows):
    """~100k-cell bench geometry, bench physics, distributed levels down to 4096
    rows then the replicated tail: two fixed-schedule steps bit-exact, R = 2..8."""
    replicate_rows(rep)
    mesh = bench_mesh(0.0055, 30)
    _three_way(mesh, nranks, dict(fixed_outer=2, fixed_inner=8), lambda s: _bench_physics(s, 0.05), 2,
               "bench_100k")


def test_rccl_transport_selftest():
    """The RCCL transport (grouped send/recv + all-gather) on a 1-rank communicator."""
    from cfd2_amd.solver import rccl_selftest
    rccl_selftest(0)


@pytest.mark.parametrize("nranks,rep", [(2, 262144), (4, 262144), (8, 262144), (8, 4096)])
def test_group_c1_scale(nranks, rep, replicate_rows):
    """BASELINE configs[1] scale (~1M cells) on 2, 4 and 8 in-process ranks (the
    driver's 8-GPU rank count; rep 4096 keeps five levels distributed down to a
    few hundred rows per rank): two fixed-schedule steps, R ranks == one GPU
    bit-exact (the oracle joins for R = 8, rep 4096)."""
    replicate_rows(rep)
    mesh = bench_mesh(0.001723, 100)
    _three_way(mesh, nranks, dict(fixed_outer=1, fixed_inner=6), _bench_physics, 2, "C1",
               oracle=(nranks == 8 and rep == 4096))


def test_group_hierarchy_is_the_global_one(replicate_rows):
    """Every rank of a distributed run holds the replicated AMG levels of the
    single-GPU (device-setup) hierarchy byte for byte: same level sizes, same
    per-level digests of the device images."""
    replicate_rows(4096)
    mesh = bench_mesh(0.0055, 30)
    cfg = default_config(fixed_outer=1, fixed_inner=4)
    g = GpuGroup(mesh, 4, config=cfg)
    one = GpuSolver(mesh, config=cfg)
    for s in (g, one):
        _bench_physics(s, 0.05)
    g.step()
    one.step()
    p1, d1 = one.amg_setup_info()
    assert p1 == 2
    levels1 = one.amg_levels()
    for r in range(4):
        pr, dr = g.ranks[r].amg_setup_info()
        lv = g.ranks[r].amg_levels()
        assert pr == 2 and len(lv) == len(levels1)
        nrep = [i for i, (a, b) in enumerate(zip(lv, levels1)) if a == b and a[0] <= 4096]
        assert nrep, "no replicated level"
        for i in nrep:
            assert dr[i] == d1[i], f"rank {r} level {i}"
    g.close()
    one.close()


@pytest.mark.parametrize("refresh", ["1", "0"])
def test_group_amg_rebuild_interval(refresh, replicate_rows, monkeypatch):
    """Re-setting up the hierarchy every step (a distributed run rebuilds its
    global hierarchy; the single GPU refreshes or rebuilds): bit-exact."""
    monkeypatch.setenv("CFD_AMG_SETUP", "device" if refresh == "1" else "rebuild")
    replicate_rows(50)
    mesh = backwards_step()
    _three_way(mesh, 2, dict(amg_rebuild_interval=1, fixed_outer=2, fixed_inner=8),
               lambda s: _setup_amg_test(s, mesh, 1), 5, "rebuild")


@pytest.mark.parametrize("nranks,which", [(2, "amg_test"), (3, "channel"), (4, "c1")])
def test_group_overlapped_halo_path(nranks, which, replicate_rows, monkeypatch):
    """The interior/boundary split that hides every halo exchange behind the
    interior rows (Solver::overlapped, and the AMG restriction / prolongation
    split around the residual / coarse-x exchanges of straddling aggregates;
    production: >= 1M rows per rank, so no other test reaches it) forced on
    for every level with >= 64 rows."""
    monkeypatch.setenv("CFD_OVERLAP_MIN_ROWS", "64")
    replicate_rows(50 if which != "c1" else 4096)
    if which == "c1":
        mesh = bench_mesh(0.001723, 100)
        cfg = dict(fixed_outer=1, fixed_inner=6)
    else:
        mesh = backwards_step() if which == "amg_test" else channel_obstacle(h=0.03)
        cfg = dict(fixed_outer=3, fixed_inner=10)

    def setup(s):
        _setup_amg_test(s, mesh, 1)
        s.set_scheme(1)  # SOU: neighbour gradients through the halo
        s.update_constants()
    _three_way(mesh, nranks, cfg, setup, 2, f"overlapped {which}", oracle=(which != "c1"))


@pytest.mark.parametrize("env", [{"CFD_AMG_FULL": "0"}, {"CFD_AMG_TAIL_ROWS": "0"},
                                 {"CFD_AMG_FUSED_PROLONG_ROWS": "0"}, {"CFD_SMALL_MESH_FORMS": "0"},
                                 # every level pair of the replicated levels in one launch
                                 {"CFD_AMG_FUSED_PAIR": "2", "CFD_AMG_TAIL_ROWS": "0"},
                                 # every level split around its exchanges
                                 {"CFD_OVERLAP_MIN_ROWS": "64", "CFD_AMG_TAIL": "global"}],
                         ids=lambda e: ",".join(f"{k}={v}" for k, v in e.items()))
def test_group_variants_parity(env, replicate_rows, monkeypatch):
    """Distributed runs through the alternative AMG kernel paths: bit-exact.
    (The packed halo path -- non-contiguous send lists -- is the Voronoi
    meshes' own: tests/test_voronoi.py test_voronoi_group_parity.)"""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    replicate_rows(50)
    mesh = backwards_step()
    _three_way(mesh, 3, dict(fixed_outer=3, fixed_inner=10), lambda s: _setup_amg_test(s, mesh, 1), 3, str(env))


@pytest.mark.parametrize("nranks,rep,which", [(4, 4096, "bench_100k"), (3, 50, "amg_test"), (8, 4096, "c1")])
def test_group_device_setup_equals_host_setup(nranks, rep, which, replicate_rows, monkeypatch):
    """The distributed DEVICE setup (aggregation pipeline over the ranks,
    member rows of straddling aggregates imported from their owners, Galerkin
    and packing on each rank's GPU) builds every rank's level images byte for
    byte as the host setup of the all-gathered global matrix does: equal
    per-rank, per-level digests, then equal fields after two steps."""
    replicate_rows(rep)
    mesh = {"bench_100k": lambda: bench_mesh(0.0055, 30), "amg_test": backwards_step,
            "c1": lambda: bench_mesh(0.001723, 100)}[which]()
    cfg = default_config(fixed_outer=1, fixed_inner=6)
    groups = {}
    for path in ("host", "device"):
        monkeypatch.setenv("CFD_AMG_SETUP", path)
        g = GpuGroup(mesh, nranks, config=cfg)
        _bench_physics(g, 0.05)
        g.step()
        groups[path] = g
    monkeypatch.delenv("CFD_AMG_SETUP")
    h, d = groups["host"], groups["device"]
    for r in range(nranks):
        ph, dh = h.ranks[r].amg_setup_info()
        pd, dd = d.ranks[r].amg_setup_info()
        assert (ph, pd) == (1, 2)
        assert h.ranks[r].amg_levels() == d.ranks[r].amg_levels(), f"rank {r}"
        assert dh == dd, f"rank {r}: level digests differ at {[i for i, (a, b) in enumerate(zip(dh, dd)) if a != b]}"
    d.step()
    h.step()
    _assert_same_fields(d, h, f"{which} R={nranks} device vs host setup")
    _assert_same_info(d, h, f"{which} R={nranks} device vs host setup")
    h.close()
    d.close()


def test_comm_timing_categories_and_bits(replicate_rows):
    """cfd_comm_timing (the multi-GPU line's exposed-communication fields):
    with timing on, every category of the distributed step shows up with its
    calls and non-negative times, AMG halos per level, and the bracketing
    events change no result bit (group == one GPU == oracle)."""
    replicate_rows(64)  # distributed coarse levels + the replicated-level all-gather
    mesh = backwards_step()
    grp = GpuGroup(mesh, 3)
    one = GpuSolver(mesh)
    orc = OracleSolver(mesh)
    for s in (grp, one, orc):
        _setup_amg_test(s, mesh, 1)
    for r in grp.ranks:
        r.comm_timing_enable(True)
    for step in range(2):
        grp.step()
        one.step()
        orc.step()
        _assert_same_fields(grp, one, f"timed group step {step}")
        _assert_same_fields(one, orc, f"one GPU step {step}")
    for r in grp.ranks:
        t = r.comm_timing()
        cats = {(e["category"], e["level"]) for e in t}
        for need in [("krylov_halo", -1), ("state_halo", -1), ("reduction_allgather", -1),
                     ("replicated_level_allgather", -1), ("amg_halo", 0)]:
            assert need in cats, (need, cats)
        for e in t:
            assert e["calls"] > 0 and e["wait_us"] >= 0.0 and e["comm_us"] >= 0.0, e
        r.comm_timing_enable(False)
        assert r.comm_timing() == []
    grp.close()
    one.close()


# ---- partition-aware aggregation (cfd_config.amg_local_aggregation) --------
# "aggregation restricted to owned rows (block-diagonal P/R,
# local restriction and prolongation)".  Opt-in: the hierarchy then depends on
# the rank count, so the bar is GpuGroup(R, local) == OracleSolver(R, local),
# bit for bit (the oracle runs the same per-rank greedy pass on the same
# partition), and the V-cycle drops the residual and coarse-x halos of every
# distributed level.

@pytest.mark.parametrize("nranks,rep,which", [(2, 50, "amg_test"), (4, 120, "amg_test"), (8, 4096, "bench_100k"),
                                              (2, 262144, "c1"), (8, 4096, "c1")])
def test_group_local_aggregation_parity(nranks, rep, which, replicate_rows):
    replicate_rows(rep)
    if which == "amg_test":
        mesh = backwards_step()
        cfg = dict(amg_local_aggregation=1)
        setup = lambda s: _setup_amg_test(s, mesh, 1)  # noqa: E731
        steps = 4
    else:
        mesh = bench_mesh(0.0055, 30) if which == "bench_100k" else bench_mesh(0.001723, 100)
        cfg = dict(amg_local_aggregation=1, fixed_outer=1, fixed_inner=6)
        setup = lambda s: _bench_physics(s, 0.05)  # noqa: E731
        steps = 2
    g = GpuGroup(mesh, nranks, config=default_config(**cfg))
    o = OracleSolver(mesh, config=default_config(**cfg), nranks=nranks)
    glob = OracleSolver(mesh, config=default_config(**{**cfg, "amg_local_aggregation": 0}), nranks=nranks)
    for s in (g, o, glob):
        setup(s)
    for k in range(steps):
        for s in (g, o, glob):
            s.step()
        _assert_same_fields(g, o, f"local {which} R={nranks} vs oracle(R, local), step {k}")
        _assert_same_info(g, o, f"local {which} R={nranks} vs oracle(R, local), step {k}")
    # a different hierarchy from the global one (the mode did something), the
    # same depth on every rank as the oracle's, level 0 split over the ranks,
    # the coarsest level replicated
    ol = o.amg_levels()
    assert ol != glob.amg_levels()
    for r in g.ranks:
        rl = r.amg_levels()
        assert len(rl) == len(ol) and rl[-1] == ol[-1], (rl, ol)
    assert sum(r.amg_levels()[0][0] for r in g.ranks) == ol[0][0]
    g.close()


@pytest.mark.parametrize("nranks,rep,which", [(3, 50, "amg_test"), (8, 4096, "c1")])
def test_group_local_aggregation_host_setup(nranks, rep, which, replicate_rows, monkeypatch):
    """Partition-aware mode: the device setup (per-rank greedy pass, no
    imported member rows) builds the host setup's level images byte for byte."""
    replicate_rows(rep)
    mesh = backwards_step() if which == "amg_test" else bench_mesh(0.001723, 100)
    cfg = default_config(fixed_outer=1, fixed_inner=6, amg_local_aggregation=1)
    groups = {}
    for path in ("host", "device"):
        monkeypatch.setenv("CFD_AMG_SETUP", path)
        g = GpuGroup(mesh, nranks, config=cfg)
        _bench_physics(g, 0.05)
        g.step()
        groups[path] = g
    monkeypatch.delenv("CFD_AMG_SETUP")
    h, d = groups["host"], groups["device"]
    for r in range(nranks):
        assert h.ranks[r].amg_levels() == d.ranks[r].amg_levels(), f"rank {r}"
        assert h.ranks[r].amg_setup_info()[1] == d.ranks[r].amg_setup_info()[1], f"rank {r} digests"
    d.step()
    h.step()
    _assert_same_fields(d, h, f"local {which} R={nranks} device vs host setup")
    h.close()
    d.close()


def test_group_local_aggregation_fewer_exchanges(replicate_rows):
    """The partition-aware mode removes two halo exchanges per distributed
    level and V-cycle (the residual before the restriction, the coarse x
    before the prolongation): exchanges per FGMRES iteration, global vs local."""
    replicate_rows(4096)
    mesh = bench_mesh(0.0055, 30)
    per_it = {}
    for local in (0, 1):
        g = GpuGroup(mesh, 4, config=default_config(fixed_outer=1, fixed_inner=8, amg_local_aggregation=local))
        _bench_physics(g, 0.05)
        g.step()
        for r in g.ranks:
            r.comm_stats(reset=True)
        g.step()
        its = g.step_info().total_linear_iterations
        per_it[local] = max(r.comm_stats()["exchanges"] for r in g.ranks) / its
        g.close()
    assert per_it[1] < per_it[0], per_it


@pytest.mark.parametrize("refresh", ["1", "0"])
def test_group_local_aggregation_rebuild(refresh, replicate_rows, monkeypatch):
    """Partition-aware mode with the AMG re-setup every step (numeric refresh
    over the per-rank structure, or a full rebuild): == oracle(R, local)."""
    monkeypatch.setenv("CFD_AMG_SETUP", "device" if refresh == "1" else "rebuild")
    replicate_rows(50)
    mesh = backwards_step()
    cfg = dict(amg_local_aggregation=1, amg_rebuild_interval=1, fixed_outer=2, fixed_inner=8)
    g = GpuGroup(mesh, 3, config=default_config(**cfg))
    o = OracleSolver(mesh, config=default_config(**cfg), nranks=3)
    for s in (g, o):
        _setup_amg_test(s, mesh, 1)
    for k in range(5):
        g.step()
        o.step()
        _assert_same_fields(g, o, f"local rebuild refresh={refresh} step {k}")
        _assert_same_info(g, o, f"local rebuild refresh={refresh} step {k}")
    g.close()
