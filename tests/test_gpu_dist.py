"""Distributed solver vs the oracle's distributed semantics.

The in-process group (cfd_group_*) runs R ranks on ONE GPU with the same
halo / all-gather / partition-aware AMG code the RCCL path runs, so the whole
distributed algorithm is checked bit-for-bit here against
OracleSolver(nranks=R) (partition-aware aggregation, rank-segmented
reductions added in rank order).  RCCL itself refuses two ranks on one device;
its transport is exercised by bench.py --gpus N on a multi-GPU node.
"""
import os

import numpy as np
import pytest

from cfd2_amd import GpuGroup, default_config
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


@pytest.mark.parametrize("nranks,precond,rep", [(2, 1, 32768), (2, 1, 50), (3, 1, 50), (2, 0, 32768),
                                                (4, 1, 120)])
def test_group_amg_test_parity(nranks, precond, rep, replicate_rows):
    """tests/amg_test.rs setup, 4 steps, R ranks on one GPU == oracle(R), bit-exact."""
    replicate_rows(rep)
    mesh = backwards_step()
    g = GpuGroup(mesh, nranks)
    o = OracleSolver(mesh, nranks=nranks)
    for s in (g, o):
        _setup_amg_test(s, mesh, precond)
    for k in range(4):
        g.step()
        o.step()
        _assert_same_fields(g, o, f"R={nranks} step {k}")
        _assert_same_info(g, o, f"R={nranks} step {k}")
    if precond == 1:  # rank 0 stores its own rows of the distributed levels
        assert len(g.amg_levels()) == len(o.amg_levels())
    g.close()


@pytest.mark.parametrize("nranks", [2, 3])
def test_group_fixed_schedule_schemes(nranks, replicate_rows):
    """Fixed schedule, SOU scheme (neighbour gradients through the halo), BDF2."""
    replicate_rows(200)
    mesh = channel_obstacle(h=0.03)
    cfg = dict(fixed_outer=3, fixed_inner=10)
    g = GpuGroup(mesh, nranks, config=default_config(**cfg))
    o = OracleSolver(mesh, config=default_config(**cfg), nranks=nranks)
    for s in (g, o):
        _setup_amg_test(s, mesh, 1)
        s.set_scheme(1)
        s.set_time_scheme(1)
    for k in range(3):
        g.step()
        o.step()
        _assert_same_fields(g, o, f"R={nranks} step {k}")
        _assert_same_info(g, o, f"R={nranks} step {k}")
    g.close()


def test_group_bench_geometry(replicate_rows):
    """~100k-cell bench geometry on 4 ranks, bench physics, distributed levels down
    to 4096 rows then the replicated tail: one fixed-schedule step bit-exact."""
    replicate_rows(4096)
    mesh = bench_mesh(0.0055, 30)
    cfg = default_config(fixed_outer=2, fixed_inner=8)
    g = GpuGroup(mesh, 4, config=cfg)
    o = OracleSolver(mesh, config=default_config(fixed_outer=2, fixed_inner=8), nranks=4)
    for s in (g, o):
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
    for k in range(2):
        g.step()
        o.step()
        _assert_same_fields(g, o, f"bench geometry step {k}")
    g.close()


def test_rccl_transport_selftest():
    """The RCCL transport (grouped send/recv + all-gather) on a 1-rank communicator."""
    from cfd2_amd.solver import rccl_selftest
    rccl_selftest(0)


@pytest.mark.parametrize("nranks,rep", [(4, 262144), (8, 262144), (8, 4096)])
def test_group_c1_scale(nranks, rep, replicate_rows):
    """BASELINE configs[1] scale (~1M cells) on 4 and 8 in-process ranks (the
    driver's 8-GPU rank count; rep 4096 keeps five levels distributed down to a
    few hundred rows per rank): one real fixed-schedule step bit-exact vs
    oracle(R)."""
    replicate_rows(rep)
    mesh = bench_mesh(0.001723, 100)
    cfg = dict(fixed_outer=1, fixed_inner=6)
    g = GpuGroup(mesh, nranks, config=default_config(**cfg))
    o = OracleSolver(mesh, config=default_config(**cfg), nranks=nranks)
    for s in (g, o):
        s.set_dt(1e-3)
        s.set_viscosity(0.01)
        s.set_density(1.0)
        s.set_alpha_u(0.7)
        s.set_alpha_p(0.3)
        s.set_precond_type(1)
        s.initialize_history()
    for k in range(2):
        g.step()
        o.step()
        _assert_same_fields(g, o, f"C1 R={nranks} step {k}")
        _assert_same_info(g, o, f"C1 R={nranks} step {k}")
    g.close()


@pytest.mark.parametrize("nranks,rep,which", [(2, 50, "amg_test"), (3, 50, "amg_test"), (4, 4096, "bench_100k"),
                                              (4, 262144, "c1")])
def test_group_amg_device_setup_matches_host(nranks, rep, which, replicate_rows, monkeypatch):
    """Distributed device-side AMG setup: every rank
    builds its rows of the distributed levels and the replicated tail on the
    GPU (aggregate ids of ghost columns by halo exchange, first replicated
    level all-gathered) -- byte-identical, rank by rank and level by level, to
    the host setup that all-gathers the whole fine matrix."""
    replicate_rows(rep)
    mesh = {"amg_test": backwards_step, "bench_100k": lambda: bench_mesh(0.0055, 30),
            "c1": lambda: bench_mesh(0.001723, 100)}[which]()
    groups = []
    for path in ("device", "host"):
        if path == "host":
            monkeypatch.setenv("CFD_AMG_SETUP", "host")
        else:
            monkeypatch.delenv("CFD_AMG_SETUP", raising=False)
        g = GpuGroup(mesh, nranks, config=default_config(fixed_outer=1, fixed_inner=4))
        g.set_dt(1e-3)
        g.set_viscosity(0.01)
        g.set_density(1.0)
        g.set_alpha_u(0.7)
        g.set_alpha_p(0.3)
        g.set_precond_type(1)
        g.initialize_history()
        c = g.constants
        c.time = 0.05
        g.constants = c
        g.step()
        groups.append(g)
    monkeypatch.delenv("CFD_AMG_SETUP", raising=False)
    dev, host = groups
    for r in range(nranks):
        pd, dd = dev.ranks[r].amg_setup_info()
        ph, dh = host.ranks[r].amg_setup_info()
        assert (pd, ph) == (2, 1), f"rank {r}"
        assert dev.ranks[r].amg_levels() == host.ranks[r].amg_levels(), f"rank {r}"
        assert dd == dh, f"rank {r} levels differ: {[i for i, (a, b) in enumerate(zip(dd, dh)) if a != b]}"
    _assert_same_fields(dev, host, f"{which} R={nranks} device vs host setup")
    dev.close()
    host.close()


@pytest.mark.parametrize("refresh", ["1", "0"])
def test_group_amg_rebuild_interval(refresh, replicate_rows, monkeypatch):
    """Re-setting up the distributed hierarchy -- numeric refresh (Galerkin
    fill, packing and the replicated level's value all-gather over the kept
    structure) or full rebuild (device memory released and re-made, halo
    plans included) -- stays bit-exact with oracle(R)."""
    monkeypatch.setenv("CFD_AMG_REFRESH", refresh)
    replicate_rows(50)
    mesh = backwards_step()
    cfg = dict(amg_rebuild_interval=1, fixed_outer=2, fixed_inner=8)
    g = GpuGroup(mesh, 2, config=default_config(**cfg))
    o = OracleSolver(mesh, nranks=2, config=default_config(**cfg))
    for s in (g, o):
        _setup_amg_test(s, mesh, 1)
    for k in range(5):
        g.step()
        o.step()
        _assert_same_fields(g, o, f"R=2 rebuild step {k}")
        _assert_same_info(g, o, f"R=2 rebuild step {k}")
    g.close()


@pytest.mark.parametrize("nranks,which", [(2, "amg_test"), (3, "channel"), (4, "c1")])
def test_group_overlapped_halo_path(nranks, which, replicate_rows, monkeypatch):
    """The interior/boundary split that hides every halo exchange behind the
    interior rows (Solver::overlapped; production: >= 1M rows per rank, so no
    other test reaches it) forced on for every level with >= 64 rows:
    bit-exact vs oracle(R)."""
    monkeypatch.setenv("CFD_OVERLAP_MIN_ROWS", "64")
    replicate_rows(50 if which != "c1" else 4096)
    if which == "c1":
        mesh = bench_mesh(0.001723, 100)
        cfg = dict(fixed_outer=1, fixed_inner=6)
    else:
        mesh = backwards_step() if which == "amg_test" else channel_obstacle(h=0.03)
        cfg = dict(fixed_outer=3, fixed_inner=10)
    g = GpuGroup(mesh, nranks, config=default_config(**cfg))
    o = OracleSolver(mesh, config=default_config(**cfg), nranks=nranks)
    for s in (g, o):
        _setup_amg_test(s, mesh, 1)
        s.set_scheme(1)  # SOU: neighbour gradients through the halo
        s.update_constants()
    for k in range(2):
        g.step()
        o.step()
        _assert_same_fields(g, o, f"overlapped R={nranks} {which} step {k}")
        _assert_same_info(g, o, f"overlapped R={nranks} {which} step {k}")
    g.close()


@pytest.mark.parametrize("env", [{"CFD_HALO_PACK": "1"}, {"CFD_AMG_FULL": "0"}, {"CFD_AMG_TAIL_ROWS": "0"}],
                         ids=lambda e: ",".join(f"{k}={v}" for k, v in e.items()))
def test_group_variants_parity(env, replicate_rows, monkeypatch):
    """Distributed runs through the packed halo path and the alternative AMG
    kernel paths: bit-exact vs oracle(R)."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    replicate_rows(50)
    mesh = backwards_step()
    cfg = dict(fixed_outer=3, fixed_inner=10)
    g = GpuGroup(mesh, 3, config=default_config(**cfg))
    o = OracleSolver(mesh, config=default_config(**cfg), nranks=3)
    for s in (g, o):
        _setup_amg_test(s, mesh, 1)
    for k in range(3):
        g.step()
        o.step()
        _assert_same_fields(g, o, f"{env} step {k}")
        _assert_same_info(g, o, f"{env} step {k}")
    g.close()
