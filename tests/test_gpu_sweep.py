"""Seeded parity sweep: random geometries (backwards step, channel + obstacle,
rectangular channel, graded meshes with hanging faces; cut-cell, seeded
Voronoi and Delaunay meshes), random physics and
solver settings, 1-3 ranks -- the HIP path must equal the oracle bit for bit
on every case.  Each case is a few thousand cells and two or three steps."""
import os
import random

import numpy as np
import pytest

from cfd2_amd import GpuGroup, GpuSolver, default_config
from cfd2_amd.mesh import (BackwardsStep, ChannelWithObstacle, RectangularChannel, generate_cut_cell_mesh,
                           generate_delaunay_mesh, generate_voronoi_mesh)
from tests.oracle_py import OracleSolver
from tests.synthetic import max_ranks
from tests.test_gpu_parity import _assert_same_fields, _assert_same_info

pytestmark = pytest.mark.gpu


def _case(seed):
    rng = random.Random(seed)
    kind = rng.choice(["step", "obstacle", "rect", "graded", "voronoi", "delaunay"])
    h = rng.uniform(0.045, 0.07) * float(os.environ.get("CFD_SWEEP_H_SCALE", "1"))  # < 1: bigger meshes
    mn = mx = h
    if kind == "step":
        length = rng.uniform(2.0, 3.5)
        geo = BackwardsStep(length=length, height_inlet=rng.uniform(0.3, 0.7), height_outlet=1.0,
                            step_x=rng.uniform(0.3, 1.0))
        dom = (length, 1.0)
    elif kind == "rect":
        length = rng.uniform(1.0, 3.0)
        geo = RectangularChannel(length=length, height=1.0)
        dom = (length, 1.0)
    elif kind in ("voronoi", "delaunay") and rng.random() < 0.5:
        length = rng.uniform(1.5, 3.0)
        geo = BackwardsStep(length=length, height_inlet=rng.uniform(0.3, 0.7), height_outlet=1.0,
                            step_x=rng.uniform(0.3, 1.0))
        dom = (length, 1.0)
    else:
        geo = ChannelWithObstacle(length=3.0, height=1.0,
                                  obstacle_center=(rng.uniform(0.6, 1.6), rng.uniform(0.35, 0.65)),
                                  obstacle_radius=rng.uniform(0.08, 0.22))
        dom = (3.0, 1.0)
        if kind == "graded":  # quadtree refinement towards the obstacle: hanging faces, 5+-face cells
            mn, mx = h * 0.5, h * 2.0
    if kind in ("voronoi", "delaunay"):  # seeded polygonal / triangle meshes (voronoi.cpp)
        gen = generate_voronoi_mesh if kind == "voronoi" else generate_delaunay_mesh
        mesh = gen(geo, h * 0.8, h * 2.0, 1.2, dom, seed=rng.randrange(1 << 20))
    else:
        mesh = generate_cut_cell_mesh(geo, mn, mx, 1.2, dom)
    mesh.smooth(geo, 0.3, rng.choice([0, 20]))
    cfg = dict(convergence_lag=rng.choice([0, 1]))
    if rng.random() < 0.6:
        cfg.update(fixed_outer=rng.choice([2, 3]), fixed_inner=rng.choice([6, 12, 20]))
    if rng.random() < 0.25:
        cfg.update(amg_rebuild_interval=1)
    phys = dict(dt=rng.choice([1e-3, 5e-3, 1e-2]), nu=rng.choice([1e-3, 1e-2]), scheme=rng.choice([0, 1, 2]),
                time_scheme=rng.choice([0, 1]), precond=rng.choice([0, 1, 1]), alpha_u=rng.choice([0.7, 0.9]),
                alpha_p=rng.choice([0.3, 0.9]))
    nranks = rng.choice([1, 1, 2, 3] + ([4, 6, 8] if os.environ.get("CFD_SWEEP_MANY_RANKS") else []))
    useed = rng.randrange(1 << 30)
    # round 5 (drawn after the earlier choices, so older seeds keep their cases):
    # the partition-aware AMG mode on several ranks (the oracle runs the same
    # mode at the same rank count), hipGraph replay on one GPU
    if rng.random() < 0.35:
        cfg.update(amg_local_aggregation=1)
    graph = rng.random() < 0.3
    # round 6: every candidate AMG level pair in one launch, the tail off (so
    # that these small meshes have candidate pairs)
    pairs = rng.random() < 0.3
    # round 6: the reference-semantics test mode (one GPU; the oracle with the
    # same flags): its reduction order, the in-place smoother / racy prepare
    # with ordered workgroups, the clamped restrict rows
    refsem = rng.choice([4, 13, 15, 1, 2, 8]) if rng.random() < 0.25 else 0
    return kind, mesh, cfg, phys, nranks, useed, graph, pairs, refsem


def _setup(s, mesh, phys, useed):
    s.set_dt(phys["dt"])
    s.set_viscosity(phys["nu"])
    s.set_density(1.0)
    s.set_alpha_u(phys["alpha_u"])
    s.set_alpha_p(phys["alpha_p"])
    s.set_scheme(phys["scheme"])
    s.set_time_scheme(phys["time_scheme"])
    a = mesh.arrays()
    r = np.random.default_rng(useed)
    u = np.zeros((mesh.num_cells(), 2))
    u[:, 0] = 0.5 + 0.5 * np.sin(3.0 * a["cell_cx"]) * np.cos(2.0 * a["cell_cy"])
    u[:, 1] = 0.1 * r.standard_normal(mesh.num_cells())
    s.set_u(u)
    s.initialize_history()
    s.set_precond_type(phys["precond"])
    s.update_constants()


_SEED0 = int(os.environ.get("CFD_SWEEP_SEED0", "0"))  # fresh cases: CFD_SWEEP_SEED0=1000


@pytest.mark.parametrize("seed", range(_SEED0, _SEED0 + int(os.environ.get("CFD_SWEEP_CASES", "32"))))  # wider: CFD_SWEEP_CASES=N
def test_random_case_parity(seed, monkeypatch):
    kind, mesh, cfg, phys, nranks, useed, graph, pairs, refsem = _case(seed)
    # ranks own whole reduction segments (>= 256 cells): small meshes take fewer ranks
    nranks = min(nranks, max_ranks(mesh.num_cells()))
    monkeypatch.setenv("CFD_AMG_REPLICATE_ROWS", "200")  # distributed coarse levels on these small meshes
    if pairs:
        monkeypatch.setenv("CFD_AMG_FUSED_PAIR", "2")
        monkeypatch.setenv("CFD_AMG_TAIL_ROWS", "0")
    c = default_config(**cfg)
    g = GpuSolver(mesh, config=c) if nranks == 1 else GpuGroup(mesh, nranks, config=c)
    if nranks == 1 and graph:
        g.graph_enable(True)
    o = OracleSolver(mesh, config=default_config(**cfg), nranks=nranks)
    if nranks > 1:
        refsem = 0
    if refsem:
        g.debug_reference_semantics(refsem)
        o.set_semantics(refsem)
    for s in (g, o):
        _setup(s, mesh, phys, useed)
    ctx = (f"seed {seed}: {kind} {mesh.num_cells()} cells, R={nranks}, {cfg}, {phys}, graph={graph}, pairs={pairs}, "
           f"reference semantics {refsem}")
    for k in range(3):
        g.step()
        o.step()
        _assert_same_fields(g, o, f"{ctx} step {k}")
        _assert_same_info(g, o, f"{ctx} step {k}")
    if nranks > 1:
        g.close()
