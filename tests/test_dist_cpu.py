"""Distributed path on CPU (no GPU): world_size-2/3 gloo process groups check
the host side of SURVEY §8(e) -- the slab partition and halo plans the C ABI
builds (cfd_dist_plan) are consistent across ranks, and a gloo transport that
follows them delivers every ghost value; the partition is cut at segment
boundaries of the canonical reduction tree, so R ranks reproduce the
single-GPU reduction bits (checked here on a numpy restatement of the tree,
and on the GPU by tests/test_gpu_dist.py)."""
import os
import socket

import numpy as np
import pytest

from cfd2_amd import default_config, dist_plan
from tests.meshes import backwards_step
from tests.oracle_py import OracleSolver


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, out_q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "cfd-demo2_amd"))
    sys.path.insert(0, root)
    import torch
    import torch.distributed as dist
    from cfd2_amd import dist_plan as plan_of
    from tests.meshes import backwards_step as mk

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mesh = mk()
        P = plan_of(mesh, world, rank)
        plans = [None] * world
        dist.all_gather_object(plans, P)
        # 1. partition covers the mesh exactly, in rank order
        assert plans[0]["c0"] == 0 and plans[-1]["c1"] == mesh.num_cells()
        for q in range(world - 1):
            assert plans[q]["c1"] == plans[q + 1]["c0"]
        # 2. what I send to q is exactly q's ghost list from my range
        off = 0
        for q, sc in zip(P["peers"], P["send"]):
            mine = P["send_ids"][off:off + sc]
            off += sc
            g = plans[q]["ghost"]
            theirs = g[(g >= P["c0"]) & (g < P["c1"])]
            assert np.array_equal(mine, theirs), (rank, q)
        # 3. a gloo halo following the plan delivers f(ghost) to every ghost
        f = lambda ids: (ids.astype(np.float64) * 1.5 + 7.0)  # noqa: E731
        reqs, bufs = [], {}
        off = 0
        for q, sc, rc in zip(P["peers"], P["send"], P["recv"]):
            sbuf = torch.from_numpy(f(P["send_ids"][off:off + sc]))
            off += sc
            rbuf = torch.zeros(rc, dtype=torch.float64)
            bufs[q] = rbuf
            reqs.append(dist.isend(sbuf, q))
            reqs.append(dist.irecv(rbuf, q))
        for r in reqs:
            r.wait()
        ghosts = P["ghost"]
        for q in P["peers"]:
            lo, hi = plans[q]["c0"], plans[q]["c1"]
            want = f(ghosts[(ghosts >= lo) & (ghosts < hi)])
            assert np.array_equal(bufs[q].numpy(), want), (rank, q)
        out_q.put((rank, "ok"))
    except Exception as e:  # reported to the parent
        out_q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_halo_plan_gloo(world):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert all(v == "ok" for v in res.values()), res


def test_plan_single_rank_has_no_ghosts():
    P = dist_plan(backwards_step(), 1, 0)
    assert P["peers"] == [] and len(P["ghost"]) == 0


def _pairwise(v):
    v = list(v)
    while len(v) > 1:
        v = [v[2 * i] + v[2 * i + 1] for i in range(len(v) // 2)]
    return v[0]


def _pow2(n):
    p = 1
    while p < n:
        p *= 2
    return p


def _geom(n):
    g = 0
    while g < 8 and (n >> (g + 1)) >= 16384:
        g += 1
    G = 1 << g
    nch = -(-n // 256)
    return G, nch, -(-nch // G)


def _canonical(leaves):
    """kernels.hpp canonical order: 256-leaf chunk trees, G-chunk segment trees,
    pairwise total over the segments padded to a power of two (float32)."""
    n = len(leaves)
    G, nch, nseg = _geom(n)
    z = np.float32(0)
    chunks = [_pairwise([leaves[c] if c < n else z for c in range(256 * k, 256 * k + 256)]) for k in range(nch)]
    segs = [_pairwise([chunks[k] if k < nch else z for k in range(G * s, G * s + G)]) for s in range(nseg)]
    return _pairwise(segs + [z] * (_pow2(nseg) - nseg))


@pytest.mark.parametrize("n,world", [(1300, 2), (1300, 3), (5000, 4), (40000, 3), (70001, 8)])
def test_partition_keeps_reduction_bits(n, world):
    """Every rank reduces its own segments (the plan's c0/c1 fall on segment
    boundaries); the all-gathered segment values finish to the same float32
    bits as the single-GPU order, for any rank count."""
    from tests.synthetic import strip
    rng = np.random.default_rng(n + world)
    leaves = (rng.standard_normal(n) * 10.0 ** rng.integers(-3, 4, n)).astype(np.float32)
    G, nch, nseg = _geom(n)
    seg_cells = 256 * G
    m = strip(n)
    segs = []
    for r in range(world):
        P = dist_plan(m, world, r)
        c0, c1 = P["c0"], P["c1"]
        assert c0 % seg_cells == 0 and (c1 % seg_cells == 0 or c1 == n)
        own = leaves[c0:c1]  # this rank's cells, chunk-aligned: its segments in its own order
        z = np.float32(0)
        nloc = len(own)
        chunks = [_pairwise([own[c] if c < nloc else z for c in range(256 * k, 256 * k + 256)])
                  for k in range(-(-nloc // 256))]
        for s in range(-(-len(chunks) // G)):
            segs.append(_pairwise([chunks[k] if k < len(chunks) else z for k in range(G * s, G * s + G)]))
    assert len(segs) == nseg
    total = _pairwise(segs + [np.float32(0)] * (_pow2(nseg) - nseg))
    assert total.dtype == np.float32 and total == _canonical(leaves)


def test_oracle_rank_count_invariant():
    """The oracle's distributed semantics are the single-GPU ones (global AMG
    hierarchy, canonical reductions): nranks changes no bit."""
    from tests.test_oracle import setup_amg_test
    mesh = backwards_step()
    for precond in (0, 1):
        a = OracleSolver(mesh, config=default_config(convergence_lag=0))
        b = OracleSolver(mesh, config=default_config(convergence_lag=0), nranks=3)
        for s in (a, b):
            setup_amg_test(s, mesh, precond)
        for _ in range(3):
            a.step()
            b.step()
        assert np.array_equal(a.get_u(), b.get_u()) and np.array_equal(a.get_p(), b.get_p())
