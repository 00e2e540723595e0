"""Distributed path on CPU (no GPU): world_size-2/3 gloo process groups check
the host side of SURVEY §8(e) -- the slab partition and halo plans the C ABI
builds (cfd_dist_plan) are consistent across ranks, and a gloo transport that
follows them delivers every ghost value; plus the oracle's distributed
semantics (partition-aware AMG, rank-ordered reductions) stay a faithful
solver of the same problem."""
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


def test_oracle_distributed_semantics():
    """oracle(R=2): Jacobi preconditioner differs from R=1 only by reduction
    order (fields agree to ~1e-5); AMG with partition-aware aggregation is a
    different but equally converged preconditioner (same step count, close fields)."""
    from tests.test_oracle import setup_amg_test
    mesh = backwards_step()
    for precond, tol in ((0, 1e-4), (1, 2e-2)):
        a = OracleSolver(mesh, config=default_config(convergence_lag=0))
        b = OracleSolver(mesh, config=default_config(convergence_lag=0), nranks=2)
        for s in (a, b):
            setup_amg_test(s, mesh, precond)
        for _ in range(3):
            a.step()
            b.step()
        ua, ub = a.get_u(), b.get_u()
        assert np.all(np.isfinite(ub))
        rel = np.linalg.norm(ua - ub) / np.linalg.norm(ua)
        assert rel < tol, (precond, rel)
    la, lb = a.amg_levels(), b.amg_levels()
    assert la[0] == lb[0] and len(lb) >= len(la) - 1
