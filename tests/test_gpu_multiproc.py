"""The distributed solver with one PROCESS per rank, as
bench.py --gpus N runs it, on a one-GPU box: RCCL refuses two ranks on one
device, so the ranks use the host-staged transport (cfd_solver_create_dist_host,
gloo underneath) -- everything else (per-process mesh, slab topology, halo
plans, device AMG setup with halo-exchanged aggregates, rank-ordered
reductions) is the production code.  Fields must equal the oracle's
distributed semantics (OracleSolver(nranks=R)) bit-for-bit."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from cfd2_amd.state import read_state
from tests.meshes import backwards_step
from tests.oracle_py import OracleSolver
from tests.test_gpu_parity import _setup_amg_test

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("nranks,overlap,local", [(2, False, 0), (3, False, 0), (2, True, 0), (3, False, 1)])
def test_multiprocess_host_transport_parity(nranks, overlap, local, tmp_path, monkeypatch):
    """local: the partition-aware AMG mode (cfd_config.amg_local_aggregation),
    against the oracle run with the same mode and rank count."""
    steps = 3
    monkeypatch.setenv("CFD_AMG_REPLICATE_ROWS", "50")  # the oracle's partitioned levels (local mode) follow it
    env = dict(os.environ, CFD_AMG_REPLICATE_ROWS="50", MASTER_ADDR="127.0.0.1", CFD_TEST_AMG_LOCAL=str(local))
    if overlap:  # the interior/boundary split of every halo'd launch (production: >= 1M rows per rank)
        env["CFD_OVERLAP_MIN_ROWS"] = "64"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nranks}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(ROOT, "tests", "mp_worker.py"), str(tmp_path), str(steps), str(tmp_path / "state.bin")]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    mesh = backwards_step()
    # the replication threshold moves work, not results -- except in the local mode, where it
    # decides which levels aggregate per rank (the same threshold on both sides)
    from cfd2_amd import default_config
    o = OracleSolver(mesh, config=default_config(amg_local_aggregation=local), nranks=nranks)
    _setup_amg_test(o, mesh, 1)
    for _ in range(steps):
        o.step()
    n = mesh.num_cells()
    u, p, dp = np.zeros((n, 2)), np.zeros(n), np.zeros(n)
    for k in range(nranks):
        d = np.load(tmp_path / f"rank{k}.npz")
        c0, c1 = int(d["c0"]), int(d["c1"])
        u[c0:c1], p[c0:c1], dp[c0:c1] = d["u"], d["p"], d["d_p"]
        io = o.step_info()
        assert int(d["outer_iterations"]) == io.outer_iterations
        assert float(d["res_p"]) == io.outer_residual_p
    assert np.array_equal(u, o.get_u())
    assert np.array_equal(p, o.get_p())
    assert np.array_equal(dp, o.get_d_p())
    # the checkpoint the processes wrote together holds the same global fields
    st = read_state(tmp_path / "state.bin")
    assert np.array_equal(st.current["u"].astype(np.float64), u)
    assert np.array_equal(st.current["p"].astype(np.float64), p)
    assert st.amg_val is not None
