"""Progress watchdog of the distributed transports (cfd_config.comm_timeout_s,
csrc/host/comm.hpp): an operation that does not complete within the limit
ends the process with status 70 and a report naming the rank, the operation
and its category, instead of hanging the job without a diagnostic.

CPU: cfd_debug_comm_watchdog (the watchdog around a host-blocking wait, run in
a child process since it exits it).  GPU: two processes on the host-staged
transport where rank 1 stops participating: rank 0's watchdog fires inside
its exchange callback."""
import os
import socket
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_CHILD = """
import sys, ctypes as C
sys.path.insert(0, {pkg!r})
from cfd2_amd import _ffi
L = _ffi.lib()
L.cfd_debug_comm_watchdog.argtypes = [C.c_float, C.c_int32]
print("status", L.cfd_debug_comm_watchdog({t}, {hang}), flush=True)
"""


def _run(t, hang):
    code = _CHILD.format(pkg=os.path.join(ROOT, "cfd-demo2_amd"), t=t, hang=hang)
    return subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)


def test_watchdog_fires_on_stalled_operation():
    t0 = time.time()
    r = _run(0.5, 20000)
    assert r.returncode == 70, (r.returncode, r.stdout, r.stderr)
    assert time.time() - t0 < 15  # fired near the limit, not after the 20 s stall
    assert "cfd2 comm watchdog: rank 0" in r.stderr and "timed out" in r.stderr
    assert "cfd_debug_comm_watchdog host wait" in r.stderr and "status" not in r.stdout


def test_watchdog_quiet_within_limit_and_when_off():
    r = _run(5.0, 100)
    assert r.returncode == 0 and "status 0" in r.stdout and r.stderr == ""
    r = _run(0.0, 800)  # <= 0: disabled
    assert r.returncode == 0 and "status 0" in r.stdout


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.gpu
def test_watchdog_host_transport_stalled_peer(tmp_path):
    """Rank 1 creates its solver, then stops (sleeps past the limit) while
    rank 0 steps: rank 0 blocks in the gloo exchange callback and its watchdog
    (3 s) ends it with status 70; the launcher then tears rank 1 down."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", CFD_TEST_STALL_RANK="1", CFD_TEST_COMM_TIMEOUT="3")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(ROOT, "tests", "mp_worker.py"), str(tmp_path), "2"]
    t0 = time.time()
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=110)
    out = r.stdout + r.stderr
    assert r.returncode != 0, out[-3000:]
    assert "cfd2 comm watchdog: rank 0" in out, out[-3000:]
    assert "host-staged" in out and "exiting with status 70" in out
    assert time.time() - t0 < 100
