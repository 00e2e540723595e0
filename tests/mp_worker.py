"""Worker of tests/test_gpu_multiproc.py: one rank (one process) of the
distributed solver over the host-staged gloo transport, all ranks on GPU 0.
Launched by torch.distributed.run; writes its owned fields to <out>/rank<r>.npz."""
import os
import sys

import numpy as np
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "cfd-demo2_amd"))

from cfd2_amd import GpuSolver, default_config  # noqa: E402
from tests.meshes import backwards_step  # noqa: E402
from tests.test_gpu_parity import _setup_amg_test  # noqa: E402


def main():
    out = sys.argv[1]
    steps = int(sys.argv[2])
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    mesh = backwards_step()
    local = int(os.environ.get("CFD_TEST_AMG_LOCAL", "0"))  # partition-aware AMG aggregation
    timeout = float(os.environ.get("CFD_TEST_COMM_TIMEOUT", "180"))  # tests/test_watchdog.py
    s = GpuSolver.create_dist_host(mesh, world, rank, device=0,
                                   config=default_config(amg_local_aggregation=local, comm_timeout_s=timeout))
    _setup_amg_test(s, mesh, 1)
    if rank == int(os.environ.get("CFD_TEST_STALL_RANK", "-1")):
        import time
        time.sleep(60)  # a stalled peer: the other ranks' watchdogs must end the job
        sys.exit(3)
    for _ in range(steps):
        s.step()
    if len(sys.argv) > 3:  # collective checkpoint: every process writes its rows
        s.save_state(sys.argv[3])
    c0, c1 = s.owned
    info = s.step_info()
    np.savez(os.path.join(out, f"rank{rank}.npz"), c0=c0, c1=c1, u=s.get_u(), p=s.get_p(), d_p=s.get_d_p(),
             outer_iterations=info.outer_iterations, linear=info.total_linear_iterations,
             res_u=info.outer_residual_u, res_p=info.outer_residual_p)
    s.close()
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
