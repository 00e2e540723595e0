"""cfd2_amd — MI355X-native coupled incompressible-flow step (drop-in for
``cfd2::solver::gpu::GpuSolver`` of TSultanov/cfd-demo2).

Python mirror of the reference API over the C ABI in include/cfd2_amd.h.
"""
from . import mesh  # noqa: F401
from .mesh import (BackwardsStep, ChannelWithObstacle, CircleObstacle, Mesh,  # noqa: F401
                   RectangularChannel, generate_cut_cell_mesh)
from .solver import GpuGroup, GpuSolver, dist_plan, dist_unique_id  # noqa: F401,E402
from ._ffi import Config, Constants, build_id, default_config  # noqa: F401,E402
