"""Test meshes: the ones the reference's own solver tests build."""
import functools

from cfd2_amd.mesh import (BackwardsStep, ChannelWithObstacle, bench_channel,
                           generate_cut_cell_mesh)

STEP = BackwardsStep(length=3.5, height_inlet=0.5, height_outlet=1.0, step_x=0.5)


@functools.lru_cache(maxsize=None)
def backwards_step(h=0.05, smooth_iters=50):
    """tests/coupled_schemes_test.rs:14-26 and tests/amg_test.rs:8-19 (h=0.05, smooth 0.3/50)."""
    m = generate_cut_cell_mesh(STEP, h, h, 1.2, (3.5, 1.0))
    m.smooth(STEP, 0.3, smooth_iters)
    return m


@functools.lru_cache(maxsize=None)
def channel_obstacle(h=0.05, smooth_iters=50, r=0.2, center=(1.0, 0.5)):
    """tests/gpu_divergence_test.rs:8-22 (ChannelWithObstacle 3x1, r=0.2, h=0.05)."""
    geo = ChannelWithObstacle(length=3.0, height=1.0, obstacle_center=center, obstacle_radius=r)
    m = generate_cut_cell_mesh(geo, h, h, 1.2, (3.0, 1.0))
    m.smooth(geo, 0.3, smooth_iters)
    return m


@functools.lru_cache(maxsize=None)
def bench_mesh(h, smooth_iters=100):
    """SURVEY §8(d) benchmark geometry (obstacle (1.0, 0.51), r 0.1)."""
    return bench_channel(h, smooth_iters)
