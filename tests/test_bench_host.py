"""Host-side logic of bench.py's multi-GPU line (no GPU): the per-iteration
communication table built from every rank's cfd_comm_timing entries."""
import bench


def _entry(cat, level, calls, wait_us, comm_us, nbytes=100):
    return {"category": cat, "level": level, "calls": calls, "bytes": nbytes, "wait_us": wait_us, "comm_us": comm_us}


def test_comm_timing_summary_per_iteration_and_efficiency():
    its = 10
    ranks = [
        [_entry("krylov_halo", -1, 30, 300.0, 900.0), _entry("amg_halo", 0, 40, 100.0, 400.0),
         _entry("reduction_allgather", -1, 21, 210.0, 210.0)],
        [_entry("krylov_halo", -1, 30, 500.0, 950.0), _entry("amg_halo", 0, 40, 0.0, 380.0),
         _entry("reduction_allgather", -1, 21, 50.0, 50.0), _entry("amg_halo", 3, 40, 400.0, 400.0)],
    ]
    t = {"iterations": its, "step_ms_with_timing": 20.0, "ranks": ranks}
    s = bench.comm_timing_summary(t)
    p = s["per_iteration"]
    assert set(p) == {"krylov_halo", "amg_halo_l0", "amg_halo_l3", "reduction_allgather"}
    assert p["krylov_halo"]["calls"] == 3.0
    assert p["krylov_halo"]["wait_us_max"] == 50.0 and p["krylov_halo"]["wait_us_mean"] == 40.0
    assert p["amg_halo_l0"]["comm_us_max"] == 40.0 and p["amg_halo_l0"]["comm_us_mean"] == 39.0
    assert p["amg_halo_l3"]["wait_us_mean"] == 40.0  # only one rank reported it
    # exposed = max over ranks of the summed waits per iteration: rank 0 61, rank 1 95
    assert abs(s["exposed_us_per_iteration"] - 95.0) < 1e-9
    assert abs(s["iteration_us"] - 2000.0) < 1e-9
    assert abs(s["predicted_efficiency"] - (1.0 - 95.0 / 2000.0)) < 1e-12


def test_comm_timing_summary_empty_ranks():
    s = bench.comm_timing_summary({"iterations": 5, "step_ms_with_timing": 1.0, "ranks": [[], []]})
    assert s["per_iteration"] == {} and s["exposed_us_per_iteration"] == 0.0


def test_check_world_matches_launcher():
    assert bench.check_world(1, {}) == (1, None)
    assert bench.check_world(4, {"WORLD_SIZE": "4"}) == (4, None)
    w, err = bench.check_world(8, {"WORLD_SIZE": "2"})
    assert w == 2 and "WORLD_SIZE=2" in err
    w, err = bench.check_world(1, {"WORLD_SIZE": "2"})
    assert err is not None
    assert bench.check_world(0, {})[1] is not None


def test_rank_launch_cmd_is_the_driver_launch_line():
    cmd = bench.rank_launch_cmd(4, ["--gpus", "4", "--steps", "3"], 29511)
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index("--master-port") + 1] == "29511"
    assert cmd[-4:] == ["--gpus", "4", "--steps", "3"] and cmd[-5].endswith("bench.py")


def test_bench_refuses_gpus_world_mismatch_before_gpu():
    """Under a launcher that started 2 ranks, --gpus 3 exits 2 at once (before
    any import of torch or the library)."""
    import os
    import subprocess
    import sys
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, bench.__file__, "--gpus", "3"], env=env, capture_output=True, text=True,
                       timeout=60)
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr and r.stdout == ""
