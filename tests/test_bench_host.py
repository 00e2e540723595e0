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
