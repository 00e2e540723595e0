"""bench.py keeps the driver's contract: one JSON line with the metric, the
roofline and (N = 1) the CPU baseline objects (C1 workload, 1 timed step)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_json_contract():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--config", "c1", "--steps", "1",
                        "--warmup", "1", "--outer", "2", "--inner", "6"],
                       capture_output=True, text=True, timeout=110, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 1 and d["warmup"] == 1
    assert d["unit"] == "cell-updates/sec" and d["value"] > 0 and d["higher_is_better"] is True
    assert d["dtype"] == "f32" and d["scaling"] == "weak" and d["vs_baseline"] is None
    assert "workload" in d["config"]
    rf = d["roofline"]
    assert rf["bound"] == "hbm" and rf["unit"] == "GB/s" and rf["peak"] == 8000.0
    assert 0 < rf["achieved"] < rf["peak"] * 1.2 and abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-9
    assert rf["traffic"] is None  # PMC traffic is committed for the C2 workload only
    cb = d["cpu_baseline"]
    assert cb["value"] > 0 and cb["kind"] == "port" and cb["cores"] >= 1 and cb["sample"]
    g = cb["gbs"]  # the CPU GB/s from the same algorithmic byte counts
    assert g["reference_format_gbs"] > 0 and g["layout_true_gbs"] > 0
    assert abs(g["reference_format_gbs"] - d["step_reference_format_bytes_count"] / g["seconds_per_step"] / 1e9) \
        <= 1e-9 * g["reference_format_gbs"]


def test_bench_two_process_launch_contract():
    """The N > 1 launch: ``python bench.py --gpus 2`` WITHOUT a launcher starts
    torch.distributed.run itself (a child process, one process per rank,
    RANK/WORLD_SIZE from the env, 127.0.0.1 rendezvous) -- the driver's own
    launch line, bench.rank_launch_cmd; rank 0 alone prints one JSON line
    whose value is the whole job's rate.  The one-GPU box has no second device
    for RCCL, so both ranks share GPU 0 over the host-staged transport (DESIGN
    §7); the line then says so in `parallelism`."""
    env = dict(os.environ, CFD_DIST_TRANSPORT="host", CFD_BENCH_DEVICE="0")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--config", "c1", "--steps", "1", "--warmup", "1", "--outer", "1", "--inner", "4"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=110, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "without a launcher: starting 2 ranks" in r.stderr
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 1 and d["scaling"] == "weak"
    assert "cpu_baseline" not in d or d["cpu_baseline"] is None  # rank 0 at N = 1 only
    cells = d["config"]["cells_total"]
    assert d["config"]["cells_per_gpu"] * 2 >= cells * 0.99
    # value = every rank's cells x steps / the max-over-ranks time
    assert abs(d["value"] - cells * d["steps"] / (d["ms_per_step"] * d["steps"] / 1e3)) <= 1e-6 * d["value"]
    assert "host-staged" in d["config"]["parallelism"]
