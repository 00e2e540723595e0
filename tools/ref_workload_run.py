"""Run one of the reference's criterion workloads (bench.reference_workloads)
on its own, for profiling: python tools/ref_workload_run.py [solver_step|fine_mesh]."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "cfd-demo2_amd"))
import bench  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "solver_step"
which = None if which == "all" else which
t0 = time.perf_counter()
out = bench.reference_workloads(only=which)
print(json.dumps(out))
print(f"total {time.perf_counter() - t0:.1f}s", file=sys.stderr)
