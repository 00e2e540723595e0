"""Reference-semantics sensitivity: how far each canonical
resolution of the reference's non-determinism moves the fields.
Runs the oracle under the canonical semantics and under each flag of
oracle_set_semantics (and all together) on the reference's own solver tests
and the C0 channel at natural convergence; prints relative L2 deltas of u and
p after the last step, plus FGMRES iteration totals.  Usage:
python tools/sensitivity.py [--json out.json]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cfd-demo2_amd"))
sys.path.insert(0, ROOT)

from cfd2_amd import default_config  # noqa: E402
from tests.meshes import backwards_step, bench_mesh  # noqa: E402
from tests.oracle_py import OracleSolver  # noqa: E402
from tests.test_oracle import setup_amg_test, setup_schemes_test  # noqa: E402

FLAGS = [("in-place AMG smoother", 1), ("racy prepare reads", 2), ("reference reduction order", 4),
         ("restrict_residual clamp", 8), ("all four", 15)]


def c0_setup(s, mesh):
    s.set_dt(1e-3)
    s.set_viscosity(0.01)
    s.set_density(1.0)
    s.set_alpha_u(0.7)
    s.set_alpha_p(0.3)
    s.set_precond_type(1)
    s.initialize_history()
    c = s.constants
    c.time = 0.05
    s.constants = c


CASES = [
    ("amg_test AMG (5 steps)", backwards_step, lambda s, m: setup_amg_test(s, m, 1), 5),
    ("amg_test Jacobi (5 steps)", backwards_step, lambda s, m: setup_amg_test(s, m, 0), 5),
    ("coupled_schemes SOU (2 steps)", backwards_step, lambda s, m: setup_schemes_test(s, m, 1, 0), 2),
    ("coupled_schemes QUICK (2 steps)", backwards_step, lambda s, m: setup_schemes_test(s, m, 2, 0), 2),
    ("coupled_schemes BDF2 (2 steps)", backwards_step, lambda s, m: setup_schemes_test(s, m, 0, 1), 2),
    ("C0 channel AMG (3 steps)", lambda: bench_mesh(0.0172, 100), c0_setup, 3),
]


def run(mesh, setup, steps, flags):
    s = OracleSolver(mesh, config=default_config())
    s.set_semantics(flags)
    setup(s, mesh)
    its = 0
    for _ in range(steps):
        s.step()
        its += s.step_info().total_linear_iterations
    return s.get_u(), s.get_p(), its


def rel(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def main():
    rows = []
    for name, mk, setup, steps in CASES:
        mesh = mk()
        u0, p0, it0 = run(mesh, setup, steps, 0)
        for fname, fl in FLAGS:
            u, p, it = run(mesh, setup, steps, fl)
            du, dp = rel(u, u0), rel(p, p0)
            row = dict(case=name, switch=fname, du=du, dp=dp, iters=it, iters_canonical=it0)
            if fl & 3:  # the same reference semantics under a second schedule: its own spread
                ur, pr, _ = run(mesh, setup, steps, fl | 16)
                row.update(du_sched=rel(ur, u), dp_sched=rel(pr, p))
            rows.append(row)
            extra = (f"   | reference vs itself (reversed workgroups) u {row['du_sched']:9.2e} p {row['dp_sched']:9.2e}"
                     if "du_sched" in row else "")
            print(f"{name:34s} {fname:28s} u {du:9.2e}  p {dp:9.2e}  FGMRES its {it} (canonical {it0}){extra}",
                  flush=True)
    if len(sys.argv) > 2 and sys.argv[1] == "--json":
        with open(sys.argv[2], "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
