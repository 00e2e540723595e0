"""profiles/<round>/wgsl_pin_summary.txt from the reference-kernel fixtures
(tests/golden/wgsl_ref*.npz, tests/golden/make_wgsl_golden.py): the cases,
their schedules, and the reference's own spread between schedules (host only).
Usage: python tools/wgsl_pin_summary.py > profiles/r06/wgsl_pin_summary.txt"""
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
G = os.path.join(ROOT, "tests", "golden")


def rel(z, n, m1, m2):
    if f"{n}/{m1}/u" not in z.files or f"{n}/{m2}/u" not in z.files:
        return "-"
    r = [np.linalg.norm(z[f"{n}/{m1}/{f}"].astype(float) - z[f"{n}/{m2}/{f}"].astype(float))
         / np.linalg.norm(z[f"{n}/{m2}/{f}"].astype(float)) for f in "up"]
    return f"{r[0]:.1e} / {r[1]:.1e}"


def main():
    print("# The oracle and the HIP path against the reference's OWN WGSL kernels")
    print("# Fixtures tests/golden/wgsl_ref.npz (+ wgsl_ref_c1.npz), made by tests/golden/make_wgsl_golden.py")
    print("# in the build container: the reference's eight hot-path shaders executed on the CPU from its")
    print("# source (oracle/wgsl/wgsl_exec.py) under the Rust host sequence restated in tests/wgsl_ref.py.")
    print("#   A: workgroups in dispatch order, lanes in lockstep, wgpu Restrict policy -> oracle flags 15,")
    print("#      HIP cfd_debug_reference_semantics(15)")
    print("#   B: whole dispatch resident and in lockstep, naga ReadZeroSkipWrite      -> oracle flags 4,")
    print("#      HIP flags 4")
    print("#   C: B, but the V-cycle's dispatches as in A (in-place smoother, clamped  -> oracle flags 13,")
    print("#      restrict rows)                                                          HIP flags 13")
    print("# Checked bit-exact (per-step SHA-256 of the f32 fields + step statistics) by")
    print("# tests/test_wgsl_pin.py (CPU, oracle) and tests/test_gpu_wgsl_pin.py (GPU, HIP; gpu_wgsl_pin.log).")
    print()
    z = np.load(os.path.join(G, "wgsl_ref.npz"))
    names = []
    for k in z.files:
        n = k.split("/")[0]
        if not n.startswith("kernels") and n not in names:
            names.append(n)
    print(f"{'case':18s} {'modes':5s} {'steps':5s} {'FGMRES its (B)':14s} {'A vs B rel-L2 u / p':22s} "
          f"{'C vs B rel-L2 u / p':22s}")
    for n in names:
        modes = "".join(m for m in "ABC" if f"{n}/{m}/info" in z.files)
        steps = len(z[f"{n}/B/digests"])
        its = int(z[f"{n}/B/info"][:, 0].sum())
        print(f"{n:18s} {modes:5s} {steps:<5d} {its:<14d} {rel(z, n, 'A', 'B'):22s} {rel(z, n, 'C', 'B'):22s}")
    c1 = np.load(os.path.join(G, "wgsl_ref_c1.npz"))
    print(f"{'c1 (1,001,744)':18s} {'B':5s} {len(c1['c1/B/digests']):<5d} {int(c1['c1/B/info'][:, 0].sum()):<14d} "
          f"{'-':22s} {'-':22s}")
    print("(fields are stored for meshes <= 2000 cells; larger cases are checked through the digests)")
    print()
    print("kernel cases (prepare_coupled + coupled_assembly_merged on a random state, schedule B,")
    print("every output buffer; == canonical oracle (flags 0) and == HIP k_prepare / k_assemble):")
    print(" ", ", ".join(sorted({k.split("/")[0] for k in z.files if k.startswith("kernels")})))
    print()
    print("generation times (build container, 8 CPUs):")
    with open(os.path.join(G, "wgsl_ref_generation.log")) as f:
        print(f.read().rstrip())


if __name__ == "__main__":
    main()
