"""Build kernel variants (compile-time tunables of kernels.hip) as separate
libraries for same-box A/B timing:  python tools/ab_variants.py NAME=DEF,DEF ...
e.g.  u1=CFD_SPMV_U=1  u2=CFD_SPMV_U=2,CFD_PREDICT_U=2
Libraries land in cfd-demo2_amd/cfd2_amd/_lib/variants/; select one at run
time with CFD2_AMD_LIB=<path> (tools/gpu_ab_prof.sh: copy the variants into _lib/ab/ for the run)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as g  # noqa: E402

for spec in sys.argv[1:]:
    name, _, defs = spec.partition("=")
    defines = [d for d in defs.split(",") if d]
    lib = os.path.join(g.LIB_DIR, "variants", f"libcfd2_amd_{name}.so")
    g.build_product(lib=lib, hip_defines=defines, obj_dir=os.path.join(g.OBJ_DIR, "v_" + name))
    print(name, lib)
