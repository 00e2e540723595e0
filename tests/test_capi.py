"""The C ABI library: loads on a CPU-only host, exports every symbol declared in
include/*.h, reports errors as status codes (no compute calls without a GPU)."""
import ctypes as C
import glob
import os
import re

import pytest

from cfd2_amd import _ffi
from cfd2_amd.solver import _bind

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    syms = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        txt = open(h).read()
        txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
        for m in re.finditer(r"\b(cfd_[a-z0-9_]+)\s*\(", txt):
            syms.add(m.group(1))
    return syms


def test_library_exports_every_declared_symbol():
    L = _bind()
    syms = declared_symbols()
    assert len(syms) > 40
    missing = [s for s in sorted(syms) if not hasattr(L, s)]
    assert not missing, missing
    assert set(_ffi.EXPORTED) <= syms


def test_config_defaults_match_reference():
    L = _bind()
    c = _ffi.Config()
    L.cfd_config_default(C.byref(c))
    assert c.n_outer_correctors == 20 and c.max_restart == 50 and c.max_outer_restarts == 20
    assert abs(c.fgmres_rtol - 1e-5) < 1e-12 and abs(c.fgmres_atol - 1e-7) < 1e-14
    assert c.convergence_lag == 1


def test_null_handles_return_status():
    L = _bind()
    assert L.cfd_step(None) == 1
    assert L.cfd_set_dt(None, C.c_float(1.0)) == 1
    assert b"null" in L.cfd_last_error()


def test_bad_geometry_rejected():
    L = _bind()
    g = _ffi.Geometry(kind=9)
    h = C.c_void_p()
    assert L.cfd_mesh_generate_cut_cell(C.byref(g), 0.1, 0.1, 1.2, 1.0, 1.0, C.byref(h)) == 1


def test_solver_without_gpu_fails_loudly(gpu_available):
    if gpu_available:
        pytest.skip("GPU present")
    from cfd2_amd import GpuSolver
    from tests.meshes import backwards_step
    with pytest.raises(RuntimeError, match="status 2"):
        GpuSolver(backwards_step())
