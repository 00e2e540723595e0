"""ctypes wrapper of the CPU oracle (oracle/liboracle_cfd.so).

TEST INFRASTRUCTURE ONLY: used by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py.  Mirrors the GpuSolver API so parity tests can
drive both with the same script.  Pinned to the reference's own WGSL kernels
(tests/test_wgsl_pin.py; see oracle/oracle.h).
"""
from __future__ import annotations

import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cfd-demo2_amd"))
from cfd2_amd import _ffi  # noqa: E402

ORACLE_LIB = os.path.join(ROOT, "oracle", "liboracle_cfd.so")
_olib = None


def olib():
    global _olib
    if _olib is None:
        if not os.path.exists(ORACLE_LIB):
            raise RuntimeError("oracle not built (run __graft_entry__.build())")
        L = C.CDLL(ORACLE_LIB)
        vp = C.c_void_p
        L.oracle_create.restype = vp
        L.oracle_create.argtypes = [C.POINTER(_ffi.MeshView), C.POINTER(_ffi.Config)]
        L.oracle_create_dist.restype = vp
        L.oracle_create_dist.argtypes = [C.POINTER(_ffi.MeshView), C.POINTER(_ffi.Config), C.c_int]
        L.oracle_destroy.argtypes = [vp]
        L.oracle_destroy.restype = None
        L.oracle_set_threads.argtypes = [C.c_int]
        L.oracle_set_threads.restype = None
        for name in ("oracle_set_u", "oracle_set_p", "oracle_get_u", "oracle_get_p", "oracle_get_d_p"):
            getattr(L, name).argtypes = [vp, C.POINTER(C.c_double)]
        L.oracle_get_constants.argtypes = [vp, C.POINTER(_ffi.Constants)]
        L.oracle_set_constants.argtypes = [vp, C.POINTER(_ffi.Constants)]
        L.oracle_set_dt.argtypes = [vp, C.c_float]
        L.oracle_initialize_history.argtypes = [vp]
        L.oracle_step.argtypes = [vp]
        L.oracle_get_step_info.argtypes = [vp, C.POINTER(_ffi.StepInfo)]
        L.oracle_set_stop_state.argtypes = [vp, C.c_int, C.c_uint32, C.c_uint32]
        L.oracle_set_n_outer_correctors.argtypes = [vp, C.c_int]
        L.oracle_debug_buffer_len.argtypes = [vp, C.c_int]
        L.oracle_debug_buffer_len.restype = C.c_size_t
        L.oracle_debug_buffer.argtypes = [vp, C.c_int, C.POINTER(C.c_float), C.c_size_t]
        L.oracle_debug_prepare_assemble.argtypes = [vp, C.c_int]
        L.oracle_amg_levels.argtypes = [vp, C.POINTER(C.c_int), C.POINTER(C.c_uint32),
                                        C.POINTER(C.c_uint64)]
        L.oracle_last_error.restype = C.c_char_p
        L.oracle_set_semantics.argtypes = [vp, C.c_int]
        _olib = L
    return _olib


def set_threads(n: int) -> None:
    olib().oracle_set_threads(int(n))


def _ck(st, what):
    if st != 0:
        raise RuntimeError(f"{what}: {olib().oracle_last_error().decode()}")


class OracleSolver:
    """Same surface as cfd2_amd.GpuSolver, backed by the CPU oracle."""

    def __init__(self, mesh, config=None, nranks=1, **cfg_overrides):
        """nranks: accepted for the distributed tests; results do not depend on it
        (the distributed solver reproduces the single-GPU bits)."""
        self._mesh = mesh  # keep the mesh alive (view borrows its arrays)
        cfg = config if config is not None else _ffi.default_config(**cfg_overrides)
        self._cfg = cfg
        view = mesh.view()
        h = olib().oracle_create_dist(C.byref(view), C.byref(cfg), int(nranks))
        if not h:
            raise RuntimeError("oracle_create failed: " + olib().oracle_last_error().decode())
        self._h = C.c_void_p(h)
        self.num_cells = int(view.num_cells)
        self.num_faces = int(view.num_faces)

    # reference-semantics sensitivity flags (oracle/oracle.h oracle_set_semantics)
    SEM_INPLACE_SMOOTHER, SEM_RACY_PREPARE, SEM_REF_REDUCTIONS, SEM_RESTRICT_CLAMP = 1, 2, 4, 8

    def set_semantics(self, flags: int) -> None:
        olib().oracle_set_semantics(self._h, int(flags))

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            olib().oracle_destroy(h)
            self._h = None

    # --- constants -------------------------------------------------------
    @property
    def constants(self) -> _ffi.Constants:
        c = _ffi.Constants()
        olib().oracle_get_constants(self._h, C.byref(c))
        return c

    @constants.setter
    def constants(self, c) -> None:
        olib().oracle_set_constants(self._h, C.byref(c))

    def _set(self, **kv):
        c = self.constants
        for k, v in kv.items():
            setattr(c, k, v)
        self.constants = c

    def set_dt(self, dt):
        olib().oracle_set_dt(self._h, float(dt))

    def set_viscosity(self, v): self._set(viscosity=v)
    def set_alpha_p(self, v): self._set(alpha_p=v)
    def set_alpha_u(self, v): self._set(alpha_u=v)
    def set_density(self, v): self._set(density=v)
    def set_scheme(self, v): self._set(scheme=int(v))
    def set_time_scheme(self, v): self._set(time_scheme=int(v))
    def set_inlet_velocity(self, v): self._set(inlet_velocity=v)
    def set_ramp_time(self, v): self._set(ramp_time=v)
    def set_precond_type(self, v): self._set(precond_type=int(v))
    def update_constants(self): pass

    # --- state -----------------------------------------------------------
    def set_u(self, u):
        a = np.ascontiguousarray(np.asarray(u, dtype=np.float64).reshape(-1))
        assert a.size == 2 * self.num_cells
        _ck(olib().oracle_set_u(self._h, a.ctypes.data_as(C.POINTER(C.c_double))), "set_u")

    def set_p(self, p):
        a = np.ascontiguousarray(np.asarray(p, dtype=np.float64).reshape(-1))
        assert a.size == self.num_cells
        _ck(olib().oracle_set_p(self._h, a.ctypes.data_as(C.POINTER(C.c_double))), "set_p")

    def initialize_history(self):
        olib().oracle_initialize_history(self._h)

    def step(self):
        _ck(olib().oracle_step(self._h), "step")

    def get_u(self):
        a = np.zeros(2 * self.num_cells)
        olib().oracle_get_u(self._h, a.ctypes.data_as(C.POINTER(C.c_double)))
        return a.reshape(-1, 2)

    def get_p(self):
        a = np.zeros(self.num_cells)
        olib().oracle_get_p(self._h, a.ctypes.data_as(C.POINTER(C.c_double)))
        return a

    def get_d_p(self):
        a = np.zeros(self.num_cells)
        olib().oracle_get_d_p(self._h, a.ctypes.data_as(C.POINTER(C.c_double)))
        return a

    def step_info(self) -> _ffi.StepInfo:
        i = _ffi.StepInfo()
        olib().oracle_get_step_info(self._h, C.byref(i))
        return i

    def set_stop_state(self, should_stop, degenerate_count, steady_state_count):
        _ck(olib().oracle_set_stop_state(self._h, int(bool(should_stop)), int(degenerate_count),
                                         int(steady_state_count)), "set_stop_state")

    def _set_stop_field(self, **kw):
        i = self.step_info()
        cur = dict(should_stop=i.should_stop, degenerate_count=i.degenerate_count,
                   steady_state_count=i.steady_state_count)
        cur.update(kw)
        self.set_stop_state(**cur)

    @property
    def n_outer_correctors(self): return int(self._cfg.n_outer_correctors)
    @n_outer_correctors.setter
    def n_outer_correctors(self, v):
        self._cfg.n_outer_correctors = int(v)
        olib().oracle_set_n_outer_correctors(self._h, int(v))

    @property
    def should_stop(self): return bool(self.step_info().should_stop)
    @should_stop.setter
    def should_stop(self, v): self._set_stop_field(should_stop=bool(v))
    @property
    def degenerate_count(self): return int(self.step_info().degenerate_count)
    @degenerate_count.setter
    def degenerate_count(self, v): self._set_stop_field(degenerate_count=int(v))
    @property
    def steady_state_count(self): return int(self.step_info().steady_state_count)
    @steady_state_count.setter
    def steady_state_count(self, v): self._set_stop_field(steady_state_count=int(v))

    def debug_buffer(self, bid: int) -> np.ndarray:
        n = olib().oracle_debug_buffer_len(self._h, bid)
        a = np.zeros(n, dtype=np.float32)
        _ck(olib().oracle_debug_buffer(self._h, bid, a.ctypes.data_as(C.POINTER(C.c_float)), n),
            "debug_buffer")
        return a

    def debug_prepare_assemble(self, assemble=True):
        olib().oracle_debug_prepare_assemble(self._h, 1 if assemble else 0)

    def amg_levels(self):
        nl = C.c_int()
        rows = (C.c_uint32 * 20)()
        nnz = (C.c_uint64 * 20)()
        olib().oracle_amg_levels(self._h, C.byref(nl), rows, nnz)
        return [(int(rows[i]), int(nnz[i])) for i in range(nl.value)]
