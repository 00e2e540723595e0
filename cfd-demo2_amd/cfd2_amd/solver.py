"""``GpuSolver`` — Python mirror of the reference's ``cfd2::solver::gpu::GpuSolver``
(src/solver/gpu/structs.rs, solver.rs) over the C ABI.  Every method is one
C call into libcfd2_amd.so; the HIP kernels run on the library's own stream.
There is no CPU fallback: constructing a solver without a GPU raises.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import _ffi

_vp = C.c_void_p
_bound = False


# cfd_exchange_fn / cfd_allgather_fn (include/cfd2_amd.h)
EXCHANGE_FN = C.CFUNCTYPE(C.c_int32, C.c_void_p, C.c_int32, C.POINTER(C.c_int32), C.POINTER(C.c_void_p),
                          C.POINTER(C.c_uint64), C.POINTER(C.c_void_p), C.POINTER(C.c_uint64))
ALLGATHER_FN = C.CFUNCTYPE(C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64)


def _bind():
    global _bound
    if _bound:
        return _ffi.lib()
    L = _ffi.lib()
    dp = C.POINTER(C.c_double)
    L.cfd_config_default.argtypes = [C.POINTER(_ffi.Config)]
    L.cfd_config_default.restype = None
    L.cfd_solver_create.argtypes = [C.POINTER(_ffi.MeshView), C.POINTER(_ffi.Config), C.c_int32,
                                    C.POINTER(_vp)]
    L.cfd_solver_destroy.argtypes = [_vp]
    L.cfd_solver_destroy.restype = None
    for n in ("cfd_set_u", "cfd_set_p", "cfd_get_u", "cfd_get_p", "cfd_get_d_p"):
        getattr(L, n).argtypes = [_vp, dp]
    L.cfd_get_constants.argtypes = [_vp, C.POINTER(_ffi.Constants)]
    L.cfd_set_constants.argtypes = [_vp, C.POINTER(_ffi.Constants)]
    for n in ("cfd_set_dt", "cfd_set_viscosity", "cfd_set_alpha_p", "cfd_set_alpha_u",
              "cfd_set_density", "cfd_set_inlet_velocity", "cfd_set_ramp_time"):
        getattr(L, n).argtypes = [_vp, C.c_float]
    for n in ("cfd_set_scheme", "cfd_set_time_scheme", "cfd_set_precond_type"):
        getattr(L, n).argtypes = [_vp, C.c_uint32]
    for n in ("cfd_update_constants", "cfd_initialize_history", "cfd_step", "cfd_synchronize"):
        getattr(L, n).argtypes = [_vp]
    L.cfd_get_step_info.argtypes = [_vp, C.POINTER(_ffi.StepInfo)]
    L.cfd_set_stop_state.argtypes = [_vp, C.c_int32, C.c_uint32, C.c_uint32]
    L.cfd_set_n_outer_correctors.argtypes = [_vp, C.c_int32]
    L.cfd_num_cells.argtypes = [_vp]
    L.cfd_num_cells.restype = C.c_uint32
    L.cfd_num_faces.argtypes = [_vp]
    L.cfd_num_faces.restype = C.c_uint32
    L.cfd_profile_enable.argtypes = [_vp, C.c_int32]
    L.cfd_profile_reset.argtypes = [_vp]
    L.cfd_profile_smoother.argtypes = [_vp, dp, C.POINTER(C.c_uint64), dp]
    L.cfd_graph_enable.argtypes = [_vp, C.c_int32]
    L.cfd_graph_stats.argtypes = [_vp, C.POINTER(C.c_int32), C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
    L.cfd_amg_levels.argtypes = [_vp, C.POINTER(C.c_int32), C.POINTER(C.c_uint32),
                                 C.POINTER(C.c_uint64)]
    L.cfd_step_algorithmic_bytes.argtypes = [_vp]
    L.cfd_step_algorithmic_bytes.restype = C.c_double
    L.cfd_smoother_layout_bytes.argtypes = [_vp]
    L.cfd_smoother_layout_bytes.restype = C.c_double
    L.cfd_step_layout_bytes.argtypes = [_vp]
    L.cfd_step_layout_bytes.restype = C.c_double
    L.cfd_debug_buffer_len.argtypes = [_vp, C.c_int32]
    L.cfd_debug_buffer_len.restype = C.c_size_t
    L.cfd_debug_buffer.argtypes = [_vp, C.c_int32, C.POINTER(C.c_float), C.c_size_t]
    L.cfd_debug_prepare_assemble.argtypes = [_vp, C.c_int32]
    L.cfd_debug_reference_semantics.argtypes = [_vp, C.c_int32]
    L.cfd_debug_amg_info.argtypes = [_vp, C.c_int32, C.POINTER(C.c_int32), C.POINTER(C.c_uint64)]
    u8p = C.POINTER(C.c_uint8)
    u32p = C.POINTER(C.c_uint32)
    L.cfd_dist_unique_id.argtypes = [u8p]
    L.cfd_solver_create_dist.argtypes = [C.POINTER(_ffi.MeshView), C.POINTER(_ffi.Config), C.c_int32,
                                         C.c_int32, C.c_int32, u8p, C.POINTER(_vp)]
    L.cfd_solver_create_dist_host.argtypes = [C.POINTER(_ffi.MeshView), C.POINTER(_ffi.Config), C.c_int32,
                                              C.c_int32, C.c_int32, EXCHANGE_FN, ALLGATHER_FN, _vp,
                                              C.POINTER(_vp)]
    L.cfd_group_create.argtypes = [C.POINTER(_ffi.MeshView), C.POINTER(_ffi.Config), C.c_int32,
                                   C.POINTER(C.c_int32), C.POINTER(_vp)]
    L.cfd_group_step.argtypes = [C.POINTER(_vp), C.c_int32]
    L.cfd_dist_info.argtypes = [_vp, C.POINTER(C.c_int32), C.POINTER(C.c_int32), u32p, u32p, u32p]
    L.cfd_dist_plan.argtypes = [C.POINTER(_ffi.MeshView), C.c_int32, C.c_int32, u32p, u32p, u32p, u32p,
                                u32p, u32p, C.POINTER(C.c_int32), u32p, u32p, u32p]
    L.cfd_debug_rccl_selftest.argtypes = [C.c_int32]
    L.cfd_state_save.argtypes = [_vp, C.c_char_p]
    L.cfd_state_load.argtypes = [_vp, C.c_char_p]
    L.cfd_group_state_save.argtypes = [C.POINTER(_vp), C.c_int32, C.c_char_p]
    L.cfd_dist_comm_stats.argtypes = [_vp, C.POINTER(_ffi.CommStats), C.c_int32]
    L.cfd_debug_group_fault.argtypes = [C.POINTER(_vp), C.c_int32, C.c_int32]
    L.cfd_debug_group_fault_midstep.argtypes = [C.POINTER(_vp), C.c_int32, C.c_int32]
    L.cfd_group_reset.argtypes = [C.POINTER(_vp), C.c_int32]
    L.cfd_group_needs_restore.argtypes = [C.POINTER(_vp), C.c_int32]
    L.cfd_group_needs_restore.restype = C.c_int32
    L.cfd_comm_timing_enable.argtypes = [_vp, C.c_int32]
    L.cfd_comm_timing.argtypes = [_vp, C.POINTER(_ffi.CommTimingEntry), C.c_int32, C.POINTER(C.c_int32)]
    _bound = True
    return L


class GpuSolver:
    """Drop-in for ``GpuSolver`` (init/mod.rs:15).  ``mesh`` is a cfd2_amd.Mesh."""

    JACOBI = 0
    AMG = 1

    def __init__(self, mesh, config: _ffi.Config | None = None, device: int = 0, _handle=None,
                  **cfg_overrides):
        L = _bind()
        # the library copies what it needs at creation: no reference to the mesh is kept
        cfg = config if config is not None else _ffi.default_config(**cfg_overrides)
        self._cfg = cfg
        self._n_outer = int(cfg.n_outer_correctors)
        if _handle is None:
            view = mesh.view()
            h = _vp()
            _ffi.check(L.cfd_solver_create(C.byref(view), C.byref(cfg), int(device), C.byref(h)),
                       "cfd_solver_create")
        else:
            h = _handle
        self._h = h
        self.num_cells = int(L.cfd_num_cells(h))
        self.num_faces = int(L.cfd_num_faces(h))
        r, n, c0, c1, ng = C.c_int32(), C.c_int32(), C.c_uint32(), C.c_uint32(), C.c_uint32()
        _ffi.check(L.cfd_dist_info(h, C.byref(r), C.byref(n), C.byref(c0), C.byref(c1), C.byref(ng)),
                   "cfd_dist_info")
        self.rank, self.nranks = r.value, n.value
        self.owned = (c0.value, c1.value)  # global cell range this handle owns
        self.num_global_cells = ng.value

    @classmethod
    def create_dist(cls, mesh, nranks: int, rank: int, unique_id: bytes, device: int = 0,
                    config: _ffi.Config | None = None, **cfg_overrides):
        """One rank of the RCCL-distributed solver (one process per GPU).  Collective."""
        L = _bind()
        cfg = config if config is not None else _ffi.default_config(**cfg_overrides)
        view = mesh.view()
        uid = (C.c_uint8 * 128).from_buffer_copy(bytes(unique_id))
        h = _vp()
        _ffi.check(L.cfd_solver_create_dist(C.byref(view), C.byref(cfg), int(device), int(nranks), int(rank),
                                            uid, C.byref(h)), "cfd_solver_create_dist")
        return cls(mesh, config=cfg, _handle=h)

    @classmethod
    def create_dist_host(cls, mesh, nranks: int, rank: int, device: int = 0,
                         config: _ffi.Config | None = None, **cfg_overrides):
        """One rank of the distributed solver over the host-staged transport
        (test / rehearsal mode: torch.distributed's process group -- gloo --
        carries every halo and all-gather; several ranks may share one GPU).
        torch.distributed must be initialised.  Collective."""
        import torch
        import torch.distributed as dist
        L = _bind()
        cfg = config if config is not None else _ffi.default_config(**cfg_overrides)
        view = mesh.view()

        def buf(addr, nbytes):
            return torch.frombuffer((C.c_uint8 * int(nbytes)).from_address(addr), dtype=torch.uint8)

        def exchange(_user, n, peer, send, sbytes, recv, rbytes):
            try:
                reqs, ks, kr = [], {}, {}
                for i in range(n):
                    q = int(peer[i])
                    if sbytes[i]:
                        reqs.append(dist.isend(buf(send[i], sbytes[i]), q, tag=ks.setdefault(q, 0)))
                        ks[q] += 1
                    if rbytes[i]:
                        reqs.append(dist.irecv(buf(recv[i], rbytes[i]), q, tag=kr.setdefault(q, 0)))
                        kr[q] += 1
                for r in reqs:
                    r.wait()
                return 0
            except Exception as e:  # noqa: BLE001 -- reported through the status code
                print("cfd2 host transport exchange failed:", e, flush=True)
                return 1

        def allgather(_user, send, recv, nbytes):
            try:
                out = [buf(recv + r * nbytes, nbytes) for r in range(nranks)] if nbytes else None
                if nbytes:
                    dist.all_gather(out, buf(send, nbytes).clone())
                return 0
            except Exception as e:  # noqa: BLE001
                print("cfd2 host transport allgather failed:", e, flush=True)
                return 1

        ex_cb, ag_cb = EXCHANGE_FN(exchange), ALLGATHER_FN(allgather)
        h = _vp()
        _ffi.check(L.cfd_solver_create_dist_host(C.byref(view), C.byref(cfg), int(device), int(nranks), int(rank),
                                                 ex_cb, ag_cb, None, C.byref(h)), "cfd_solver_create_dist_host")
        s = cls(mesh, config=cfg, _handle=h)
        s._transport = (ex_cb, ag_cb)  # the callbacks must outlive the handle
        return s

    def close(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            _ffi.lib().cfd_solver_destroy(h)
        self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- constants (public `constants` field + setters, solver.rs:36-95) --------
    @property
    def constants(self) -> _ffi.Constants:
        c = _ffi.Constants()
        _ffi.check(_ffi.lib().cfd_get_constants(self._h, C.byref(c)), "cfd_get_constants")
        return c

    @constants.setter
    def constants(self, c: _ffi.Constants) -> None:
        _ffi.check(_ffi.lib().cfd_set_constants(self._h, C.byref(c)), "cfd_set_constants")

    def _call(self, name, *args):
        _ffi.check(getattr(_ffi.lib(), name)(self._h, *args), name)

    def set_dt(self, dt): self._call("cfd_set_dt", float(dt))
    def set_viscosity(self, v): self._call("cfd_set_viscosity", float(v))
    def set_alpha_p(self, v): self._call("cfd_set_alpha_p", float(v))
    def set_alpha_u(self, v): self._call("cfd_set_alpha_u", float(v))
    def set_density(self, v): self._call("cfd_set_density", float(v))
    def set_scheme(self, v): self._call("cfd_set_scheme", int(v))
    def set_time_scheme(self, v): self._call("cfd_set_time_scheme", int(v))
    def set_inlet_velocity(self, v): self._call("cfd_set_inlet_velocity", float(v))
    def set_ramp_time(self, v): self._call("cfd_set_ramp_time", float(v))
    def set_precond_type(self, v): self._call("cfd_set_precond_type", int(v))
    def update_constants(self): self._call("cfd_update_constants")

    # -- state ------------------------------------------------------------------
    def set_u(self, u):
        a = np.ascontiguousarray(np.asarray(u, dtype=np.float64).reshape(-1))
        if a.size != 2 * self.num_global_cells:
            raise ValueError("set_u expects one (u, v) pair per mesh cell")
        self._call("cfd_set_u", a.ctypes.data_as(C.POINTER(C.c_double)))

    def set_p(self, p):
        a = np.ascontiguousarray(np.asarray(p, dtype=np.float64).reshape(-1))
        if a.size != self.num_global_cells:
            raise ValueError("set_p expects one value per mesh cell")
        self._call("cfd_set_p", a.ctypes.data_as(C.POINTER(C.c_double)))

    def initialize_history(self): self._call("cfd_initialize_history")
    def step(self): self._call("cfd_step")
    def synchronize(self): self._call("cfd_synchronize")

    # set_u / set_p take GLOBAL arrays (a distributed rank keeps its cells + ghosts)
    def _global_len(self):
        return self.num_global_cells

    def get_u(self) -> np.ndarray:
        a = np.zeros(2 * self.num_cells)
        self._call("cfd_get_u", a.ctypes.data_as(C.POINTER(C.c_double)))
        return a.reshape(-1, 2)

    def get_p(self) -> np.ndarray:
        a = np.zeros(self.num_cells)
        self._call("cfd_get_p", a.ctypes.data_as(C.POINTER(C.c_double)))
        return a

    def get_d_p(self) -> np.ndarray:
        a = np.zeros(self.num_cells)
        self._call("cfd_get_d_p", a.ctypes.data_as(C.POINTER(C.c_double)))
        return a

    # -- public status fields of the reference struct -------------------------
    def step_info(self) -> _ffi.StepInfo:
        i = _ffi.StepInfo()
        self._call("cfd_get_step_info", C.byref(i))
        return i

    # should_stop / degenerate_count / steady_state_count are plain public
    # fields in the reference (structs.rs:244-247): the GUI clears should_stop
    # before it resumes stepping (src/ui/app.rs:852-857)
    def set_stop_state(self, should_stop, degenerate_count, steady_state_count):
        self._call("cfd_set_stop_state", 1 if should_stop else 0, int(degenerate_count), int(steady_state_count))

    def _set_stop_field(self, **kw):
        i = self.step_info()
        cur = dict(should_stop=i.should_stop, degenerate_count=i.degenerate_count,
                   steady_state_count=i.steady_state_count)
        cur.update(kw)
        self.set_stop_state(**cur)

    @property
    def should_stop(self) -> bool: return bool(self.step_info().should_stop)
    @should_stop.setter
    def should_stop(self, v): self._set_stop_field(should_stop=bool(v))
    @property
    def degenerate_count(self) -> int: return int(self.step_info().degenerate_count)
    @degenerate_count.setter
    def degenerate_count(self, v): self._set_stop_field(degenerate_count=int(v))
    @property
    def steady_state_count(self) -> int: return int(self.step_info().steady_state_count)
    @steady_state_count.setter
    def steady_state_count(self, v): self._set_stop_field(steady_state_count=int(v))
    @property
    def outer_iterations(self) -> int: return int(self.step_info().outer_iterations)

    # n_outer_correctors: a public field as well (structs.rs:238), read by every
    # step (coupled_solver.rs:111); its initial value comes from the config
    @property
    def n_outer_correctors(self) -> int: return int(self._n_outer)
    @n_outer_correctors.setter
    def n_outer_correctors(self, v):
        self._call("cfd_set_n_outer_correctors", int(v))
        self._n_outer = int(v)

    # -- instrumentation --------------------------------------------------------
    def profile_enable(self, on=True): self._call("cfd_profile_enable", 1 if on else 0)
    def profile_reset(self): self._call("cfd_profile_reset")

    def graph_enable(self, on=True): self._call("cfd_graph_enable", 1 if on else 0)

    def graph_stats(self):
        """(enabled, graphs captured, iterations replayed) of the FGMRES iteration graphs."""
        e, c, r = C.c_int32(), C.c_uint64(), C.c_uint64()
        self._call("cfd_graph_stats", C.byref(e), C.byref(c), C.byref(r))
        return bool(e.value), c.value, r.value

    def profile_smoother(self):
        ms, n, b = C.c_double(), C.c_uint64(), C.c_double()
        self._call("cfd_profile_smoother", C.byref(ms), C.byref(n), C.byref(b))
        return ms.value, n.value, b.value

    def amg_levels(self):
        nl = C.c_int32()
        rows = (C.c_uint32 * 20)()
        nnz = (C.c_uint64 * 20)()
        self._call("cfd_amg_levels", C.byref(nl), rows, nnz)
        return [(int(rows[i]), int(nnz[i])) for i in range(nl.value)]

    def amg_setup_info(self):
        """(setup path: 0 not built / 1 host / 2 device, [digest of every level image])."""
        path = C.c_int32()
        dig = []
        for li in range(len(self.amg_levels())):
            d = C.c_uint64()
            self._call("cfd_debug_amg_info", li, C.byref(path), C.byref(d))
            dig.append(int(d.value))
        return int(path.value), dig

    def step_algorithmic_bytes(self) -> float:
        return float(_ffi.lib().cfd_step_algorithmic_bytes(self._h))

    def step_layout_bytes(self) -> float:
        """Layout-true bytes of one fixed-schedule step (cfd_step_layout_bytes)."""
        return float(_ffi.lib().cfd_step_layout_bytes(self._h))

    def smoother_layout_bytes(self) -> float:
        """Layout-true bytes of one level-0 smoother sweep (cfd_smoother_layout_bytes)."""
        return float(_ffi.lib().cfd_smoother_layout_bytes(self._h))

    def debug_buffer(self, bid: int) -> np.ndarray:
        n = _ffi.lib().cfd_debug_buffer_len(self._h, bid)
        a = np.zeros(n, dtype=np.float32)
        self._call("cfd_debug_buffer", int(bid), a.ctypes.data_as(C.POINTER(C.c_float)), n)
        return a

    # checkpoint / resume (cfd_state_file_header; read the file with cfd2_amd.state)
    def save_state(self, path):
        """Write the whole solver state to ``path`` (collective on a distributed rank)."""
        self._call("cfd_state_save", os.fsencode(path))

    def load_state(self, path):
        """Replace the state with a saved one (drops this solver's AMG hierarchy)."""
        self._call("cfd_state_load", os.fsencode(path))

    def debug_prepare_assemble(self, assemble=True):
        self._call("cfd_debug_prepare_assemble", 1 if assemble else 0)

    def debug_reference_semantics(self, flags):
        """Test mode: the reference's own semantics (oracle flag bits 1 / 4 /
        8) instead of the canonical resolutions (cfd_debug_reference_semantics;
        one GPU)."""
        self._call("cfd_debug_reference_semantics", int(flags))

    def comm_stats(self, reset=False) -> dict:
        """Transport of this handle (RCCL: ncclCommCount / ncclCommUserRank),
        its HIP device, and the collective traffic since the last reset."""
        c = _ffi.CommStats()
        self._call("cfd_dist_comm_stats", C.byref(c), 1 if reset else 0)
        d = {k: getattr(c, k) for k, _ in _ffi.CommStats._fields_}
        d["transport"] = _ffi.TRANSPORTS.get(c.transport, str(c.transport))
        return d

    def comm_timing_enable(self, enable=True) -> None:
        """cfd_comm_timing_enable: time every halo / all-gather (resets the totals)."""
        self._call("cfd_comm_timing_enable", 1 if enable else 0)

    def comm_timing(self) -> list:
        """cfd_comm_timing: per category (AMG halos per level) the calls, bytes,
        the compute stream's exposed wait and the transport's own time (us)."""
        cap = 64
        buf = (_ffi.CommTimingEntry * cap)()
        n = C.c_int32(0)
        self._call("cfd_comm_timing", buf, cap, C.byref(n))
        out = []
        for e in buf[:n.value]:
            out.append({"category": _ffi.COMM_CATEGORIES.get(e.category, str(e.category)), "level": e.level,
                        "calls": e.calls, "bytes": e.bytes, "wait_us": e.wait_us, "comm_us": e.comm_us})
        return out


def dist_unique_id() -> bytes:
    """RCCL unique id (rank 0 creates it, every rank passes it to create_dist)."""
    L = _bind()
    buf = (C.c_uint8 * 128)()
    _ffi.check(L.cfd_dist_unique_id(buf), "cfd_dist_unique_id")
    return bytes(buf)


class GpuGroup:
    """In-process distributed solver: ``nranks`` ranks on ``devices`` (default
    all on GPU 0), one host thread per rank inside the library.  Same surface
    as GpuSolver; getters return global arrays (owned slices concatenated)."""

    def __init__(self, mesh, nranks: int, devices=None, config: _ffi.Config | None = None,
                 **cfg_overrides):
        L = _bind()
        cfg = config if config is not None else _ffi.default_config(**cfg_overrides)
        view = mesh.view()
        devs = list(devices) if devices is not None else [0] * nranks
        if len(devs) != nranks:
            raise ValueError("one device per rank")
        darr = (C.c_int32 * nranks)(*devs)
        harr = (_vp * nranks)()
        _ffi.check(L.cfd_group_create(C.byref(view), C.byref(cfg), int(nranks), darr, harr),
                   "cfd_group_create")
        self._harr = harr
        self.ranks = [GpuSolver(mesh, config=cfg, _handle=_vp(harr[r])) for r in range(nranks)]
        self.nranks = nranks
        self.num_cells = self.ranks[0].num_global_cells

    def close(self):
        for r in self.ranks:
            r.close()
        self.ranks = []

    def __getattr__(self, name):
        # setters / state writers apply to every rank
        if name.startswith("set_") or name in ("update_constants", "initialize_history",
                                               "profile_enable", "profile_reset", "synchronize"):
            def f(*a, **k):
                for r in self.ranks:
                    getattr(r, name)(*a, **k)
            return f
        raise AttributeError(name)

    @property
    def constants(self):
        return self.ranks[0].constants

    @constants.setter
    def constants(self, c):
        for r in self.ranks:
            r.constants = c

    def step(self):
        _ffi.check(_bind().cfd_group_step(self._harr, self.nranks), "cfd_group_step")

    def _gather(self, getter, comps):
        out = np.zeros((self.num_cells, comps) if comps > 1 else self.num_cells)
        for r in self.ranks:
            c0, c1 = r.owned
            out[c0:c1] = getattr(r, getter)()
        return out

    def debug_fault(self, fail_rank: int) -> None:
        """cfd_debug_group_fault: raises (the injected failure of ``fail_rank``)."""
        _ffi.check(_bind().cfd_debug_group_fault(self._harr, self.nranks, int(fail_rank)),
                   "cfd_debug_group_fault")

    def debug_fault_midstep(self, fail_rank: int) -> None:
        """cfd_debug_group_fault_midstep: a group step in which ``fail_rank``
        fails right after its first prepare(); raises, and the group is then
        marked needs-restore."""
        _ffi.check(_bind().cfd_debug_group_fault_midstep(self._harr, self.nranks, int(fail_rank)),
                   "cfd_debug_group_fault_midstep")

    @property
    def needs_restore(self) -> bool:
        return bool(_bind().cfd_group_needs_restore(self._harr, self.nranks))

    def reset(self) -> None:
        """cfd_group_reset: accept the ranks' current state after a failed step."""
        _ffi.check(_bind().cfd_group_reset(self._harr, self.nranks), "cfd_group_reset")

    def save_state(self, path):
        _ffi.check(_bind().cfd_group_state_save(self._harr, self.nranks, os.fsencode(path)),
                   "cfd_group_state_save")

    def load_state(self, path):
        for r in self.ranks:
            r.load_state(path)

    def get_u(self): return self._gather("get_u", 2)
    def get_p(self): return self._gather("get_p", 1)
    def get_d_p(self): return self._gather("get_d_p", 1)
    def step_info(self): return self.ranks[0].step_info()
    def amg_levels(self): return self.ranks[0].amg_levels()

    @property
    def should_stop(self): return self.ranks[0].should_stop
    @should_stop.setter
    def should_stop(self, v):
        for r in self.ranks:
            r.should_stop = v
    @property
    def degenerate_count(self): return self.ranks[0].degenerate_count
    @property
    def steady_state_count(self): return self.ranks[0].steady_state_count
    @property
    def n_outer_correctors(self): return self.ranks[0].n_outer_correctors
    @n_outer_correctors.setter
    def n_outer_correctors(self, v):
        for r in self.ranks:
            r.n_outer_correctors = v


def dist_plan(mesh, nranks: int, rank: int) -> dict:
    """Host-only halo plan of one rank (no GPU): owned range, ghost ids, and per
    peer the receive / send counts and the owned ids sent."""
    L = _bind()
    view = mesh.view()
    c0, c1, ng, npeer, ns = (C.c_uint32() for _ in range(5))
    z = None
    _ffi.check(L.cfd_dist_plan(C.byref(view), nranks, rank, C.byref(c0), C.byref(c1), C.byref(ng),
                               C.byref(npeer), C.byref(ns), z, z, z, z, z), "cfd_dist_plan")
    ghost = np.zeros(max(ng.value, 1), dtype=np.uint32)
    prank = np.zeros(max(npeer.value, 1), dtype=np.int32)
    precv = np.zeros(max(npeer.value, 1), dtype=np.uint32)
    psend = np.zeros(max(npeer.value, 1), dtype=np.uint32)
    sendg = np.zeros(max(ns.value, 1), dtype=np.uint32)
    u32 = lambda a: a.ctypes.data_as(C.POINTER(C.c_uint32))  # noqa: E731
    _ffi.check(L.cfd_dist_plan(C.byref(view), nranks, rank, None, None, None, None, None, u32(ghost),
                               prank.ctypes.data_as(C.POINTER(C.c_int32)), u32(precv), u32(psend),
                               u32(sendg)), "cfd_dist_plan")
    n = npeer.value
    return dict(c0=c0.value, c1=c1.value, ghost=ghost[:ng.value], peers=prank[:n].tolist(),
                recv=precv[:n].tolist(), send=psend[:n].tolist(), send_ids=sendg[:ns.value])


def rccl_selftest(device: int = 0) -> None:
    """RCCL transport plumbing check on one GPU (raises on failure)."""
    _ffi.check(_bind().cfd_debug_rccl_selftest(int(device)), "cfd_debug_rccl_selftest")
