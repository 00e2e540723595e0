"""Reader / writer of the solver checkpoint file (``cfd_state_save`` /
``cfd_state_load``; layout in include/cfd2_amd.h, ``cfd_state_file_header``).

The file is: a 512-byte header, then GLOBAL per-cell f32 arrays -- the three
FluidState ring slots and the check_evolution snapshot (u[N,2], p[N], d_p[N],
grad_p[N,2] each), the FGMRES solution x[N,3] -- and, when the AMG hierarchy
had been built, the scalar matrix it was built from (CSR row pointers u64[N+1],
values f32[nnz]).  Reading maps the file (no copy); writing lets a caller
build a state from arrays (initial conditions with a full time history, or
fixtures) that ``GpuSolver.load_state`` then resumes from.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field

import numpy as np

from ._ffi import Constants, StateFileHeader, StepInfo

MAGIC = b"CFD2STAT"
VERSION = 1
HEADER_BYTES = 512
_FIELDS = (("u", 2), ("p", 1), ("d_p", 1), ("grad_p", 2))  # order inside a FluidState block


def _offsets(n: int, nnz: int) -> dict:
    off, o = {}, HEADER_BYTES
    for blk in ("slot0", "slot1", "slot2", "prev"):
        for name, comps in _FIELDS:
            off[(blk, name)] = o
            o += 4 * comps * n
    off["x"] = o
    o += 12 * n
    if nnz:
        off["amg_rowptr"] = o
        o += 8 * (n + 1)
        off["amg_val"] = o
        o += 4 * nnz
    off["total"] = o
    return off


@dataclass
class SolverState:
    """One checkpoint.  ``slots[k]`` / ``prev`` are dicts of u (N,2), p (N,),
    d_p (N,), grad_p (N,2), all float32; ``x`` is (N,3) float32."""
    num_faces: int
    step_index: int
    constants: Constants
    info: StepInfo
    slots: list
    prev: dict
    x: np.ndarray
    have_prev: bool = False
    inner_has_last: bool = False
    inner_last: float = 0.0
    variance: list = field(default_factory=list)   # [(var_u, var_v)], oldest first, <= 10
    amg_age: int = 0                                # steps since the hierarchy was built
    amg_local_aggregation: int = 0                  # the saving run's aggregation mode
    nranks: int = 0                                 # the saving run's rank count (0: not recorded)
    amg_rowptr: np.ndarray | None = None            # uint64 (N+1,) or None
    amg_val: np.ndarray | None = None               # float32 (nnz,)

    @property
    def num_cells(self) -> int:
        return int(self.x.shape[0])

    @property
    def current(self) -> dict:
        """The FluidState slot the solver reports (get_u / get_p): ring slot
        ``state`` of the rotation table of coupled_solver.rs:43-71."""
        return self.slots[(0, 2, 1)[self.step_index]]


def read_state(path) -> SolverState:
    mm = np.memmap(path, dtype=np.uint8, mode="r")
    if mm.size < HEADER_BYTES:
        raise ValueError(f"{path}: not a solver state file")
    h = StateFileHeader.from_buffer_copy(bytes(mm[:HEADER_BYTES]))
    if h.magic != MAGIC or h.version != VERSION or h.header_bytes != HEADER_BYTES:
        raise ValueError(f"{path}: bad magic / version")
    n, nnz = int(h.num_cells), int(h.amg_nnz)
    off = _offsets(n, nnz)
    if off["total"] != mm.size:
        raise ValueError(f"{path}: size {mm.size} != {off['total']} expected")

    def arr(o, dtype, count, shape=None):
        a = np.frombuffer(mm, dtype=dtype, count=count, offset=o)
        return a.reshape(shape) if shape else a

    def block(blk):
        return {name: arr(off[(blk, name)], np.float32, comps * n, (n, comps) if comps > 1 else None)
                for name, comps in _FIELDS}

    return SolverState(
        num_faces=int(h.num_faces), step_index=int(h.step_index), constants=h.constants, info=h.info,
        slots=[block(f"slot{k}") for k in range(3)], prev=block("prev"),
        x=arr(off["x"], np.float32, 3 * n, (n, 3)),
        have_prev=bool(h.have_prev), inner_has_last=bool(h.inner_has_last), inner_last=float(h.inner_last),
        variance=[(h.variance[k][0], h.variance[k][1]) for k in range(h.n_variance)], amg_age=int(h.amg_age),
        amg_local_aggregation=int(h.amg_local_aggregation), nranks=int(h.nranks),
        amg_rowptr=arr(off["amg_rowptr"], np.uint64, n + 1) if nnz else None,
        amg_val=arr(off["amg_val"], np.float32, nnz) if nnz else None)


def write_state(path, st: SolverState) -> None:
    """Write ``st`` in the format cfd_state_load reads (atomic replace)."""
    n = st.num_cells
    nnz = 0 if st.amg_val is None else int(st.amg_val.size)
    if nnz and (st.amg_rowptr is None or st.amg_rowptr.shape != (n + 1,) or int(st.amg_rowptr[-1]) != nnz):
        raise ValueError("amg_rowptr must be (N+1,) ending at amg_val.size")
    if len(st.variance) > 10:
        raise ValueError("at most 10 variance entries")
    h = StateFileHeader()
    h.magic = MAGIC
    h.version = VERSION
    h.header_bytes = HEADER_BYTES
    h.num_cells, h.num_faces, h.amg_nnz = n, int(st.num_faces), nnz
    h.step_index = int(st.step_index)
    h.have_prev, h.inner_has_last = int(st.have_prev), int(st.inner_has_last)
    h.inner_last = float(st.inner_last)
    h.n_variance = len(st.variance)
    for k, (a, b) in enumerate(st.variance):
        h.variance[k][0], h.variance[k][1] = float(a), float(b)
    h.constants = st.constants
    h.info = st.info
    h.amg_age = int(st.amg_age)
    h.amg_local_aggregation = int(st.amg_local_aggregation)
    h.nranks = int(st.nranks)
    tmp = f"{path}.tmp{os.getpid()}"
    with open(tmp, "wb") as f:
        f.write(bytes(h))
        for blk in list(st.slots) + [st.prev]:
            for name, comps in _FIELDS:
                a = np.ascontiguousarray(blk[name], dtype=np.float32)
                if a.size != comps * n:
                    raise ValueError(f"{name}: {a.size} values, expected {comps * n}")
                f.write(a.tobytes())
        x = np.ascontiguousarray(st.x, dtype=np.float32)
        if x.size != 3 * n:
            raise ValueError("x must hold 3N values")
        f.write(x.tobytes())
        if nnz:
            f.write(np.ascontiguousarray(st.amg_rowptr, dtype=np.uint64).tobytes())
            f.write(np.ascontiguousarray(st.amg_val, dtype=np.float32).tobytes())
    os.replace(tmp, path)
