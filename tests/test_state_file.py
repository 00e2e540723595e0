"""Checkpoint file format (cfd2_amd.state <-> cfd_state_file_header), CPU only."""
import ctypes as C

import numpy as np
import pytest

from cfd2_amd import _ffi
from cfd2_amd.state import HEADER_BYTES, SolverState, _offsets, read_state, write_state


def _state(n, nnz, seed=0):
    rng = np.random.default_rng(seed)

    def blk():
        return {"u": rng.standard_normal((n, 2), dtype=np.float32), "p": rng.standard_normal(n, dtype=np.float32),
                "d_p": rng.standard_normal(n, dtype=np.float32),
                "grad_p": rng.standard_normal((n, 2), dtype=np.float32)}
    c = _ffi.Constants(dt=1e-3, dt_old=2e-3, time=0.5, precond_type=1, time_scheme=1)
    info = _ffi.StepInfo(degenerate_count=3, outer_iterations=7)
    rp = None if not nnz else np.concatenate([[0], np.sort(rng.integers(0, nnz, n - 1)), [nnz]]).astype(np.uint64)
    return SolverState(num_faces=4 * n, step_index=1, constants=c, info=info, slots=[blk(), blk(), blk()],
                       prev=blk(), x=rng.standard_normal((n, 3), dtype=np.float32), have_prev=True,
                       inner_has_last=True, inner_last=0.25, variance=[(1.0, 2.0), (3.0, 4.0)],
                       amg_rowptr=rp, amg_val=rng.standard_normal(nnz, dtype=np.float32) if nnz else None,
                       amg_local_aggregation=1, nranks=4)


def test_header_layout_matches_c():
    assert C.sizeof(_ffi.StateFileHeader) == HEADER_BYTES == 512
    assert _ffi.StateFileHeader.variance.offset == 64
    assert _ffi.StateFileHeader.constants.offset == 224
    assert _ffi.StateFileHeader.info.offset == 280
    assert _ffi.StateFileHeader.amg_age.offset == 336 and _ffi.StateFileHeader.nranks.offset == 344


@pytest.mark.parametrize("nnz", [0, 37])
def test_round_trip(tmp_path, nnz):
    n = 11
    st = _state(n, nnz)
    p = tmp_path / "s.bin"
    write_state(p, st)
    assert p.stat().st_size == _offsets(n, nnz)["total"]
    r = read_state(p)
    assert r.num_cells == n and r.num_faces == 4 * n and r.step_index == 1
    assert r.have_prev and r.inner_has_last and r.inner_last == 0.25
    assert r.variance == [(1.0, 2.0), (3.0, 4.0)]
    assert r.constants.time == np.float32(0.5) and r.constants.time_scheme == 1
    assert r.info.degenerate_count == 3 and r.info.outer_iterations == 7
    assert r.amg_local_aggregation == 1 and r.nranks == 4
    for a, b in zip(r.slots + [r.prev], st.slots + [st.prev]):
        for k in a:
            assert np.array_equal(a[k], b[k])
    assert np.array_equal(r.x, st.x)
    assert r.current is r.slots[2]  # step_index 1 -> ring slot 2 (coupled_solver.rs:43-71)
    if nnz:
        assert np.array_equal(r.amg_rowptr, st.amg_rowptr) and np.array_equal(r.amg_val, st.amg_val)
    else:
        assert r.amg_val is None
    # write(read(f)) == f
    q = tmp_path / "t.bin"
    write_state(q, r)
    assert q.read_bytes() == p.read_bytes()


def test_rejects_bad_files(tmp_path):
    p = tmp_path / "s.bin"
    write_state(p, _state(5, 0))
    raw = p.read_bytes()
    (tmp_path / "short.bin").write_bytes(raw[:-1])
    with pytest.raises(ValueError, match="size"):
        read_state(tmp_path / "short.bin")
    (tmp_path / "magic.bin").write_bytes(b"XXXXXXXX" + raw[8:])
    with pytest.raises(ValueError, match="magic"):
        read_state(tmp_path / "magic.bin")
    st = _state(5, 4)
    st.amg_rowptr[-1] = 3
    with pytest.raises(ValueError, match="amg_rowptr"):
        write_state(tmp_path / "bad.bin", st)
