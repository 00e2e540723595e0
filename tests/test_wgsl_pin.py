"""The oracle pinned to the REFERENCE'S OWN KERNELS (CPU tests).

The reference's WGSL shaders, executed on the CPU by oracle/wgsl/wgsl_exec.py
under the Rust host sequence restated in tests/wgsl_ref.py, produced
tests/golden/wgsl_ref.npz (tests/golden/make_wgsl_golden.py, run in the
build container where /root/reference exists).  Two legal executions of the
reference are recorded per case:
  A  workgroups in dispatch order, a workgroup's lanes in lockstep, wgpu's
     Restrict bounds policy  == oracle with reference-semantics flags 15;
  B  the whole dispatch resident and in lockstep, naga's ReadZeroSkipWrite
     policy                  == oracle with flags 4 (the reference's
     reduction order; prepare's snapshot reads, the out-of-place smoother and
     restrict_residual's skipped rows are then the reference's own
     behaviour, not choices).
The canonical oracle (flags 0, what the HIP path reproduces bit for bit)
differs from B only by the summation tree of its reductions.  Kernels
without a reduction (prepare_coupled + coupled_assembly_merged) are pinned at
flags 0 directly; tests/test_gpu_parity.py ties the HIP kernels to the same
fixture.  Every comparison is bit-exact (f32 bytes; SHA-256 of each step's
fields)."""
import hashlib
import os

import numpy as np
import pytest

from cfd2_amd import default_config
from tests.golden.make_wgsl_golden import MODES, cases, digest, info_vec
from tests.oracle_py import OracleSolver

FIX = os.path.join(os.path.dirname(__file__), "golden", "wgsl_ref.npz")
F = np.float32


@pytest.fixture(scope="module")
def fix():
    with np.load(FIX) as z:
        return {k: z[k] for k in z.files}


def _case_ids():
    return [(c[0], m) for c in cases() for m in c[5]]


@pytest.mark.parametrize("name,mode", _case_ids())
def test_oracle_equals_reference_kernels(fix, name, mode):
    """every step's fields (SHA-256 of their f32 bytes) and statistics, the
    final fields element by element"""
    c = {x[0]: x for x in cases()}[name]
    _, mk, setup, kw, steps, _ = c
    mesh = mk()
    cfg = dict(kw)
    o = OracleSolver(mesh, config=default_config(**cfg))
    o.set_semantics(MODES[mode][2])
    setup(o, mesh)
    key = f"{name}/{mode}"
    for k in range(steps):
        o.step()
        assert digest(o) == str(fix[f"{key}/digests"][k]), f"{key} step {k}: fields differ from the reference kernels"
        np.testing.assert_array_equal(info_vec(o), fix[f"{key}/info"][k], err_msg=f"{key} step {k} statistics")
    if f"{key}/u" in fix:
        assert np.array_equal(o.get_u().astype(F), fix[f"{key}/u"])
        assert np.array_equal(o.get_p().astype(F), fix[f"{key}/p"])
        assert np.array_equal(o.get_d_p().astype(F), fix[f"{key}/d_p"])


# canonical (flags 0) vs reference kernels (B), relative L2 bounds: the
# reference's own tests reach natural convergence, the fixed 3 x 10 schedule
# stops its solves early (p is then set by the last inexact solve)
_CANON_BOUND = {"amg_test_amg": (1e-5, 1e-5), "amg_test_jacobi": (1e-5, 1e-5), "schemes_s0t0": (1e-5, 1e-5),
                "schemes_s1t0": (1e-5, 1e-5), "schemes_s2t0": (1e-5, 1e-5), "schemes_s0t1": (1e-5, 1e-5),
                "fixed_amg": (1e-5, 1e-4), "fixed_jacobi": (1e-5, 5e-4)}


@pytest.mark.parametrize("name", sorted(_CANON_BOUND))
def test_canonical_differs_from_reference_only_by_reduction_order(fix, name):
    """flags 0 (the HIP path's semantics) vs the reference kernels under B:
    not bit-equal (the reduction tree), within the rounding-level bounds"""
    _, mk, setup, kw, steps, _ = [c for c in cases() if c[0] == name][0]
    mesh = mk()
    o = OracleSolver(mesh, config=default_config(**kw))
    setup(o, mesh)
    for _ in range(steps):
        o.step()
    for f, got, bound in (("u", o.get_u(), _CANON_BOUND[name][0]), ("p", o.get_p(), _CANON_BOUND[name][1])):
        ref = fix[f"{name}/B/{f}"].astype(np.float64)
        rel = np.linalg.norm(got - ref) / max(np.linalg.norm(ref), 1e-30)
        assert 0 < rel <= bound, (f, rel)


@pytest.mark.parametrize("scheme,time_scheme", [(0, 0), (1, 0), (2, 0), (0, 1)])
def test_kernels_canonical_equal_reference(fix, scheme, time_scheme):
    """prepare_coupled + coupled_assembly_merged on a random state: the
    canonical oracle's buffers == the reference shaders' (schedule B)"""
    from tests.meshes import channel_obstacle
    mesh = channel_obstacle()
    o = OracleSolver(mesh)
    rng = np.random.default_rng(11 + scheme + 3 * time_scheme)
    u0 = rng.uniform(-1, 1, size=(mesh.num_cells(), 2))
    u1 = rng.uniform(-1, 1, size=(mesh.num_cells(), 2))
    o.set_u(u1)
    o.initialize_history()
    o.set_u(u0)
    o.set_dt(0.002)
    o.set_dt(0.003)
    o.set_scheme(scheme)
    o.set_time_scheme(time_scheme)
    c = o.constants
    c.time = 0.05
    o.constants = c
    o.debug_prepare_assemble(False)
    o.debug_prepare_assemble(True)
    key = f"kernels_s{scheme}t{time_scheme}"
    got = dict(fluxes=o.debug_buffer(0), grad_u=o.debug_buffer(1), grad_v=o.debug_buffer(2),
               rhs=o.debug_buffer(3), diag_u_inv=o.debug_buffer(5), diag_v_inv=o.debug_buffer(6),
               diag_p_inv=o.debug_buffer(7), scalar_matrix=o.debug_buffer(8), matrix=o.debug_buffer(9),
               grad_p=o.debug_buffer(10), d_p=o.get_d_p().astype(F))
    for k, v in got.items():
        ref = fix[f"{key}/{k}"]
        assert v.shape == ref.shape, k
        assert np.array_equal(v, ref), f"{key} {k}: max diff {np.abs(v - ref).max()}"


def test_fixture_holds_no_reference_text():
    """the fixture is data: numeric arrays and hex digests only"""
    with np.load(FIX) as z:
        for k in z.files:
            a = z[k]
            assert a.dtype.kind in "fiu" or (a.dtype.kind == "U" and all(len(s) == 64 for s in a.reshape(-1))), k


# ------------------------------------------------------------------ live
from tests import wgsl_ref  # noqa: E402


@pytest.mark.skipif(not wgsl_ref.available(), reason="/root/reference is present only in the build container")
@pytest.mark.parametrize("mode", ["A", "B", "C"])
def test_live_reference_kernels(mode):
    """re-runs the reference shaders now (1 step of 2 Picard x 4 FGMRES, AMG,
    amg_test setup) against the oracle in the matching semantics"""
    from tests.meshes import backwards_step
    from tests.test_oracle import setup_amg_test
    mesh = backwards_step()
    kw = dict(convergence_lag=0, fixed_outer=2, fixed_inner=4)
    sched, bounds, flags, amg = MODES[mode]
    r = wgsl_ref.WgslRefSolver(mesh, schedule=sched, bounds=bounds, amg=amg, **kw)
    o = OracleSolver(mesh, config=default_config(**kw))
    o.set_semantics(flags)
    for s in (r, o):
        setup_amg_test(s, mesh, 1)
        s.step()
    assert digest(r) == digest(o)
    np.testing.assert_array_equal(info_vec(r), info_vec(o))


# ------------------------------------------------------- the executor itself
_PROBE = """
struct P { n: u32, w: f32, z: u32, }
@group(0) @binding(0) var<storage, read_write> x: array<f32>;
@group(0) @binding(1) var<storage, read_write> y: array<u32>;
@group(0) @binding(2) var<uniform> prm: P;
var<workgroup> sh: array<f32, 64>;

fn inv(v: f32) -> f32 {
    if (abs(v) > 1e-14) { return 1.0 / v; }
    return 0.0;
}

@compute @workgroup_size(64)
fn left(@builtin(global_invocation_id) g: vec3<u32>) {
    let i = g.x;
    if (i > 0u && i < prm.n) { x[i] = x[i - 1u]; }
}

@compute @workgroup_size(64)
fn oob(@builtin(global_invocation_id) g: vec3<u32>) {
    let i = g.x;
    y[i] = u32(x[i + 1000u]);
}

@compute @workgroup_size(64)
fn same_address(@builtin(global_invocation_id) g: vec3<u32>, @builtin(local_invocation_id) l: vec3<u32>) {
    y[0] = l.x + 1u;
}

@compute @workgroup_size(64)
fn loops(@builtin(global_invocation_id) g: vec3<u32>) {
    let i = g.x;
    var s = 0.0;
    for (var k = 0u; k < 100u; k++) {
        if (k >= i) { break; }
        if (k % 2u == 1u) { continue; }
        s += 1.0;
    }
    x[i] = s + inv(f32(i)) + mix(0.25, 2.0, prm.w) + smoothstep(0.0, 2.0, prm.w);
    y[i] = i / prm.z + (i % prm.z);
}

@compute @workgroup_size(64)
fn tree(@builtin(local_invocation_id) l: vec3<u32>, @builtin(workgroup_id) w: vec3<u32>) {
    sh[l.x] = x[w.x * 64u + l.x];
    workgroupBarrier();
    for (var s = 32u; s > 0u; s >>= 1u) {
        if (l.x < s) { sh[l.x] += sh[l.x + s]; }
        workgroupBarrier();
    }
    if (l.x == 0u) { y[w.x] = bitcast<u32>(sh[0]); }
}
"""


def _probe(entry, x, y, n, w=0.5, z=0, groups=2, schedule="workgroups", bounds="restrict"):
    from wgsl.wgsl_exec import Binding, Dispatcher, buffer
    d = Dispatcher(_PROBE)
    bx, by = buffer(np.asarray(x, F)), buffer(np.asarray(y, np.uint32))
    prm = buffer(np.array([n, np.array(w, F).view(np.uint32), z], np.uint32))
    d.dispatch(entry, {(0, 0): Binding(bx), (0, 1): Binding(by), (0, 2): Binding(prm)}, (groups,),
               schedule=schedule, bounds=bounds)
    return bx.f.copy(), by.u.copy()


def test_executor_schedules():
    """workgroups in order see earlier workgroups' stores; a resident
    dispatch reads everything first; a workgroup's lanes always read first"""
    x0 = np.arange(128, dtype=F)
    xw, _ = _probe("left", x0, np.zeros(1), 128)
    xd, _ = _probe("left", x0, np.zeros(1), 128, schedule="dispatch")
    assert np.array_equal(xd[1:], x0[:-1])             # snapshot reads
    assert np.array_equal(xw[1:64], x0[0:63])           # inside workgroup 0: lockstep
    assert xw[64] == x0[62]                             # workgroup 1 lane 0 read wg 0's new x[63]
    assert np.array_equal(xw[65:], x0[64:127])


def test_executor_bounds_policies():
    x0 = np.arange(100, dtype=F)
    _, yr = _probe("oob", x0, np.zeros(100), 100, groups=1)
    assert np.all(yr[:64] == 99)  # Restrict: clamped to the last element
    _, yz = _probe("oob", x0, np.full(100, 7), 100, groups=1, bounds="zero")
    assert np.all(yz[:64] == 0)   # ReadZeroSkipWrite: reads 0
    _, y2 = _probe("oob", x0, np.full(40, 7), 100, groups=1, bounds="zero")
    assert np.all(y2 == 0)        # lanes >= 40 dropped their stores, the rest wrote 0
    _, y3 = _probe("oob", x0, np.full(40, 7), 100, groups=1)
    assert y3[39] == 99           # Restrict: lanes >= 40 wrote onto the last element


def test_executor_same_address_highest_lane():
    _, y = _probe("same_address", np.zeros(4), np.zeros(4), 4, groups=1)
    assert y[0] == 64


def test_executor_control_flow_and_arithmetic():
    x, y = _probe("loops", np.zeros(128), np.zeros(128), 128, w=0.5, z=3)
    i = np.arange(128)
    s = ((np.minimum(i, 100) + 1) // 2).astype(F)  # even k below min(i, 100)
    inv = np.where(i > 0, F(1) / np.maximum(i, 1).astype(F), F(0))
    mix = F(0.25) * (F(1) - F(0.5)) + F(2.0) * F(0.5)
    t = np.clip((F(0.5) - F(0)) / (F(2) - F(0)), F(0), F(1)).astype(F)
    sm = t * t * (F(3) - F(2) * t)
    assert np.array_equal(x, ((s + inv) + mix) + sm)
    assert np.array_equal(y, i // 3 + i % 3)
    _, y0 = _probe("loops", np.zeros(128), np.zeros(128), 128, z=0)
    assert np.array_equal(y0, i)  # integer division by zero: the dividend; modulo: 0


def test_executor_workgroup_tree():
    x0 = np.random.default_rng(3).standard_normal(128).astype(F)
    for sched in ("workgroups", "dispatch"):
        _, y = _probe("tree", x0, np.zeros(2), 128, schedule=sched)
        for w in range(2):
            s = x0[64 * w:64 * w + 64].copy()
            st = 32
            while st:
                s[:st] = s[:st] + s[st:2 * st]
                st //= 2
            assert y[w] == s[:1].view(np.uint32)[0], (sched, w)


def test_digest_is_field_bytes():
    class S:
        def get_u(self): return np.ones((2, 2))
        def get_p(self): return np.zeros(2)
        def get_d_p(self): return np.zeros(2)
    h = hashlib.sha256()
    for a in (np.ones((2, 2), F), np.zeros(2, F), np.zeros(2, F)):
        h.update(a.tobytes())
    assert digest(S()) == h.hexdigest()


FIX_C1 = os.path.join(os.path.dirname(__file__), "golden", "wgsl_ref_c1.npz")


def test_oracle_equals_reference_kernels_c1():
    """BASELINE configs[1] (1.0 M cells, bench geometry and physics, 2 Picard
    x 6 FGMRES, AMG with its 9-level hierarchy): oracle flags 4 == the
    reference's kernels under B at every step"""
    from tests.golden.make_wgsl_golden import C1
    name, mk, setup, kw, steps = C1
    mesh = mk()
    o = OracleSolver(mesh, config=default_config(**kw))
    o.set_semantics(4)
    setup(o, mesh)
    with np.load(FIX_C1) as z:
        for k in range(steps):
            o.step()
            assert digest(o) == str(z[f"{name}/B/digests"][k]), f"C1 step {k}"
            np.testing.assert_array_equal(info_vec(o), z[f"{name}/B/info"][k], err_msg=f"C1 step {k}")
