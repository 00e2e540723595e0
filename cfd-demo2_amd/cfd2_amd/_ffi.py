"""ctypes binding of include/cfd2_amd.h (the C ABI of the native library).

The library is built in-tree by ``__graft_entry__.build()`` into
``cfd2_amd/_lib/libcfd2_amd.so``.  There is no fallback: if the library is
missing, importing the solver raises.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# CFD2_AMD_LIB selects an alternative build of the same library (A/B variants
# made by tools/ab_variants.py); default: the in-tree build.
LIB_PATH = os.environ.get("CFD2_AMD_LIB") or os.path.join(_HERE, "_lib", "libcfd2_amd.so")

u32p = C.POINTER(C.c_uint32)
f64p = C.POINTER(C.c_double)


class MeshView(C.Structure):
    _fields_ = [
        ("num_cells", C.c_uint32),
        ("num_faces", C.c_uint32),
        ("face_owner", u32p),
        ("face_neighbor", u32p),
        ("face_boundary", u32p),
        ("face_area", f64p),
        ("face_nx", f64p),
        ("face_ny", f64p),
        ("face_cx", f64p),
        ("face_cy", f64p),
        ("cell_cx", f64p),
        ("cell_cy", f64p),
        ("cell_vol", f64p),
        ("cell_face_offsets", u32p),
        ("cell_faces", u32p),
    ]


class Geometry(C.Structure):
    _fields_ = [("kind", C.c_int32), ("p", C.c_double * 8)]


class Constants(C.Structure):
    _fields_ = [
        ("dt", C.c_float),
        ("dt_old", C.c_float),
        ("time", C.c_float),
        ("viscosity", C.c_float),
        ("density", C.c_float),
        ("component", C.c_uint32),
        ("alpha_p", C.c_float),
        ("scheme", C.c_uint32),
        ("alpha_u", C.c_float),
        ("stride_x", C.c_uint32),
        ("time_scheme", C.c_uint32),
        ("inlet_velocity", C.c_float),
        ("ramp_time", C.c_float),
        ("precond_type", C.c_uint32),
    ]


class Config(C.Structure):
    _fields_ = [
        ("n_outer_correctors", C.c_int32),
        ("convergence_lag", C.c_int32),
        ("fixed_outer", C.c_int32),
        ("fixed_inner", C.c_int32),
        ("max_restart", C.c_int32),
        ("max_outer_restarts", C.c_int32),
        ("fgmres_rtol", C.c_float),
        ("fgmres_atol", C.c_float),
        ("log_level", C.c_int32),
        ("amg_rebuild_interval", C.c_int32),
        ("amg_local_aggregation", C.c_int32),
        ("comm_timeout_s", C.c_float),
    ]


class LinearStats(C.Structure):
    _fields_ = [
        ("iterations", C.c_uint32),
        ("residual", C.c_float),
        ("converged", C.c_int32),
        ("diverged", C.c_int32),
        ("time_s", C.c_double),
    ]


class StepInfo(C.Structure):
    _fields_ = [
        ("should_stop", C.c_int32),
        ("degenerate_count", C.c_uint32),
        ("steady_state_count", C.c_uint32),
        ("outer_residual_u", C.c_float),
        ("outer_residual_p", C.c_float),
        ("outer_iterations", C.c_uint32),
        ("stats_p", LinearStats),
        ("total_linear_iterations", C.c_uint32),
    ]


class CommTimingEntry(C.Structure):  # cfd_comm_timing_entry
    _fields_ = [
        ("category", C.c_int32),
        ("level", C.c_int32),
        ("calls", C.c_uint64),
        ("bytes", C.c_uint64),
        ("wait_us", C.c_double),
        ("comm_us", C.c_double),
    ]


COMM_CATEGORIES = {0: "krylov_halo", 1: "state_halo", 2: "reduction_allgather", 3: "replicated_level_allgather",
                   4: "amg_halo"}


class CommStats(C.Structure):  # cfd_comm_stats
    _fields_ = [
        ("transport", C.c_int32),
        ("comm_count", C.c_int32),
        ("comm_rank", C.c_int32),
        ("device", C.c_int32),
        ("exchanges", C.c_uint64),
        ("allgathers", C.c_uint64),
        ("bytes_sent", C.c_uint64),
        ("bytes_gathered", C.c_uint64),
    ]


TRANSPORTS = {0: "none", 1: "rccl", 2: "in-process", 3: "host-staged"}


class StateFileHeader(C.Structure):  # cfd_state_file_header (512 bytes)
    _fields_ = [
        ("magic", C.c_char * 8),
        ("version", C.c_uint32),
        ("header_bytes", C.c_uint32),
        ("num_cells", C.c_uint64),
        ("num_faces", C.c_uint64),
        ("amg_nnz", C.c_uint64),
        ("step_index", C.c_int32),
        ("have_prev", C.c_int32),
        ("inner_has_last", C.c_int32),
        ("inner_last", C.c_float),
        ("n_variance", C.c_uint32),
        ("reserved0", C.c_uint32),
        ("variance", (C.c_double * 2) * 10),
        ("constants", Constants),
        ("info", StepInfo),
        ("amg_age", C.c_uint32),
        ("amg_local_aggregation", C.c_int32),
        ("nranks", C.c_int32),
        ("reserved", C.c_uint8 * 164),
    ]


def default_config(**overrides) -> Config:
    cfg = Config(
        n_outer_correctors=20,
        convergence_lag=1,
        fixed_outer=0,
        fixed_inner=0,
        max_restart=50,
        max_outer_restarts=20,
        fgmres_rtol=1e-5,
        fgmres_atol=1e-7,
        log_level=0,
        amg_rebuild_interval=0,
        amg_local_aggregation=0,
        comm_timeout_s=180.0,
    )
    for k, v in overrides.items():
        setattr(cfg, k, v)
    return cfg


# Every symbol include/cfd2_amd.h declares (checked by tests/test_capi.py).
EXPORTED = [
    "cfd_last_error", "cfd_build_id",
    "cfd_mesh_generate_cut_cell", "cfd_mesh_generate_voronoi", "cfd_mesh_generate_delaunay", "cfd_mesh_get_topology", "cfd_mesh_smooth", "cfd_mesh_max_skewness", "cfd_mesh_get_view",
    "cfd_mesh_get_vertices", "cfd_mesh_save", "cfd_mesh_load", "cfd_mesh_destroy",
    "cfd_config_default", "cfd_solver_create", "cfd_solver_destroy", "cfd_set_u", "cfd_set_p",
    "cfd_get_constants", "cfd_set_constants", "cfd_set_dt", "cfd_set_viscosity", "cfd_set_alpha_p",
    "cfd_set_alpha_u", "cfd_set_density", "cfd_set_scheme", "cfd_set_time_scheme",
    "cfd_set_inlet_velocity", "cfd_set_ramp_time", "cfd_set_precond_type", "cfd_update_constants",
    "cfd_initialize_history", "cfd_step", "cfd_get_u", "cfd_get_p", "cfd_get_d_p",
    "cfd_get_step_info", "cfd_set_stop_state", "cfd_set_n_outer_correctors", "cfd_num_cells", "cfd_num_faces", "cfd_state_save", "cfd_state_load", "cfd_synchronize",
    "cfd_group_state_save", "cfd_profile_enable", "cfd_profile_reset",
    "cfd_profile_smoother", "cfd_graph_enable", "cfd_graph_stats", "cfd_amg_levels", "cfd_step_algorithmic_bytes", "cfd_smoother_layout_bytes", "cfd_step_layout_bytes", "cfd_debug_buffer",
    "cfd_debug_buffer_len", "cfd_debug_prepare_assemble", "cfd_debug_reference_semantics", "cfd_debug_amg_info",
    "cfd_dist_unique_id", "cfd_solver_create_dist", "cfd_solver_create_dist_host", "cfd_group_create",
    "cfd_group_step",
    "cfd_dist_info", "cfd_dist_plan", "cfd_debug_rccl_selftest", "cfd_debug_comm_watchdog", "cfd_dist_comm_stats",
    "cfd_debug_group_fault", "cfd_debug_group_fault_midstep", "cfd_group_reset", "cfd_group_needs_restore",
    "cfd_comm_timing_enable", "cfd_comm_timing",
]

_lib = None


def lib() -> C.CDLL:
    """Load the native library (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(
            f"native library not built: {LIB_PATH} (run __graft_entry__.build())")
    L = C.CDLL(LIB_PATH)
    vp = C.c_void_p
    L.cfd_last_error.restype = C.c_char_p
    L.cfd_build_id.restype = C.c_char_p
    L.cfd_mesh_generate_cut_cell.argtypes = [C.POINTER(Geometry), C.c_double, C.c_double, C.c_double,
                                             C.c_double, C.c_double, C.POINTER(vp)]
    u32pp = C.POINTER(C.POINTER(C.c_uint32))
    L.cfd_mesh_get_topology.argtypes = [vp, u32pp, u32pp, u32pp, u32pp]
    for fn in (L.cfd_mesh_generate_voronoi, L.cfd_mesh_generate_delaunay):
        fn.argtypes = [C.POINTER(Geometry), C.c_double, C.c_double, C.c_double, C.c_double, C.c_double,
                       C.c_uint64, C.POINTER(vp)]
    L.cfd_mesh_smooth.argtypes = [vp, C.POINTER(Geometry), C.c_double, C.c_int32, C.POINTER(C.c_int32)]
    L.cfd_mesh_max_skewness.argtypes = [vp]
    L.cfd_mesh_max_skewness.restype = C.c_double
    L.cfd_mesh_get_view.argtypes = [vp, C.POINTER(MeshView)]
    L.cfd_mesh_get_vertices.argtypes = [vp, C.POINTER(C.c_uint32), C.POINTER(f64p), C.POINTER(f64p),
                                        C.POINTER(C.POINTER(C.c_uint8))]
    L.cfd_mesh_save.argtypes = [vp, C.c_char_p]
    L.cfd_mesh_load.argtypes = [C.c_char_p, C.POINTER(vp)]
    L.cfd_mesh_destroy.argtypes = [vp]
    L.cfd_mesh_destroy.restype = None
    _lib = L
    return L


def build_id() -> str:
    """cfd_build_id(): the source hash the loaded library was built from."""
    return lib().cfd_build_id().decode()


def check(status: int, what: str = "") -> None:
    if status != 0:
        msg = lib().cfd_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed (status {status}): {msg}")
