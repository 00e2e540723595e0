/*
 * CPU oracle for the coupled-step hot path — TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library, and only as the checker / reported CPU baseline.  The
 * product (cfd-demo2_amd/) never links or calls it.
 *
 * Parity pinned to the reference's own kernels (round 6): the reference's
 * WGSL shaders, executed on the CPU from its source (oracle/wgsl/, driven by
 * tests/wgsl_ref.py; fixtures tests/golden/wgsl_ref.npz), reproduce this
 * oracle bit for bit with reference-semantics flags 15 (workgroups in order,
 * Restrict policy) and 4 (whole dispatch resident, ReadZeroSkipWrite); the
 * canonical mode (flags 0, what the HIP path reproduces) differs from the
 * latter only by its reduction tree.  The Rust host sequence (dispatch order,
 * AMG setup, readbacks) is restated, not executed: the reference program
 * itself (Rust + wgpu) cannot be built here.
 */
#ifndef CFD2_ORACLE_H
#define CFD2_ORACLE_H
#include "../include/cfd2_amd.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_solver oracle_solver;

oracle_solver* oracle_create(const cfd_mesh_view* mesh, const cfd_config* cfg);
/* Kept for the distributed tests: the distributed solver is rank-count
 * invariant (global AMG hierarchy, canonical reduction tree whose segments
 * ranks own whole), so `nranks` changes no result; = oracle_create.       */
oracle_solver* oracle_create_dist(const cfd_mesh_view* mesh, const cfd_config* cfg, int nranks);
/* Reference-semantics sensitivity mode: bit flags replacing the canonical
 * deterministic resolutions of SURVEY §0.1 by the reference's behaviour under
 * one plausible schedule: 1 in-place AMG smoother (64-row workgroups in
 * order), 2 racy prepare_coupled reads (workgroups in order), 4 the
 * reference's reduction order (64-wide trees + serial / strided finals, serial
 * f64 check_evolution), 8 restrict_residual's out-of-bounds rows under wgpu's
 * Restrict policy (last coarse entry zeroed when n_c % 64 != 0), 16 flags 1
 * and 2 with the workgroups run last-to-first (a second plausible schedule).
 * 0 = canonical (what the HIP path reproduces).                              */
int oracle_set_semantics(oracle_solver* s, int flags);
void oracle_destroy(oracle_solver* s);
void oracle_set_threads(int n);
int oracle_set_u(oracle_solver* s, const double* uv);
int oracle_set_p(oracle_solver* s, const double* p);
int oracle_get_constants(const oracle_solver* s, cfd_constants* c);
int oracle_set_constants(oracle_solver* s, const cfd_constants* c);
int oracle_set_dt(oracle_solver* s, float dt);
int oracle_initialize_history(oracle_solver* s);
int oracle_step(oracle_solver* s);
int oracle_get_u(oracle_solver* s, double* uv);
int oracle_get_p(oracle_solver* s, double* p);
int oracle_get_d_p(oracle_solver* s, double* dp);
int oracle_get_step_info(const oracle_solver* s, cfd_step_info* out);
int oracle_set_stop_state(oracle_solver* s, int should_stop, uint32_t degenerate_count,
                          uint32_t steady_state_count);
int oracle_set_n_outer_correctors(oracle_solver* s, int n);
/* same buffer ids as cfd_debug_buffer */
size_t oracle_debug_buffer_len(const oracle_solver* s, int id);
int oracle_debug_buffer(oracle_solver* s, int id, float* out, size_t count);
int oracle_debug_prepare_assemble(oracle_solver* s, int assemble);
int oracle_amg_levels(const oracle_solver* s, int* num_levels, uint32_t* rows, uint64_t* nnz);
const char* oracle_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
