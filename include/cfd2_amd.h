/*
 * cfd2_amd.h — C ABI of the MI355X-native coupled incompressible-flow step.
 *
 * Drop-in boundary for the reference crate `cfd2` (TSultanov/cfd-demo2).
 * Every solver entry point replaces one method of the reference's
 * `impl GpuSolver` (Rust, src/solver/gpu/solver.rs / init/mod.rs); the Rust
 * extern "C" shim that binds them is in INTEGRATION.md.  Plain pointers and
 * sizes only; no torch types.  Calls are blocking and single-threaded per
 * handle, as in the reference (GpuSolver holds RefCells; GUI wraps it in a
 * Mutex).  Errors are returned as cfd_status (the reference panics instead);
 * cfd_last_error() gives a thread-local message.
 */
#ifndef CFD2_AMD_H
#define CFD2_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum cfd_status {
  CFD_OK = 0,
  CFD_ERR_INVALID = 1,    /* bad argument / inconsistent mesh                    */
  CFD_ERR_HIP = 2,        /* HIP runtime failure (no device, OOM, launch error)  */
  CFD_ERR_DIVERGED = 3,   /* NaN residual: coupled_solver.rs:344-346, 421-426    */
  CFD_ERR_DIAGONAL = 4,   /* "Diagonal not found in CSR cols": init/mesh.rs:210   */
  CFD_ERR_RCCL = 5,       /* collective failure (distributed solver)            */
  CFD_ERR_INTERNAL = 6
} cfd_status;

const char* cfd_last_error(void);
/* Source hash of this build (sha256 prefix over csrc/ and include/, computed by
 * __graft_entry__.source_hash()); no reference counterpart -- it ties every
 * measured number to the code that produced it. */
const char* cfd_build_id(void);

/* ------------------------------------------------------------------------ */
/* Mesh (input format).  Mirrors `Mesh` SoA, src/solver/mesh/structs.rs:12-42.
 * face_neighbor == UINT32_MAX marks a boundary face (Option<usize>::None,
 * init/mesh.rs:63-70); face_boundary: 0 none, 1 inlet, 2 outlet, 3 wall
 * (init/mesh.rs:76-84).  Geometry is f64 and is rounded to f32 on upload
 * exactly like init/mesh.rs:93-155.                                          */
typedef struct cfd_mesh_view {
  uint32_t num_cells;
  uint32_t num_faces;
  const uint32_t* face_owner;        /* [num_faces]     */
  const uint32_t* face_neighbor;     /* [num_faces]     */
  const uint32_t* face_boundary;     /* [num_faces]     */
  const double* face_area;           /* [num_faces]     */
  const double* face_nx;             /* [num_faces]     */
  const double* face_ny;             /* [num_faces]     */
  const double* face_cx;             /* [num_faces]     */
  const double* face_cy;             /* [num_faces]     */
  const double* cell_cx;             /* [num_cells]     */
  const double* cell_cy;             /* [num_cells]     */
  const double* cell_vol;            /* [num_cells]     */
  const uint32_t* cell_face_offsets; /* [num_cells + 1] */
  const uint32_t* cell_faces;        /* [cell_face_offsets[num_cells]] */
} cfd_mesh_view;

/* Geometry of the reference mesher (src/solver/mesh/geometry.rs).           */
typedef struct cfd_geometry {
  int32_t kind;  /* 0 BackwardsStep{length,h_in,h_out,step_x}
                    1 ChannelWithObstacle{length,height,cx,cy,r}
                    2 RectangularChannel{length,height}
                    3 CircleObstacle{cx,cy,r,xmin,ymin,xmax,ymax} (mesh/tests.rs) */
  double p[8];
} cfd_geometry;

typedef struct cfd_mesh cfd_mesh; /* owned host mesh */

/* generate_cut_cell_mesh (src/solver/mesh/cut_cell.rs:10-16)               */
cfd_status cfd_mesh_generate_cut_cell(const cfd_geometry* geo, double min_cell_size,
                                      double max_cell_size, double growth_rate,
                                      double domain_x, double domain_y, cfd_mesh** out);
/* generate_voronoi_mesh (src/solver/mesh/voronoi.rs:23, delaunay.rs): a
 * behavioural restatement with a SEEDED generator (the reference's
 * thread_rng is unseeded): Poisson-disk generators graded like the cut-cell
 * sizing, Bowyer-Watson Delaunay, 20 generator-smoothing sweeps, polygonal
 * dual cells.  Same seed and arguments: the same mesh.  Geometry kinds 0-3. */
cfd_status cfd_mesh_generate_voronoi(const cfd_geometry* geo, double min_cell_size,
                                     double max_cell_size, double growth_rate, double domain_x,
                                     double domain_y, uint64_t seed, cfd_mesh** out);
/* generate_delaunay_mesh (delaunay.rs:732): the same seeded triangulation
 * with the triangles as cells.                                             */
cfd_status cfd_mesh_generate_delaunay(const cfd_geometry* geo, double min_cell_size,
                                      double max_cell_size, double growth_rate, double domain_x,
                                      double domain_y, uint64_t seed, cfd_mesh** out);
/* Mesh::smooth (structs.rs:159-292); returns iterations done in *iters.     */
cfd_status cfd_mesh_smooth(cfd_mesh* m, const cfd_geometry* geo, double target_skew,
                           int32_t max_iterations, int32_t* iters);
/* Mesh::calculate_max_skewness (structs.rs:294-320)                         */
double cfd_mesh_max_skewness(const cfd_mesh* m);
/* Borrowed view of the mesh arrays (valid until the mesh is modified/freed). */
cfd_status cfd_mesh_get_view(const cfd_mesh* m, cfd_mesh_view* out);
/* Vertex arrays (vx, vy, v_fixed) for mesh-validity tests.                  */
cfd_status cfd_mesh_get_vertices(const cfd_mesh* m, uint32_t* num_vertices, const double** vx,
                                 const double** vy, const uint8_t** v_fixed);
/* Vertex topology (structs.rs face_v1/face_v2, cell_vertex_offsets[N+1],
 * cell_vertices: CCW polygon of each cell) for mesh-validity tests.        */
cfd_status cfd_mesh_get_topology(const cfd_mesh* m, const uint32_t** face_v1, const uint32_t** face_v2,
                                 const uint32_t** cell_vertex_offsets, const uint32_t** cell_vertices);
/* Binary SoA dump / load.                              */
cfd_status cfd_mesh_save(const cfd_mesh* m, const char* path);
cfd_status cfd_mesh_load(const char* path, cfd_mesh** out);
void cfd_mesh_destroy(cfd_mesh* m);

/* ------------------------------------------------------------------------ */
/* Constants: same 14-field layout as GpuConstants (structs.rs:86-101).      */
typedef struct cfd_constants {
  float dt;
  float dt_old;
  float time;
  float viscosity;
  float density;
  uint32_t component;
  float alpha_p;
  uint32_t scheme;      /* 0 Upwind, 1 SOU, 2 QUICK (scheme.rs)  */
  float alpha_u;
  uint32_t stride_x;
  uint32_t time_scheme; /* 0 Euler, 1 BDF2                       */
  float inlet_velocity;
  float ramp_time;
  uint32_t precond_type; /* 0 Jacobi, 1 AMG (PreconditionerType) */
} cfd_constants;

/* Build-side configuration (hard-coded numerics of the reference). */
typedef struct cfd_config {
  int32_t n_outer_correctors; /* 20 (init/mod.rs:144)                                  */
  int32_t convergence_lag;    /* 1 = reference async-read model (default), 0 = exact  */
  int32_t fixed_outer;        /* >0: exactly this many Picard iterations, no early exit */
  int32_t fixed_inner;        /* >0: exactly this many FGMRES iterations per solve     */
  int32_t max_restart;        /* 50  (coupled_solver_fgmres.rs:1737)                   */
  int32_t max_outer_restarts; /* 20  (coupled_solver_fgmres.rs:1738)                   */
  float fgmres_rtol;          /* 1e-5                                                   */
  float fgmres_atol;          /* 1e-7                                                   */
  int32_t log_level;          /* 0 silent; 1 the reference's println! progress lines
                                 (coupled_solver.rs, coupled_solver_fgmres.rs) on stderr,
                                 rank 0 only; 2 also AMG setup timings; 3 also a stream
                                 synchronisation + error check after every kernel phase
                                 (debug: a fault is reported where it happened)          */
  int32_t amg_rebuild_interval; /* 0: AMG hierarchy frozen after the first AMG solve
                                   (reference, amg.rs); k > 0: rebuilt from the current
                                   matrix every k steps (opt-in deviation) */
  int32_t amg_local_aggregation; /* distributed solver only.  0 (default): the GLOBAL
                                   hierarchy -- the reference's greedy index-order
                                   aggregation over the whole mesh, aggregates may
                                   straddle ranks, R ranks give one GPU's bits.  1:
                                   partition-aware -- each row-partitioned level is
                                   aggregated over the rank's own rows only (cross-rank
                                   entries ignored by the greedy pass):
                                   block-diagonal P / R, so the restriction and the
                                   prolongation need no halo; the hierarchy (and the
                                   bits) then depend on the rank count, and match the
                                   oracle run with the same rank count and mode       */
  float comm_timeout_s;          /* distributed solver (RCCL and host-staged transports):
                                   progress watchdog.  An operation of the transport still
                                   incomplete after this many seconds, or an asynchronous
                                   RCCL error (ncclCommGetAsyncError), makes a background
                                   thread print the rank, device, operation and category
                                   on stderr, abort the communicator (ncclCommAbort) and
                                   end the process with status 70.  Default 180; <= 0 off.
                                   No reference counterpart (the reference is one GPU).  */
} cfd_config;

void cfd_config_default(cfd_config* cfg);

typedef struct cfd_linear_stats { /* LinearSolverStats, structs.rs:11-18 */
  uint32_t iterations;
  float residual;
  int32_t converged;
  int32_t diverged;
  double time_s;
} cfd_linear_stats;

typedef struct cfd_step_info {
  int32_t should_stop;
  uint32_t degenerate_count;
  uint32_t steady_state_count;
  float outer_residual_u;
  float outer_residual_p;
  uint32_t outer_iterations;
  cfd_linear_stats stats_p; /* the only stats field the reference writes */
  uint32_t total_linear_iterations; /* summed over the step's outer iterations */
} cfd_step_info;

typedef struct cfd_solver cfd_solver;

/* GpuSolver::new (init/mod.rs:15-19).  hip_device selects the GPU.           */
cfd_status cfd_solver_create(const cfd_mesh_view* mesh, const cfd_config* cfg, int32_t hip_device,
                             cfd_solver** out);
void cfd_solver_destroy(cfd_solver* s);

/* solver.rs:9-34: each call overwrites the WHOLE state (other fields = 0).   */
cfd_status cfd_set_u(cfd_solver* s, const double* uv /* [2N] interleaved */);
cfd_status cfd_set_p(cfd_solver* s, const double* p /* [N] */);
/* `constants` public field: host copy; takes effect at update_constants/step */
cfd_status cfd_get_constants(const cfd_solver* s, cfd_constants* out);
cfd_status cfd_set_constants(cfd_solver* s, const cfd_constants* c);
/* setters, solver.rs:36-95 (set_dt keeps the dt_old rule)                    */
cfd_status cfd_set_dt(cfd_solver* s, float dt);
cfd_status cfd_set_viscosity(cfd_solver* s, float nu);
cfd_status cfd_set_alpha_p(cfd_solver* s, float a);
cfd_status cfd_set_alpha_u(cfd_solver* s, float a);
cfd_status cfd_set_density(cfd_solver* s, float rho);
cfd_status cfd_set_scheme(cfd_solver* s, uint32_t scheme);
cfd_status cfd_set_time_scheme(cfd_solver* s, uint32_t scheme);
cfd_status cfd_set_inlet_velocity(cfd_solver* s, float v);
cfd_status cfd_set_ramp_time(cfd_solver* s, float t);
cfd_status cfd_set_precond_type(cfd_solver* s, uint32_t precond_type);
cfd_status cfd_update_constants(cfd_solver* s);
/* solver.rs:276-294                                                          */
cfd_status cfd_initialize_history(cfd_solver* s);
/* solver.rs:242 -> coupled_solver.rs:33-499                                  */
cfd_status cfd_step(cfd_solver* s);
/* Waits until the handle's GPU is idle (hipDeviceSynchronize on its device):
 * the timing fence bench.py puts on both sides of the timed steps.          */
cfd_status cfd_synchronize(cfd_solver* s);
/* solver.rs:97-128 (blocking)                                               */
cfd_status cfd_get_u(cfd_solver* s, double* uv /* [2N] */);
cfd_status cfd_get_p(cfd_solver* s, double* p /* [N] */);
cfd_status cfd_get_d_p(cfd_solver* s, double* dp /* [N] */);
cfd_status cfd_get_step_info(const cfd_solver* s, cfd_step_info* out);
/* The caller-writable part of the step info: the reference's public fields
 * should_stop / degenerate_count / steady_state_count (structs.rs:244-247),
 * which the GUI writes between steps (src/ui/app.rs:852-857: should_stop =
 * false before it resumes) and check_evolution then reads and updates
 * (coupled_solver.rs:553-578).  Distributed solver: call it on every rank
 * with the same values (the counters are global).                          */
cfd_status cfd_set_stop_state(cfd_solver* s, int32_t should_stop, uint32_t degenerate_count,
                              uint32_t steady_state_count);
/* The reference's public field n_outer_correctors (structs.rs:238, 20 from
 * init/mod.rs:144), read by every step_coupled (coupled_solver.rs:111: at
 * least 10 Picard iterations) -- caller-writable between steps like the stop
 * state; cfd_config.n_outer_correctors is its initial value.  n >= 0.       */
cfd_status cfd_set_n_outer_correctors(cfd_solver* s, int32_t n);
uint32_t cfd_num_cells(const cfd_solver* s);
uint32_t cfd_num_faces(const cfd_solver* s);

/* ------------------------------------------------------------------------ */
/* Checkpoint / resume (the reference keeps its state only in GPU
 * buffers, get_u/get_p being its only export).  The file holds everything a
 * step reads from earlier steps, in f32 exactly as the device holds it, so a
 * solver that loads it steps bit-identically to the one that saved it:
 *   header (cfd_state_file_header, 512 bytes), then GLOBAL per-cell arrays
 *   (cell order of the mesh, independent of the rank count):
 *   ring slot 0, 1, 2: u f32[2N] (interleaved), p f32[N], d_p f32[N],
 *                      grad_p f32[2N]                (FluidState x3, structs.rs)
 *   prev (check_evolution snapshot): the same four arrays
 *   x f32[3N]  (FGMRES solution = initial guess of the next solve)
 *   if amg_nnz > 0: amg_rowptr u64[N+1], amg_val f32[amg_nnz] -- the scalar
 *   pressure matrix the AMG hierarchy was built from (CSR, columns ascending;
 *   the pattern is the mesh's), so the loader rebuilds the same hierarchy --
 *   under the LOADER's aggregation mode and rank count: the default (global)
 *   hierarchy is rank-count independent; a partition-aware one
 *   (amg_local_aggregation = 1) depends on the rank count, so a file saved
 *   in that mode continues bit-identically only on the same rank count and
 *   mode.  The loader prints a warning on stderr when they differ.          */
typedef struct cfd_state_file_header {
  char magic[8];        /* "CFD2STAT" */
  uint32_t version;     /* 1 */
  uint32_t header_bytes; /* 512 */
  uint64_t num_cells;
  uint64_t num_faces;
  uint64_t amg_nnz;     /* 0: no AMG hierarchy built when saved */
  int32_t step_index;   /* ring rotation (coupled_solver.rs:43-71) */
  int32_t have_prev;
  int32_t inner_has_last; /* FGMRES lagged residual read (async_buffer.rs) */
  float inner_last;
  uint32_t n_variance;  /* entries of variance[] in use (<= 10), oldest first */
  uint32_t reserved0;
  double variance[10][2]; /* check_evolution's (var_u, var_v) history */
  cfd_constants constants;
  cfd_step_info info;
  uint32_t amg_age;     /* steps since the hierarchy was built (amg_rebuild_interval) */
  int32_t amg_local_aggregation; /* cfd_config.amg_local_aggregation of the saving run */
  int32_t nranks;       /* rank count of the saving run (0: not recorded)             */
  uint8_t reserved[164];
} cfd_state_file_header;

/* Writes the state to `path`.  Distributed solver: COLLECTIVE, every rank
 * writes its owned cells into the same file (one node: one filesystem).    */
cfd_status cfd_state_save(cfd_solver* s, const char* path);
/* Replaces the state with the file's (not collective: a distributed rank
 * reads its owned cells and ghosts).  The file may come from any rank
 * count.  The solver's own AMG hierarchy, if built, is dropped; the saved
 * scalar matrix, if any, is what the next AMG solve rebuilds it from.      */
cfd_status cfd_state_load(cfd_solver* s, const char* path);
/* In-process group: cfd_state_save on every rank (one host thread each).   */
cfd_status cfd_group_state_save(cfd_solver* const* handles, int32_t nranks, const char* path);

/* ------------------------------------------------------------------------ */
/* Instrumentation (replaces profiling.rs): HIP-event timing of the level-0
 * AMG smoother sweep, on the solver's own stream.                            */
cfd_status cfd_profile_enable(cfd_solver* s, int32_t enable);
cfd_status cfd_profile_reset(cfd_solver* s);
/* total_ms / launches over the level-0 smoother sweeps since
 * cfd_profile_reset (every sweep timed while profiling is on); bytes =
 * algorithmic bytes per sweep (4(n+1) + 8 nnz + 12 n).       */
cfd_status cfd_profile_smoother(const cfd_solver* s, double* total_ms, uint64_t* launches,
                                double* bytes_per_launch);
/* hipGraph replay of the FGMRES iteration (one executable graph per basis
 * index, captured on first use, replayed by every later solve; DESIGN.md
 * section 5).  enable: 1 on, 0 off (the launches are issued one by one);
 * default off: replay measured no faster than
 * eager launches.  One GPU only.  Same bits either
 * way.  Stats: graphs captured and iterations replayed so far.             */
cfd_status cfd_graph_enable(cfd_solver* s, int32_t enable);
cfd_status cfd_graph_stats(const cfd_solver* s, int32_t* enabled, uint64_t* captures, uint64_t* replays);
/* AMG hierarchy summary: number of levels and rows/nnz per level.            */
cfd_status cfd_amg_levels(const cfd_solver* s, int32_t* num_levels, uint32_t* rows /*[20]*/,
                          uint64_t* nnz /*[20]*/);
/* AMG setup path taken (0 not built yet, 1 host, 2 device; SURVEY §8(f)
 * rank 3) and an FNV-1a digest of every byte of level `level`'s device image
 * (matrix, diagonal, P, R) -- host and device setups must agree bit-for-bit.
 * Debug/parity only; not part of the reference surface.                     */
cfd_status cfd_debug_amg_info(cfd_solver* s, int32_t level, int32_t* setup_path, uint64_t* digest);
/* Layout-true bytes of one level-0 smoother sweep: the minimum the kernel
 * moves in this library's level image (u8 lengths, ELL values + 16/32-bit
 * columns, b, x, diagonal, x_out); the roofline of record divides this by
 * the measured sweep time (cfd_profile_smoother's bytes are the reference
 * CSR format's count).                                        */
double cfd_smoother_layout_bytes(const cfd_solver* s);
/* Layout-true bytes of one step under the fixed schedule: every kernel's
 * minimum traffic in this library's layouts (a lower bound of the HBM bytes,
 * unlike the reference-format count below) times its launches per step.    */
double cfd_step_layout_bytes(const cfd_solver* s);
/* Algorithmic bytes of one step under the fixed schedule in the reference's
 * CSR/f32/u32 format -- a count, larger than this layout's
 * traffic.                                                                  */
double cfd_step_algorithmic_bytes(const cfd_solver* s);

/* Debug/parity access to internal device buffers, copied to host.
 * ids: 0 fluxes-by-face[F], 1 grad_u[2N], 2 grad_v[2N], 3 rhs[3N], 4 x[3N],
 * 5 diag_u_inv[N], 6 diag_v_inv[N], 7 diag_p_inv[N], 8 scalar_matrix[nnz_s],
 * 9 coupled_matrix_csr[9 nnz_s] (reference CSR order), 10 grad_p[2N],
 * 11 state_old u[2N], 12 state_old_old u[2N]                                 */
cfd_status cfd_debug_buffer(cfd_solver* s, int32_t id, float* out, size_t count);
size_t cfd_debug_buffer_len(const cfd_solver* s, int32_t id);
/* Runs only prepare_coupled (+ coupled_assembly_merged when assemble != 0) on
 * the current state without rotating the ring (kernel-level parity).        */
cfd_status cfd_debug_prepare_assemble(cfd_solver* s, int32_t assemble);
/* Test mode: the reference's own semantics under a legal schedule instead of
 * the canonical resolutions, with the oracle's flag bits
 * (oracle_set_semantics): 4 the reference's reduction order -- 64-DOF
 * workgroup trees, then reduce_final's serial sum (norms, gmres_ops.wgsl:
 * 241-293) or reduce_dots_cgs's strided lanes + tree (CGS, gmres_cgs.wgsl:
 * 86-120), and check_evolution's serial f64 loops (coupled_solver.rs:504-545)
 * on the host; 1 the in-place AMG smoother (amg.wgsl:24-50) with its 64-row
 * workgroups run in order; 2 prepare_coupled's racy neighbour reads
 * (prepare_coupled.wgsl:140-143 vs :328-337), its 64-cell workgroups in order,
 * the assembly reading each face's flux as its owner stored it; 8
 * restrict_residual's out-of-bounds rows (amg.rs:707-719) under wgpu's
 * Restrict policy.  Flags 4 give the bits of the reference's WGSL kernels run
 * with the whole dispatch resident, 13 those with the V-cycle's workgroups in
 * order, 15 those with every dispatch's workgroups in order
 * (tests/test_gpu_wgsl_pin.py).  Other bits, or a distributed handle:
 * CFD_ERR_INVALID.  Slow (serial sums / workgroups); drops captured graphs;
 * 0 = canonical.                                                            */
cfd_status cfd_debug_reference_semantics(cfd_solver* s, int32_t flags);

/* ------------------------------------------------------------------------ */
/* Multi-GPU (the reference is single-GPU).  The mesh is split
 * into R contiguous cell ranges (x-major cut-cell numbering => vertical
 * slabs), rank r owning [floor(N r/R), floor(N (r+1)/R)).  Ghost-cell halos
 * of the state, the Krylov vectors and every distributed AMG level go to the
 * slab neighbours; reductions all-gather per-rank partial sums and add them
 * in rank order (deterministic, identical on every rank).  For a distributed
 * handle: `mesh` is the WHOLE mesh on every rank; cfd_set_u/cfd_set_p take
 * the global arrays; cfd_num_cells and cfd_get_u/p/d_p cover the owned cells.
 *
 * One process per GPU over RCCL (the production path): rank 0 calls
 * cfd_dist_unique_id and broadcasts the 128 bytes (e.g. torch.distributed);
 * every rank then calls cfd_solver_create_dist (collective) and steps with
 * cfd_step (collective).                                                    */
cfd_status cfd_dist_unique_id(uint8_t out[128]);
cfd_status cfd_solver_create_dist(const cfd_mesh_view* mesh, const cfd_config* cfg,
                                  int32_t hip_device, int32_t nranks, int32_t rank,
                                  const uint8_t unique_id[128], cfd_solver** out);
/* Host-staged transport (test / rehearsal mode, e.g. several processes on
 * ONE GPU, where RCCL refuses a second rank per device): the same
 * distributed solver, with every halo exchange and all-gather staged through
 * host memory and handed to caller callbacks (bench.py binds them to
 * torch.distributed's gloo backend).  exchange: transfers with the same peer
 * match in list order, send k of one rank with receive k of the other;
 * allgather: recv[r * bytes ...] = rank r's send.  Callbacks return 0 on
 * success.  Not a performance path.                                          */
typedef int32_t (*cfd_exchange_fn)(void* user, int32_t n, const int32_t* peer, void* const* send,
                                   const uint64_t* send_bytes, void* const* recv, const uint64_t* recv_bytes);
typedef int32_t (*cfd_allgather_fn)(void* user, void* send, void* recv, uint64_t bytes);
cfd_status cfd_solver_create_dist_host(const cfd_mesh_view* mesh, const cfd_config* cfg, int32_t hip_device,
                                       int32_t nranks, int32_t rank, cfd_exchange_fn exchange,
                                       cfd_allgather_fn allgather, void* user, cfd_solver** out);
/* In-process group (SURVEY §8(b) `cfd_solver_create_dist(..., nranks,
 * devices)`): nranks handles in this process, rank r on devices[r] (devices
 * may repeat: all ranks on one GPU is allowed).  Collective calls go through
 * cfd_group_step / cfd_group_debug_prepare_assemble (one host thread per rank). */
cfd_status cfd_group_create(const cfd_mesh_view* mesh, const cfd_config* cfg, int32_t nranks,
                            const int32_t* devices, cfd_solver** out /* [nranks] */);
cfd_status cfd_group_step(cfd_solver* const* handles, int32_t nranks);
/* A cfd_group_step that failed on any rank leaves the ranks at different
 * points of the step, so the group is marked "needs restore": further
 * cfd_group_step calls return CFD_ERR_INVALID until every rank has loaded a
 * consistent state (cfd_state_load, per rank) or the caller accepts the state
 * as is (cfd_group_reset).  cfd_group_needs_restore: 1 while marked.       */
cfd_status cfd_group_reset(cfd_solver* const* handles, int32_t nranks);
int32_t cfd_group_needs_restore(cfd_solver* const* handles, int32_t nranks);
/* RCCL plumbing check on one GPU: 1-rank communicator, grouped send/recv to
 * self and an all-gather through the solver's transport; CFD_OK if the data
 * arrived intact.                                                           */
cfd_status cfd_debug_rccl_selftest(int32_t hip_device);
/* Progress-watchdog self-test, no GPU needed: a watchdog with limit
 * `timeout_s` around a host-blocking operation that takes `hang_ms`.  If
 * hang_ms exceeds the limit, the watchdog ends the PROCESS with status 70
 * (as on a stalled collective; run it in a child process); else CFD_OK.    */
cfd_status cfd_debug_comm_watchdog(float timeout_s, int32_t hang_ms);
/* Transport of a distributed handle and its traffic since the last reset
 * (bench.py prints these on a --gpus N line).                               */
typedef struct {
  int32_t transport;        /* 0 none (one rank), 1 RCCL, 2 in-process group, 3 host-staged */
  int32_t comm_count;       /* RCCL: ncclCommCount; otherwise the rank count */
  int32_t comm_rank;        /* RCCL: ncclCommUserRank; otherwise the rank */
  int32_t device;           /* HIP device of this rank */
  uint64_t exchanges;       /* grouped point-to-point calls (halos) */
  uint64_t allgathers;      /* all-gather calls (reductions, replicated AMG levels) */
  uint64_t bytes_sent;      /* point-to-point payload bytes this rank sent */
  uint64_t bytes_gathered;  /* all-gather payload bytes this rank contributed */
} cfd_comm_stats;
cfd_status cfd_dist_comm_stats(cfd_solver* s, cfd_comm_stats* out, int32_t reset);
/* Timing of the distributed communication by category (measurement aid for
 * the multi-GPU runs; no reference counterpart).  While enabled, every halo
 * exchange and all-gather is bracketed by timing events (a small cost:
 * bench.py times its headline steps with it off, then one extra step with it
 * on).  category: 0 Krylov halos (V_j, p_sol, Z_j, x), 1 state / assembly
 * halos, 2 reduction all-gathers (dots, norms, max-diff), 3 the all-gather of
 * the first replicated AMG level's rhs, 4 AMG level halos (`level` = the AMG
 * level).  wait_us: time the compute stream stood still for the operation
 * (halos: from reaching the wait on the exchange to its release; all-gathers
 * run on the compute stream: their whole duration); comm_us: the
 * transport's own time (halos: the grouped send/recv on the comm stream,
 * peer waits included).  enable resets the totals.                         */
typedef struct {
  int32_t category;
  int32_t level;    /* AMG level (category 4), else -1 */
  uint64_t calls;
  uint64_t bytes;   /* payload this rank sent / contributed */
  double wait_us;
  double comm_us;
} cfd_comm_timing_entry;
cfd_status cfd_comm_timing_enable(cfd_solver* s, int32_t enable);
/* the non-empty categories, at most `cap`; *count = how many were written  */
cfd_status cfd_comm_timing(cfd_solver* s, cfd_comm_timing_entry* out, int32_t cap, int32_t* count);
/* In-process group failure path (test hook): every rank enters a collective
 * except `fail_rank`, which fails first; the others must return an error
 * instead of waiting forever, and the group must stay usable afterwards.     */
cfd_status cfd_debug_group_fault(cfd_solver* const* handles, int32_t nranks, int32_t fail_rank);
/* ... and a failure in the middle of a step: `fail_rank` throws right after
 * the step's first prepare() while the other ranks continue until their next
 * collective; the group is then marked needs-restore (see cfd_group_reset). */
cfd_status cfd_debug_group_fault_midstep(cfd_solver* const* handles, int32_t nranks, int32_t fail_rank);
/* rank, rank count, owned global range [c0, c1), global cell count         */
cfd_status cfd_dist_info(const cfd_solver* s, int32_t* rank, int32_t* nranks, uint32_t* c0,
                         uint32_t* c1, uint32_t* num_global_cells);
/* Host-only halo plan of rank `rank` (no GPU needed; for tests / tooling).
 * First call with null arrays to get the sizes.  ghost_global: ghost cell ids
 * (ascending); per peer: peer rank, recv count, send count; send_global: the
 * owned cell ids sent to each peer, concatenated in peer order.            */
cfd_status cfd_dist_plan(const cfd_mesh_view* mesh, int32_t nranks, int32_t rank, uint32_t* c0,
                         uint32_t* c1, uint32_t* num_ghosts, uint32_t* num_peers,
                         uint32_t* num_send, uint32_t* ghost_global, int32_t* peer_rank,
                         uint32_t* peer_recv, uint32_t* peer_send, uint32_t* send_global);

#ifdef __cplusplus
}
#endif
#endif /* CFD2_AMD_H */
