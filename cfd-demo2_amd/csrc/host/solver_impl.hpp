// Host-side driver state of the HIP solver (one instance per GPU handle).
#pragma once
#include <hip/hip_runtime_api.h>
#include <rocprofiler-sdk-roctx/roctx.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <stdexcept>
#include <string>
#include <vector>

#include <memory>

#include "../../../include/cfd2_amd.h"
#include "../hip/amg_setup.hpp"
#include "../hip/kernels.hpp"
#include "comm.hpp"
#include "dist.hpp"
#include "tuning.hpp"

namespace cfd2 {

struct HipError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

#define CFD_HIP(expr)                                                                   \
  do {                                                                                  \
    hipError_t _e = (expr);                                                             \
    if (_e != hipSuccess)                                                               \
      throw ::cfd2::HipError(std::string(#expr) + ": " + hipGetErrorString(_e));        \
  } while (0)

// Device allocation arena: every buffer is freed with the solver.
class DeviceArena {
 public:
  ~DeviceArena() { release(); }
  template <class T>
  T* alloc(size_t n) {
    void* p = nullptr;
    const size_t bytes = (n ? n : 1) * sizeof(T);
    CFD_HIP(hipMalloc(&p, bytes));
    ptrs_.push_back(p);
    bytes_ += bytes;
    return static_cast<T*>(p);
  }
  template <class T>
  T* upload(const std::vector<T>& v, hipStream_t s, size_t slack = 0) {
    // slack: zeroed elements after the data (16-byte vector reads that start
    // at any valid index, e.g. the fused prolongation's agg gathers)
    T* p = alloc<T>(v.size() + slack);
    if (slack) CFD_HIP(hipMemsetAsync(p + v.size(), 0, slack * sizeof(T), s));
    if (!v.empty()) CFD_HIP(hipMemcpyAsync(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, s));
    return p;
  }
  void swap(DeviceArena& o) {
    ptrs_.swap(o.ptrs_);
    std::swap(bytes_, o.bytes_);
  }
  void release() {
    for (void* p : ptrs_) (void)hipFree(p);
    ptrs_.clear();
    bytes_ = 0;
  }
  size_t bytes() const { return bytes_; }

 private:
  std::vector<void*> ptrs_;
  size_t bytes_ = 0;
};

// roctx range (rocprofv3 --marker-trace shows steps, Picard iterations,
// FGMRES solves and iterations, AMG setup / refresh, checkpoint I/O)
struct Range {
  explicit Range(const char* what) { roctxRangePushA(what); }
  ~Range() { roctxRangePop(); }
  Range(const Range&) = delete;
  Range& operator=(const Range&) = delete;
};

struct HostCsr {
  std::vector<uint32_t> row, col;
  std::vector<float> val;
  size_t rows = 0, cols = 0;
};

// Mesh-derived static topology/geometry (init/mesh.rs + the per-slot geometric
// factors every face sweep needs), computed once on the host in f32 with the
// exact operation order of the WGSL expressions they replace.
struct Topology {
  uint32_t N = 0, F = 0;  // N = owned cells
  // distributed view (one GPU: c0 = 0, c1 = NG, no ghosts)
  uint32_t NG = 0, c0 = 0, c1 = 0;
  uint32_t npad = 0;           // N rounded up to 64: first upper-ghost local index
  uint32_t glo = 0, ghi = 0;   // ghosts below c0 / at or above c1
  std::vector<uint32_t> ghost; // ghost global ids, ascending
  // signed local index of a global cell id (owned or ghost)
  int32_t rel(uint32_t g) const {
    if (g >= c0 && g < c1) return (int32_t)(g - c0);
    const auto it = std::lower_bound(ghost.begin(), ghost.end(), g);
    if (it == ghost.end() || *it != g) throw std::logic_error("cell is neither owned nor a ghost");
    const uint32_t k = (uint32_t)(it - ghost.begin());
    return k < glo ? (int32_t)k - (int32_t)glo : (int32_t)(npad + (k - glo));
  }
  int wf = 0;  // max faces per cell
  int ws = 0;  // max scalar row length (incl. diagonal)
  std::vector<float> vol;
  std::vector<uint32_t> nface;
  // face slots, [k*N + i]
  std::vector<int32_t> fs_other;
  std::vector<uint32_t> fs_meta;
  std::vector<uint32_t> fs_face;  // host only: face index of each slot
  std::vector<float> fs_area, fs_nx, fs_ny, fs_lam_s, fs_lam_f, fs_dist_a, fs_dist_e, fs_dvx,
      fs_dvy, fs_rx, fs_ry, fs_rox, fs_roy;
  // scalar CSR rows of the owned cells (init/mesh.rs:27-53), global columns,
  // and its ELL image [r*N + i] with signed local columns
  std::vector<uint32_t> srow, scol;
  uint32_t ld = 0;               // ELL slot stride (= npad)
  std::vector<int32_t> ell_col;  // [r*ld + i]
  std::vector<uint32_t> ell_len, ell_drank;  // [ld]
  bool use16 = false;            // every |col - row| < 2^15: ell_col16 valid
  std::vector<int16_t> ell_col16;
  std::vector<uint8_t> ell_len8, ell_drank8;
  // Coupled-matrix ELL (CoupledMatrix, kernels.hpp): the same rows with their
  // entries moved to aligned slots.  tmode[r] = the most frequent column - row
  // of slot r over the full rows; a row with fewer entries places each entry,
  // in CSR order, at the first slot still free whose mode is its delta, so
  // missing neighbours (walls) leave gaps instead of shifting the rest of the
  // row, and 4 consecutive rows keep 4 consecutive columns per slot.  Gaps and
  // trailing slots hold the virtual column row + tmode[r] (clamped into the
  // vectors' range; never accumulated).  Position layout when ws > 8 (the
  // Voronoi meshes).
  std::vector<int32_t> tmode;
  std::vector<uint8_t> tslot;    // [nnz] slot of CSR entry k
  std::vector<int32_t> tcol;     // [r*ld + i]
  std::vector<int16_t> tcol16;   // (use16)
  std::vector<uint16_t> tlg;     // [ld] slots in use | gap mask << 8
  std::vector<uint8_t> tdrank8;  // [ld] slot of the diagonal
};

// Throws std::invalid_argument on inconsistent meshes.
void build_topology(const cfd_mesh_view& m, Topology& t);
// Owned range [c0, c1) of a distributed rank, ghosts from the face neighbours.
void build_topology(const cfd_mesh_view& m, Topology& t, uint32_t c0, uint32_t c1);

// AMG hierarchy (linear_solver/amg.rs:84-235, 374-595) built on the host.
struct AmgHostLevel {
  HostCsr A;
  std::vector<uint32_t> agg;         // P (fine -> coarse), when has_op
  std::vector<uint32_t> r_row, r_col;  // R = P^T
  uint32_t nc = 0;
  bool has_op = false;
  std::vector<uint64_t> part;  // row partition starts of this level (one entry per rank + 1)
};
// local: partition-aware aggregation of the row-partitioned levels (those of
// more than rep_rows rows from level 0 on; cfd_config.amg_local_aggregation)
// timing: per-level SpGEMM times on stderr (cfg.log_level >= 2)
std::vector<AmgHostLevel> build_amg_hierarchy(const HostCsr& fine, size_t max_levels,
                                               const std::vector<uint64_t>& part = {}, bool local = false,
                                               uint64_t rep_rows = 0, bool timing = false);
// Block partition of a down-leg level pair (k_amg_resrestrict_pair,
// kernels.hpp AmgPairImage).  fr_row / fr_col: R of level i (its aggregates
// are the level-(i+1) rows); mr_row / mr_col: R of level i+1; mrow / mcol:
// the off-diagonal pattern of level i+1 (CSR, entries in the level image's
// slot order).  Each block takes consecutive level-(i+2) aggregates while its
// S rows (their members, then the ring of the members' columns) and those
// rows' level-i members each stay <= cap and its aggregates <= cap.  lc[k]:
// the block-local index (in S) of entry k of mcol, for the rows the block owns.
// False when one aggregate alone exceeds cap.
struct PairPartition {
  std::vector<uint32_t> jb, sb, s, fo, f;
  std::vector<uint16_t> lc;
};
bool build_pair_partition(const std::vector<uint32_t>& fr_row, const std::vector<uint32_t>& fr_col,
                          const std::vector<uint32_t>& mr_row, const std::vector<uint32_t>& mr_col,
                          const std::vector<uint32_t>& mrow, const std::vector<uint32_t>& mcol, uint32_t cap,
                          PairPartition& out);
// Block partition of an up-leg level pair (k_amg_prolong_smooth_pair,
// kernels.hpp AmgUpPairImage): blocks of `rows` consecutive fine rows; each
// block's T = the coarse rows its fine rows and their columns aggregate into
// (ascending).  frow / fcol: the fine level's off-diagonal pattern (CSR, slot
// order); agg: fine -> coarse.  lt[k]: T-local index of agg[fcol[k]] for
// entry k, lto[f]: of agg[f].  False when a block's T exceeds cap.
struct UpPairPartition {
  std::vector<uint32_t> tb, t;
  std::vector<uint16_t> lt, lto;
};
bool build_up_pair_partition(const std::vector<uint32_t>& frow, const std::vector<uint32_t>& fcol,
                             const std::vector<uint32_t>& agg, uint32_t nc, uint32_t rows, uint32_t cap,
                             UpPairPartition& out);
// Greedy index-order aggregation (amg.rs:84-116) of the pattern (row, col) of
// n rows; returns the aggregate count, agg[i] = aggregate of row i, and
// cpart = the aggregate partition induced by the row partition `part` (an
// aggregate belongs to the part of its seed, its smallest row).  local: a
// seed takes only neighbours of its own part (no aggregate straddles parts).
uint32_t aggregate_greedy(size_t n, const uint32_t* row, const uint32_t* col, const std::vector<uint64_t>& part,
                          std::vector<uint32_t>& agg, std::vector<uint64_t>& cpart, bool local = false);
// R = P^T of piecewise-constant P: rows = aggregates, fine indices ascending
void transpose_aggregates(const std::vector<uint32_t>& agg, uint32_t nagg, std::vector<uint32_t>& r_row,
                          std::vector<uint32_t>& r_col);

struct AmgGpuLevel {
  AmgLevelDev dev{};
  float* x = nullptr;   // level solution (level 0: external p_sol); owned base
  float* xt = nullptr;  // ping-pong partner for the out-of-place smoother
  bool wide = false;    // rows wider than the u8 layout: 16-bit lengths, tail kernels only
  float* b = nullptr;   // level rhs (level 0: external temp_p)
  float* r = nullptr;   // residual scratch
  uint64_t nnz = 0;     // including diagonal (rows this rank stores)
  uint64_t nglob = 0;   // rows of the whole level
  // distributed level: owned rows [C0, C1) of the global level, ghosts around
  bool dist = false;
  HaloPlan plan;
  uint32_t glo = 0, ghi = 0, npad = 0;
  // this rank's rows of the level (replicated level: restriction target range)
  uint64_t C0 = 0, C1 = 0;
  // distributed level: its aggregates [0, rc_hi) have only owned members (their
  // restriction overlaps the residual halo); fine rows [pf_lo, n) belong to
  // owned aggregates (their prolongation overlaps the coarse-x halo)
  uint32_t rc_hi = 0, pf_lo = 0;
  std::vector<uint64_t> part;  // row partition of the level over the ranks
};

struct LagReader {  // async_buffer.rs restated as a deterministic lag model
  bool has_last = false;
  float last = 0.0f;
  int pending = -1;
};

struct AmgSetupLevel;  // amg_device.cpp

// Distributed runs replicate the AMG levels with at most this many GLOBAL rows
// on every rank (CFD_AMG_REPLICATE_ROWS overrides).  DESIGN §7 "Latency
// budget": below ~1 M rows a replicated level's redundant kernels plus one
// all-gather of its rhs cost less than the four un-overlapped halos per
// V-cycle that keeping it row-partitioned costs (C4: level 4, 650 k rows).
constexpr uint64_t kAmgReplicateRowsDefault = 1u << 20;
inline uint64_t amg_replicate_rows() { return knob_u64(Knob::AmgReplicateRows, kAmgReplicateRowsDefault); }

struct Solver {
  cfd_config cfg{};
  int device = 0;
  hipStream_t stream = nullptr;
  DeviceArena arena;
  Topology topo;
  uint32_t N = 0, F = 0;  // N: cells this rank owns
  // ---- distribution (one GPU: R = 1, no comm, no ghosts) ----
  std::unique_ptr<Comm> comm;
  int R = 1, rk = 0;
  std::vector<uint64_t> starts;  // cell partition (R + 1)
  uint32_t NG = 0;               // cells of the whole mesh
  uint32_t shift = 0;            // owned base offset of every per-cell vector (>= glo, 64-aligned)
  size_t vlen = 0;               // elements per component of a per-cell vector
  HaloPlan cell_plan;
  uint64_t* d_u64 = nullptr;     // [R + 1] all-gather scratch of allgather_u64
  // canonical reductions (kernels.hpp): geometry of the global tree; a
  // distributed rank all-gathers its segment values ([v][local segment],
  // maxseg slots per vector) and every rank finishes the same tree
  RedGeom red;
  uint32_t maxseg = 0;           // most segments any rank owns
  uint32_t* d_seg_src = nullptr; // [nseg] (owner << 20) | local segment
  float* red_local = nullptr;    // [m1 * maxseg]
  float* red_gather = nullptr;   // [R * m1 * maxseg]
  double* red_local_d = nullptr; // [5 * maxseg] check_evolution
  double* red_gather_d = nullptr;
  uint32_t* mx_gather = nullptr; // [2R]
  StateView evrec{};             // check_evolution records fetched from their owners
  uint64_t ev_a = 0, ev_b = 0;   // record range [ev_a, ev_b) this rank's variance reads
  int amg_g = 0;                 // first replicated AMG level (distributed)
  // partition-aware hierarchy (cfg.amg_local_aggregation on a distributed
  // solver): the distributed levels' aggregates never straddle ranks, so the
  // restriction and the prolongation of those levels need no halo
  bool amg_local = false;
  int m = 50, m1 = 51;
  uint32_t nchunks = 0;

  // static device data
  FaceSlots fs{};
  float* d_vol = nullptr;
  int32_t* d_scol = nullptr;
  int16_t* d_scol16 = nullptr;
  uint8_t* d_slen8 = nullptr;
  uint8_t* d_sdrank8 = nullptr;
  int32_t* d_tcol = nullptr;      // coupled-matrix ELL (Topology::tslot)
  int16_t* d_tcol16 = nullptr;
  uint16_t* d_tlg = nullptr;
  uint8_t* d_tdrank8 = nullptr;
  uint32_t* d_slen = nullptr;
  uint32_t* d_sdrank = nullptr;
  // ring of 3 FluidState slots (SoA) + prepare's d_p / grad_p scratch
  StateView ring[3]{};
  float* dp_scratch = nullptr;
  float2* gp_scratch = nullptr;
  int step_index = 0, i_state = 0, i_old = 1, i_old_old = 2;
  // prev view for check_evolution
  StateView prev{};
  bool have_prev = false;
  // face-slot fluxes, gradients, matrices
  float* flux_s = nullptr;
  float2* grad_u = nullptr;
  float2* grad_v = nullptr;
  float2* cval_a = nullptr;
  float2* cval_g = nullptr;
  float2* cdiag2 = nullptr;
  float* sval = nullptr;
  float* rhs = nullptr;
  float* x = nullptr;
  float* dinv_uv = nullptr;
  float* dinv_p = nullptr;
  // FGMRES
  bool fgmres_ready = false;
  float* basis = nullptr;
  size_t stride = 0;
  float* zvec = nullptr;
  float* w = nullptr;
  float* temp = nullptr;
  float* temp_p = nullptr;
  float* p_sol = nullptr;
  uint32_t nunits = 0;           // unit partials (red.U chunks each) of this rank's cells
  uint32_t pstride = 0;          // unit partials per vector (nunits rounded up to 4: 16-byte loads)
  float* partial = nullptr;      // [(m+1) * pstride] chunk partials (256 cells each)
  float* partial_n = nullptr;    // [nchunks]
  // reference semantics (test mode, cfd_debug_reference_semantics; the
  // oracle's kSem* bits, one GPU only -- the bits of the reference's own
  // kernels under a legal schedule, tests/test_gpu_wgsl_pin.py):
  // ref_red (4) the reference's 64-DOF group partials and finishing orders
  // (ref_racy, flag 2, below)
  // instead of the canonical tree; ref_inplace (1) the in-place AMG smoother,
  // 64-row workgroups in order; ref_clamp (8) restrict_residual's
  // out-of-bounds rows under wgpu's Restrict policy (the last coarse rhs
  // entry zeroed when n_c % 64 != 0).  1 / 8 run v_cycle_reference().
  bool ref_red = false;
  bool ref_inplace = false;
  bool ref_clamp = false;
  // ref_racy (2): the racy prepare, 64-cell workgroups in order, in place;
  // d_flux_mirror[e]: the owner's slot of non-owner face slot e (else -1)
  bool ref_racy = false;
  int32_t* d_flux_mirror = nullptr;
  void v_cycle_reference();
  uint32_t ref_ng = 0;           // ceil(3N / 64) groups
  float* ref_part = nullptr;     // [(m+1) * ref_ng] CGS dot group partials
  float* ref_norm = nullptr;     // [ref_ng] norm group partials
  void set_reference_semantics(int flags);
  void evolution_reference(double tot[5]);
  RedSrc ref_src(const float* part, int order) const {
    RedSrc r;
    r.p = part;
    r.stride = ref_ng;
    r.nchunks = ref_ng;
    r.order = (uint32_t)order;
    return r;
  }
  double* partial_d = nullptr;   // [5 * pstride] check_evolution
  float* dsc = nullptr;          // device scalars
  float* H = nullptr;
  float* givens = nullptr;
  float* g = nullptr;
  float* y = nullptr;
  float* resid_hist = nullptr;
  float* binv = nullptr;         // [m+1] scales of the unnormalised basis vectors
  uint32_t* maxbits = nullptr;
  uint32_t* blockmax = nullptr;  // [2 * ceil(N/256)]
  float* h_pin = nullptr;        // pinned host scalars
  float* d_pin = nullptr;        // device view of h_pin (mapped)
  std::vector<hipEvent_t> ev_iter;
  hipEvent_t ev_outer[2]{};
  LagReader inner;
  // AMG
  bool amg_built = false;
  int amg_setup_path = 0;          // 0 not built, 1 host, 2 device (build_amg_device)
  int tail_first = 1;              // first AMG level handled by k_amg_tail
  // tail kernel form (CFD_AMG_TAIL): 2 the LDS image of matrices + vectors
  // (k_amg_tail_blob, starting up to tail_blob_shift levels lower to fit),
  // 1 vectors in LDS (k_amg_tail_lds), 0 global memory (k_amg_tail); the
  // weaker forms are also the fallbacks when the LDS does not hold the image
  int tail_form = 2;
  int tail_blob_shift = 2;
  // rows with more off-diagonals than this use the 16-bit layout (<= 255;
  // CFD_AMG_WIDE_LIMIT lowers it so that tests exercise the wide path)
  int amg_wide_limit = 255;
  size_t lds_budget = 0;           // dynamic LDS of the tail kernels on this device (init_kernel_attributes)
  // small-mesh kernel forms (CFD_SMALL_MESH_FORMS=0: the large-mesh forms on
  // every mesh): the CGS dots / update in their latency form (<= 2^17 cells,
  // several basis vectors per load round trip), the CGS totals reduced inside
  // the update kernel (<= 256 reduction units), every Jacobi relaxation sweep
  // in one single-workgroup launch (<= 8191 cells)
  bool small_forms = true;
  // nontemporal loads of the matrix streams (kernels.hip ldx), per kernel, for
  // the last readers of a matrix before the cycle moves on (CFD_NT, bit mask):
  // 1 post-smoother of the split levels, 2 level-0 AMG residual, 4 Schur
  // prediction, 8 SpMV, 16 pre-smoother, 32 the prolongation map of the split
  // levels, 64 level-1 AMG residual.  Same bits either way.  Tried and not kept:
  // the Schur correction (its lines are the SpMV's Infinity-Cache hits),
  // prepare / assemble (assemble re-reads prepare's face slots), the
  // restriction maps.
  unsigned nt_mask = 47;  // same-box A/B, profiles/r04/ab_nt_c2.txt, ab_nt2_c2.txt
  // an in-process group step failed on some rank: the ranks stopped at
  // different points of the step (ring rotation, time, FGMRES state), so the
  // group refuses to step until its state is restored on every rank
  // (cfd_state_load) or the caller accepts it (cfd_group_reset)
  bool needs_restore = false;
  // test hook (cfd_debug_group_fault_midstep): throw right after the step's
  // first prepare() when this rank's index matches
  int debug_fault_after_prepare = -1;
  bool nt(unsigned bit) const { return (nt_mask & bit) != 0; }
  // CGS: bytes of the dots pass's last blocks read with the default policy
  // (kept in the Infinity Cache for the top-down update after it); 0: every
  // basis read nontemporal, both passes bottom-up (set in the constructor:
  // 64 MB below 2^22 cells, else 0)
  size_t cgs_keep_bytes = 0;
  // post-smoothers of single-GPU / replicated levels of at most this many
  // rows read x + P xc (no prolongation launch; CFD_AMG_FUSED_PROLONG_ROWS)
  uint64_t fuse_prolong_rows = 1ull << 20;
  bool fused_prolong(int li) const { return !levels[li].dist && levels[li].dev.n <= fuse_prolong_rows; }
  AmgTailLevel* d_tail = nullptr;  // device copy of the level descriptors
  // k_amg_tail_blob: LDS image of the tail levels [tail_blob_first, L) (-1: none)
  int tail_blob_first = -1;
  uint32_t* d_tail_blob = nullptr;
  TailBlobLevel* d_tail_desc = nullptr;
  uint32_t tail_blob_words = 0, tail_vec_floats = 0;
  void build_tail_blob(int tf, bool reuse = false);  // reuse: rewrite the existing blob in place
  void set_resrestrict_blocks();
  // down-leg pairs (k_amg_resrestrict_pair): rr_pair[i].nblocks > 0 when levels
  // i and i+1 run as one launch (single-GPU / replicated levels that both take
  // k_amg_resrestrict, level i+1 pre-smoothed)
  std::vector<AmgPairImage> rr_pair;
  int pair_mode = 1;
  void build_rr_pairs();
  bool build_rr_pair(int i);
  // up-leg pairs (k_amg_prolong_smooth_pair): up_pair[c].nblocks > 0 when the
  // post-smoothers of levels c and c-1 run as one launch
  std::vector<AmgUpPairImage> up_pair;
  bool build_up_pair(int c);
  std::vector<AmgGpuLevel> levels;
  // the scalar matrix (ELL image, like sval) the hierarchy was built from:
  // snapshot at setup, or a checkpoint's (amg_src_loaded: ensure_amg builds from it)
  float* amg_src = nullptr;
  bool amg_src_loaded = false;
  // every device allocation of the hierarchy (levels, plans, tail images):
  // released as a whole when it is rebuilt (cfg.amg_rebuild_interval, load_state)
  DeviceArena amg_arena;
  uint32_t amg_age = 0;  // steps completed since the hierarchy was built
  void drop_amg();
  // numeric re-setup (device setup only): aggregation, P/R, every coarse
  // pattern, level layout and halo plan depend only on the sparsity pattern,
  // so a rebuild from new values re-runs just the Galerkin fill and the level
  // packing over the kept structure -- the same bytes as a full rebuild.
  struct AmgRefreshLevel {
    SetupMatrix fine{};                  // the level as the setup kernels read it (pack source)
    bool has_coarse = false;
    const uint32_t* gal_agg = nullptr;   // aggregate id per fine column (one GPU / replicated)
    const uint32_t* r_row = nullptr;     // R over the Galerkin input rows
    const uint32_t* r_col = nullptr;
    uint32_t nagg_own = 0;
    const uint32_t* rowptr_c = nullptr;  // this rank's coarse rows (fill output)
    uint32_t* col_c = nullptr;
    float* val_c = nullptr;
    size_t nnz_own = 0;
    // distributed level (build_amg_device_dist): the Galerkin input is the
    // member-row matrix `mem`; its values are gathered from the level's values
    // (own entries, msrc) and received from the ranks owning the imported rows
    // (val_msgs, whose send side is gathered through esrc into ebuf)
    bool dist = false;
    SetupMatrix mem{};
    const float* src_val = nullptr;
    const uint32_t* msrc = nullptr;
    const uint32_t* esrc = nullptr;
    uint32_t n_own_e = 0, n_exp_e = 0;
    float* ebuf = nullptr;
    std::vector<Msg> val_msgs;
    // last distributed level: the replicated level's values, all-gathered in place
    float* rep_val = nullptr;
    std::vector<size_t> rep_off;
  };
  std::vector<AmgRefreshLevel> amg_refresh;
  uint32_t* amg_setup_flag = nullptr;  // k_galerkin overflow flag (amg_arena)
  bool amg_refresh_pending = false;    // refresh at the next AMG solve
  void refresh_amg();
  void member_values(const AmgRefreshLevel& F);
  // host-side state
  cfd_constants constants{};
  cfd_step_info info{};
  std::vector<std::pair<double, double>> variance_history;
  // profiling of the level-0 smoother
  bool prof = false;
  std::vector<hipEvent_t> prof_ev;
  size_t prof_used = 0;
  double prof_ms = 0.0;
  uint64_t prof_launches = 0;
  // every level-0 sweep is timed while profiling is on.  An event-bracketed
  // launch is serialised with its neighbours: timing every sweep costs ~0.7 %
  // of the step, but a sample of them (round 4's CFD_PROF_STRIDE, removed:
  // under graph replay the sample was frozen into the captured graphs) read
  // ~4 % slower than the rocprofv3 average of all sweeps.
  uint64_t prof_seq = 0;
  bool prof_take() { return prof && (++prof_seq, true); }

  // ---- hipGraph replay of the FGMRES iteration (Solver::run_iteration) ----
  // One executable graph per (basis index j, residual-slot variant): the
  // iteration's launches (Schur prediction, V-cycle or Jacobi sweeps, Schur
  // correction, SpMV, CGS, Givens) depend on j only, every pointer they take is
  // fixed once the Krylov space and the AMG hierarchy exist, so the graph is
  // captured on first use and replayed by every later solve: one host call per
  // iteration instead of ~14-20 launches.  Dropped with the hierarchy
  // (drop_amg) and on a preconditioner switch.  While the level-0 smoother is
  // being timed (prof) its launches in the graph are bracketed by event nodes
  // owned by the graph; every replay's times are harvested before the next
  // replay of that graph (graph_harvest) or when the profile is read.
  // cfd_graph_enable turns it on for one GPU (R = 1); off by
  // default: the same-box A/B found replay no faster than eager launches at
  // C0 and C1 -- the GPU's kernel boundaries, not the host's launch rate,
  // bound the small-mesh iteration.
  struct IterGraph {
    hipGraphExec_t exec = nullptr;
    std::vector<hipEvent_t> ev;  // timing pairs of the level-0 smoother (prof captures)
    bool prof = false;           // captured with the timing pairs
    bool pending = false;        // replayed since the last harvest
  };
  bool graph_on = false;
  std::vector<IterGraph> graphs;   // [3 j + variant]; variant 0 fixed schedule, 1 + pinned residual slot
  int graph_precond = -1;          // precond_type the graphs were captured for
  IterGraph* capturing = nullptr;  // the graph being captured (amg_smooth's timing pairs)
  uint64_t graph_captures = 0, graph_replays = 0;
  void drop_graphs();
  void graph_harvest(IterGraph& G, bool discard);
  void graph_harvest_all(bool discard);  // the stream must be idle

  Solver(const cfd_mesh_view& mesh, const cfd_config& cfg, int device,
         std::unique_ptr<Comm> comm = nullptr);
  ~Solver();
  StateView& S() { return ring[i_state]; }

  void set_u(const double* uv);
  void set_p(const double* p);
  void initialize_history();
  void step();
  void get_u(double* uv);
  void get_p(double* p);
  void get_d_p(double* dp);
  void debug_prepare_assemble(bool assemble);
  void get_global_ids(uint32_t* c0, uint32_t* c1) const { *c0 = topo.c0; *c1 = topo.c1; }
  size_t debug_len(int id) const;
  void debug_buffer(int id, float* out);
  double algorithmic_step_bytes() const;
  double layout_step_bytes() const;
  double smoother_bytes() const;
  double smoother_layout_bytes() const;
  // checkpoint / resume (checkpoint.cpp, cfd_state_file_header)
  void save_state(const char* path);  // collective on a distributed solver
  void load_state(const char* path);
  uint64_t amg_level_digest(int li);  // FNV-1a over every byte of level li's device image
  std::vector<uint64_t> allgather_u64(uint64_t mine);  // every rank's value (collective)

 private:
  void rotate();
  void prepare();
  void assemble();
  cfd_linear_stats solve();
  void flush_inner();
  void ensure_fgmres();
  void ensure_amg();
  void build_amg_host();
  bool build_amg_device();  // false: a per-thread capacity overflowed on some rank (host path then)
  bool build_amg_device_dist();
  bool device_levels(AmgSetupLevel& cur, int li0, const std::vector<uint64_t>& part0);
  std::vector<std::vector<uint32_t>> allgatherv_u32(const std::vector<uint32_t>& mine);  // collective
  void set_amg_full_policy(AmgGpuLevel& G, int li);
  void precondition(int j, float* z);
  void iteration(int j, float* pin);  // one FGMRES iteration's launches (fixed order, no host reads)
  void run_iteration(int j, float* pin, int variant);  // eager or graph replay
  void v_cycle();
  void amg_smooth(size_t li, float*& x, const float* b, bool x_zero = false, bool nt = false);
  std::pair<hipEvent_t, hipEvent_t> prof_pair();
 public:
  static constexpr size_t kProfPoolMax = 1u << 15;
  void prof_grow(size_t n);  // event pool of at least n events
 private:
  void norm_launch(const float* v, int mode, int slot);
  float norm_blocking(const float* v, int mode, int slot);
  void residual_into_v0_launch();
  float residual_into_v0_blocking();
  void check_evolution();
  void sync() { CFD_HIP(hipStreamSynchronize(stream)); }
 public:
  // Launch-error check: hipGetLastError after each phase of the step (a host
  // call, no synchronisation); with cfg.log_level >= 3 the stream is also
  // synchronised there, so an asynchronous kernel fault is reported at the
  // phase that caused it (debug runs).
  void check_launch(const char* where) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) throw HipError(std::string("kernel launch in ") + where + ": " + hipGetErrorString(e));
    if (check_sync) {
      const hipError_t e2 = hipStreamSynchronize(stream);
      if (e2 != hipSuccess) throw HipError(std::string("kernel execution in ") + where + ": " + hipGetErrorString(e2));
    }
  }
  bool check_sync = false;
 private:
  // cfg.log_level >= 1: the reference's println! progress lines, on stderr, rank 0
  void log(const char* fmt, ...) const __attribute__((format(printf, 2, 3)));
  CoupledMatrix cmat() const;
  // per-cell vectors: allocation with ghost space, owned-base pointers
  template <class T>
  T* valloc(int comps);
  template <class T>
  T* vbase(T* p, int comps) const { return p - (size_t)shift * comps; }
  // image of a global per-cell array (f64 input or f32 checkpoint) in this
  // rank's local layout (owned + ghosts)
  template <class G>
  void local_image(const G* g, int comps, std::vector<float>& out) const {
    out.assign(vlen * comps, 0.0f);
    auto put = [&](size_t local, uint64_t gid) {
      for (int c = 0; c < comps; ++c) out[local * comps + c] = (float)g[gid * comps + c];
    };
    for (uint32_t li = 0; li < N; ++li) put(shift + li, (uint64_t)topo.c0 + li);
    for (uint32_t k = 0; k < topo.glo; ++k) put(shift - topo.glo + k, topo.ghost[k]);
    for (uint32_t k = 0; k < topo.ghi; ++k) put(shift + topo.npad + k, topo.ghost[topo.glo + k]);
  }
  // distributed plumbing
  bool dist() const { return R > 1; }
  struct HField {
    float* ptr;
    int comps;
  };
  void halo(HaloPlan& plan, std::initializer_list<HField> fields);
  // exchange on the comm stream; halo_end makes the compute stream wait for it
  void halo_begin(HaloPlan& plan, std::initializer_list<HField> fields);
  void halo_end();
  // launch(r0, r1, r2, r3) over rows [0, n): interior rows overlap the halo
  // exchange, both boundary strips follow it in one launch (one GPU: a single
  // launch over all rows).  Below
  // overlap_min_rows the interior launch is too short to hide an exchange and
  // the split only triples the launches of a latency-bound kernel: one launch
  // after the exchange.
  uint32_t overlap_min_rows = 1u << 20;
  template <class F>
  void overlapped(HaloPlan& plan, std::initializer_list<HField> fields, uint32_t n, F&& launch) {
    if (!dist()) {
      launch(0u, n, 0u, 0u);
      return;
    }
    if (n < overlap_min_rows) {
      halo(plan, fields);
      launch(0u, n, 0u, 0u);
      return;
    }
    halo_begin(plan, fields);
    if (plan.hi_begin > plan.lo_end) launch(plan.lo_end, plan.hi_begin, 0u, 0u);
    halo_end();
    // both boundary strips in one launch
    const uint32_t hb = plan.hi_begin > plan.lo_end ? plan.hi_begin : plan.lo_end;
    if (plan.lo_end > 0 || n > hb) launch(0u, plan.lo_end, hb, n > hb ? n : hb);
  }
  hipStream_t cstream = nullptr;  // RCCL / peer-copy stream of the halo exchanges
  hipEvent_t hev_pack = nullptr, hev_done = nullptr;

 public:
  // ---- timing of the distributed communication (cfd_comm_timing) ----
  // While comm_prof is on, every halo exchange and all-gather of the step is
  // bracketed by timing events: `wait` = how long the compute stream stood
  // still for it (a halo: from the wait on the exchange's completion event
  // to its release; an all-gather, which runs on the compute stream: its
  // whole duration), `comm` = the transport's own time (a halo: the grouped
  // send/recv on the comm stream, including the wait for the peers).  Per
  // category; AMG halos per level.
  enum CommCat {
    kCommKrylovHalo = 0,   // V_j / p_sol / Z_j / x halos of the FGMRES iteration
    kCommStateHalo = 1,    // FluidState, prepare / assemble outputs, check_evolution records
    kCommReduceGather = 2, // segment values of the reductions (CGS dots, norms), max-diff
    kCommRepGather = 3,    // rhs of the first replicated AMG level
    kCommAmgHalo = 4,      // + level: x / residual / coarse-x halos of AMG level l
  };
  static constexpr int kCommAmgLevels = 28;
  static constexpr int kCommCats = kCommAmgHalo + kCommAmgLevels;
  struct CommTimes {
    uint64_t calls = 0;
    double wait_ms = 0.0, comm_ms = 0.0;
    uint64_t bytes = 0;
  };
  CommTimes comm_times[kCommCats];
  bool comm_prof = false;
  void comm_prof_reset();
  static int amg_cat(int level) { return kCommAmgHalo + std::min(level, kCommAmgLevels - 1); }
  void comm_drain();  // synchronise both streams, fold the pending records into comm_times
  struct CommScope {  // category of the halos / all-gathers issued inside the scope
    Solver* s;
    int prev;
    CommScope(Solver* s_, int c) : s(s_), prev(s_->comm_cat) { s->comm_cat = c; }
    ~CommScope() { s->comm_cat = prev; }
  };

 private:
  int comm_cat = kCommStateHalo;
  int halo_cat = kCommStateHalo;  // category of the exchange in flight (halo_begin -> halo_end)
  struct CommRec {
    int cat, kind;  // kind 0: compute-stream wait, 1: comm time
    hipEvent_t a, b;
  };
  std::vector<CommRec> comm_recs;
  std::vector<hipEvent_t> comm_ev_pool;
  size_t comm_ev_used = 0;
  hipEvent_t comm_event();
  // an all-gather on the compute stream, timed when comm_prof is on
  template <class F>
  void timed_gather(int cat, size_t bytes, F&& f) {
    comm->label = cat;
    if (!comm_prof) {
      f();
      return;
    }
    hipEvent_t a = comm_event(), b = comm_event();
    CFD_HIP(hipEventRecord(a, stream));
    f();
    CFD_HIP(hipEventRecord(b, stream));
    comm_recs.push_back({cat, 2, a, b});  // kind 2: counts as both wait and comm
    comm_times[cat].calls++;
    comm_times[cat].bytes += bytes;
  }

 private:
  void halo_state(bool all);
  // the source the finishing kernels read for nvec reductions of chunk
  // partials part[v * nchunks + k]: the partials themselves on one GPU; on a
  // distributed rank its segment values are computed and all-gathered first
  RedSrc combine(const float* part, int nvec);
  RedSrcD combine_d(const double* part, int nvec);
  void make_plan_buffers(HaloPlan& p, int max_comps);
};

}  // namespace cfd2
