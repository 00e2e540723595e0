// Kernel argument blocks + launch wrappers for the gfx950 HIP kernels.
//
// Data layout in HBM:
//  * per-cell arrays are SoA (float / float2) indexed by cell;
//  * per-(cell, face-slot) static geometry and per-(cell, neighbour-slot)
//    matrix blocks are ELL "slot-major": element (slot k, cell i) at k*N + i,
//    so lane-i accesses of one slot are fully coalesced across a wavefront;
//  * the coupled 3N x 3N matrix is stored as compressed 3x3 blocks: the
//    reference CSR (init/linear_solver/mod.rs:180-216) always holds
//    A_uu == A_vv, A_uv == A_vu == 0, A_up == A_pu, A_vp == A_pv per
//    off-diagonal block (coupled_assembly_merged.wgsl:221-333), so two float2
//    per block -- cval_a {c, pp} and cval_g {gx, gy} -- reproduce every CSR
//    entry bit-for-bit.  The Schur predict/correct kernels read cval_g only.
//  * Krylov basis vectors are stored unnormalised (W_i) with their scale
//    binv[i]; every consumer forms V_i[e] = binv[i] * W_i[e] (one f32 multiply,
//    the same rounding as the reference's `scale` pass, which is thereby gone).
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>

#include <vector>

#include "../../../include/cfd2_amd.h"

namespace cfd2 {

// meta bits of a face slot
constexpr uint32_t kMetaBtypeMask = 0x3u;      // 0 internal, 1 inlet, 2 outlet, 3 wall
constexpr uint32_t kMetaOwner = 1u << 2;       // face_owner == this cell
constexpr uint32_t kMetaDegen = 1u << 3;       // d_c + d_o <= 1e-6 (lambda fallback 0.5)
constexpr uint32_t kMetaFluxFlip = 1u << 4;    // normal_flux = -stored normal
constexpr uint32_t kMetaRankShift = 8;         // scalar-row rank of the neighbour (0xFF boundary)
constexpr uint32_t kMetaTSlotShift = 16;       // its slot in the coupled-matrix ELL (Topology::tslot)

// Canonical reduction order (rank-invariant; mirrors oracle/oracle.cpp).  A
// sum over cells is ONE fixed binary tree over global cell indices:
//   chunk    256 consecutive cells [256k, 256k + 256): pairwise tree over the
//            256 cell terms (missing cells: +0).  The cell term of a dot of
//            3-component vectors (3 floats per cell) is (x_u y_u + x_v y_v) +
//            x_p y_p.  GPU: a wavefront's 64 consecutive cells by a shuffle tree
//            (strides 1, 2, ..., 32), then the chunk's 4 quarters pairwise
//   segment  G = 2^g consecutive chunks: pairwise tree over G chunk slots
//            (chunks past the end: +0).  g depends on the GLOBAL cell count
//            only: g = clamp(floor(log2(N / 16384)), 0, 8)
//   total    pairwise tree over the segment values, padded with +0 to a power
//            of two.
// A rank owns whole segments (partition_starts), so each segment value is
// computed by one rank and the total from the all-gathered segment values: R
// ranks produce exactly the bits of one GPU.  The chunk kernels combine the
// 4 chunks of their block as far as a segment allows: they write "units" of
// U = min(G, 4) chunks (the first log2(U) levels of the segment tree), so a
// segment is G / U units.
constexpr uint32_t kRedChunkCells = 256;
constexpr uint32_t kRedMaxSegLog2 = 8;
constexpr uint32_t kRedMaxSegments = 4096;  // the total's tree runs in LDS (N <= 268 M cells)

struct RedGeom {
  uint32_t g = 0;          // log2 chunks per segment
  uint32_t G = 1;          // chunks per segment
  uint32_t U = 1;          // chunks per unit written by the chunk kernels: min(G, 4)
  uint64_t seg_cells = 256;
  uint32_t nchunks = 0;    // global chunks
  uint32_t nseg = 0;       // global segments
};
inline RedGeom red_geom(uint64_t nglob) {
  RedGeom r;
  uint32_t g = 0;
  while (g < kRedMaxSegLog2 && (nglob >> (g + 1)) >= 16384u) ++g;
  r.g = g;
  r.G = 1u << g;
  r.U = r.G < 4 ? r.G : 4;
  r.seg_cells = (uint64_t)kRedChunkCells << g;
  r.nchunks = (uint32_t)((nglob + kRedChunkCells - 1) / kRedChunkCells);
  r.nseg = (uint32_t)((r.nchunks + r.G - 1) / r.G);
  return r;
}

// Source of a reduction's segment values for the kernels that finish it
// (the total's tree).  One GPU: unit partials p[v * stride + k], k < nchunks
// (here: units), G units per segment; the segment trees are built from them.  Distributed: the all-gathered
// segment values, rank q's block [q][v][local segment] of nvec x stride
// values; seg_src[s] = (q << 20) | local segment of global segment s.
template <class T>
struct RedSrcT {
  const T* p = nullptr;
  uint32_t stride = 0;
  uint32_t nchunks = 0;
  uint32_t G = 1;
  uint32_t nseg = 0;
  uint32_t nvec = 1;
  const uint32_t* seg_src = nullptr;
  // 0: the canonical tree.  Reference order (test mode, Solver::ref_red): 1
  // one thread adds the nchunks group partials in order (reduce_final,
  // gmres_ops.wgsl:257-262); 2 lanes t < 64 add partials t, t + 64, ...,
  // then the 64-wide halving tree (reduce_dots_cgs, gmres_cgs.wgsl:97-118)
  uint32_t order = 0;
};
using RedSrc = RedSrcT<float>;
using RedSrcD = RedSrcT<double>;

// Local cell numbering: every per-cell device pointer points at the first
// OWNED cell; neighbour indices are signed offsets from it.  On one GPU they
// are the global indices; on a distributed rank ghosts of lower ranks sit at
// [-glo, 0) and ghosts of higher ranks at [npad, npad + ghi) (npad = owned
// count rounded up to 64), so local order == global order.
constexpr int32_t kNoCell = INT32_MIN;  // boundary face: no neighbour

struct FaceSlots {  // ELL [k*N + i], k < wf
  const int32_t* other;  // neighbour (signed local index) or kNoCell
  const uint32_t* meta;
  const float* area;
  const float* nx;  // normal oriented out of this cell
  const float* ny;
  const float* lam_s;   // lambda from this cell's side (d_o / (d_c + d_o))
  const float* lam_f;   // lambda from the owner's side (flux interpolation)
  const float* dist_a;  // max(|d . n|, 1e-6)
  const float* dist_e;  // |other_center - center|
  const float* dvx;     // other_center - center
  const float* dvy;
  const float* rx;      // f_center - center
  const float* ry;
  const float* rox;     // f_center - other_center
  const float* roy;
  const uint32_t* nface;  // [N]
  int wf;
};

struct StateView {
  float2* u;
  float* p;
  float* dp;
  float2* gp;
};

struct PrepareArgs {
  uint32_t N;
  cfd_constants c;
  FaceSlots fs;
  const float* vol;
  StateView st;       // read (snapshot)
  float* dp_out;      // new d_p
  float2* gp_out;     // new grad_p
  float* flux_s;      // [k*N + i] oriented flux
  float2* grad_u;
  float2* grad_v;
};

struct AssembleArgs {
  uint32_t N;
  uint32_t ld;             // scalar-row ELL slot stride
  cfd_constants c;
  FaceSlots fs;
  const float* vol;
  StateView st;            // current iterate (d_p already refreshed)
  const float2* u_old;     // state_old.u
  const float2* u_old_old; // state_old_old.u
  const float* flux_s;
  const float2* grad_u;
  const float2* grad_v;
  const uint32_t* srank_diag;  // [N] diagonal rank in the scalar row
  const uint8_t* cslot_diag;   // [N] slot of the diagonal in the coupled-matrix ELL
  float2* cval_a; // [r*ld + i] {A_uu (=A_vv), A_pp}
  float2* cval_g; // [r*ld + i] {A_up (=A_pu), A_vp (=A_pv)}
  float2* cdiag2; // [ld] {s_pu, s_pv} of the diagonal block
  float* sval;    // [r*ld + i] scalar pressure matrix
  float* rhs;     // [3N]
  float* dinv_uv; // [N]
  float* dinv_p;  // [N]
};

// The Krylov kernels process 4 consecutive rows per thread: every per-slot
// array is one 16/32-byte load per thread, columns are 16-bit deltas when the
// whole matrix allows it, lengths / diagonal ranks u8.
struct CoupledMatrix {
  uint32_t N;
  uint32_t r0, r1;        // rows this launch processes (multiples of 4 except r1 = N)
  uint32_t r2, r3;        // optional second row range of the same launch (empty: r3 <= r2)
  uint32_t ld;            // slot stride (N rounded up to 64)
  int ws;
  int use16;
  // aligned-slot ELL (Topology::tslot): entries of a row sit in increasing
  // slots (CSR order), gaps where a neighbour is missing
  const int32_t* col;     // [r*ld + i] signed local column (gaps: a virtual column)
  const int16_t* col16;   // [r*ld + i] col - i (use16)
  const uint16_t* lg;     // [ld] slots in use (bits 0-6) | regular row (bit 7) | gap mask << 8
  const uint8_t* drank;   // [ld] slot of the diagonal
  const float2* cval_a;
  const float2* cval_g;
  const float2* cdiag2;   // [ld]
  // regular rows (lg bit 7): every slot's column is row + tmode[slot] (the
  // per-slot modal delta), so the kernels derive the columns instead of
  // loading them; set when ws <= kCoupledRegMaxWs (one peeled slot group)
  int reg;
  int tmode[8];
};
constexpr uint32_t kLgUsedMask = 0x7Fu, kLgRegular = 0x80u;
constexpr int kCoupledRegMaxWs = 5;

// One AMG level (linear_solver/amg.rs AmgLevel) in the layout the gfx950
// kernels stream: off-diagonal entries only, ELL slot-major with row stride
// `stride` (= n rounded up to 64, so four consecutive rows of one slot are one
// 16-byte load), columns as 16-bit deltas (col - row) when every delta of the
// level fits, else 32-bit; per-row length and diagonal position as u8.
// Off-diagonals keep the reference CSR order (ascending column), so every
// row sum accumulates in the reference order.
struct AmgLevelDev {
  uint32_t n;
  uint32_t r0, r1;       // rows a smoother / residual launch processes (default 0, n)
  uint32_t r2, r3;       // optional second row range of the same launch (empty: r3 <= r2)
  uint32_t stride;       // row stride of the ELL slots (n rounded up to 64)
  int w;                 // ELL width (max off-diagonals per row)
  int use16;             // 1: col16 holds deltas; 0: col32 holds absolute columns
  int full;              // slot-load mode of the row kernels (kernels.hip gather_group): 0 or 1
  const float* val;      // [r*stride + i]
  const int16_t* col16;  // [r*stride + i]  col - i
  const int32_t* col32;  // [r*stride + i] signed local column
  const uint8_t* len;    // [stride] off-diagonal count per row
  const uint8_t* drank;  // [stride] position of the diagonal among the row's entries
  const float* dv;       // [stride] raw diagonal value (0 if absent)
  const float* de;       // [stride] smoother diagonal (dv, or 1.0 if |dv| < 1e-14)
  // wide level (a row with more off-diagonals than kAmgWideLimit): 16-bit row
  // lengths / diagonal ranks here (len / drank then hold min(., 255) and are
  // not read).  Only the one-workgroup tail kernels run wide levels
  // (Solver::ensure_amg moves the tail up to the first wide level).
  const uint16_t* len16;
  const uint16_t* drank16;
  // coarsening operators (only when nc > 0)
  uint32_t nc;
  const uint32_t* agg;     // [stride] P: fine -> coarse (padding rows -> 0, never read)
  const uint32_t* r_row;   // [nc+1] R = P^T rows (fine indices ascending)
  const uint32_t* r_col;
  // [nc] the first 4 members of each aggregate (k_amg_restrict: one 16-byte
  // load instead of r_row -> r_col); -1 pads, r_m4[I].w < -1 flags an
  // aggregate with more than 4 members (the rest read through r_row / r_col)
  const int4* r_m4;
  // k_amg_resrestrict: aggregates per block (0: the level keeps the separate
  // residual + restriction kernels); every block's members fit kRRCap
  uint32_t rr_agg;
};
constexpr uint32_t kRRCap = 2048;  // residuals per block of k_amg_resrestrict (LDS floats)

// k_amg_resrestrict_pair: the down-leg of two adjacent single-GPU / replicated
// levels (i, i+1) in one launch.  A block owns level-(i+2) aggregates
// [jb[k], jb[k+1]); its level-(i+1) rows S = the members of those aggregates
// (R order, written by the block) then their off-diagonal columns outside
// them (the ring, recomputed redundantly); f lists the level-i members of every
// S row (R order).  Built at AMG setup (Solver::build_rr_pairs) so that every
// block's S, f and aggregates fit kPairThreads.
constexpr uint32_t kPairThreads = 1024;
constexpr int kPairW = 8;  // level-(i+1) slots prefetched before the level-i phase
struct AmgPairImage {
  uint32_t nblocks;
  uint32_t threads;    // block size = per-block capacity (256 or kPairThreads)
  const uint32_t* jb;  // [nblocks + 1] level-(i+2) aggregate ranges
  const uint32_t* sb;  // [nblocks + 1] ranges in s
  const uint32_t* s;   // level-(i+1) rows: each block's members first, then its ring
  const uint32_t* fo;  // [|s| + 1] ranges in f of each s row's level-i members
  const uint32_t* f;   // level-i rows
  const uint16_t* lc;  // [r * stride_{i+1} + row] block-local index (in s) of slot r's column
};

// k_amg_prolong_smooth_pair: the up-leg of two adjacent single-GPU /
// replicated levels in one launch -- the post-smoother of coarse level c (its
// prolongation from c+1 applied to its reads, k_amg_smooth<..., PRO>) for the
// rows T the block needs, kept in LDS, then the post-smoother of fine level
// c-1 reading x_f + P x_c.  A block owns kUpPairRows consecutive fine rows;
// level c's smoothed x is never stored (nothing reads it after the up-leg).
constexpr uint32_t kUpPairRows = 256;
constexpr uint32_t kUpPairCap = 1024;  // T rows per block (LDS floats)
struct AmgUpPairImage {
  uint32_t nblocks;
  const uint32_t* tb;   // [nblocks + 1] ranges in t
  const uint32_t* t;    // level-c rows of each block (ascending)
  const uint16_t* lt;   // [r * stride_f + row] T-local index of agg_f[col] of fine slot r
  const uint16_t* lto;  // [stride_f] T-local index of agg_f[row]
};
// zeroed entries after every level's agg array: the fused prolongation reads
// agg with 16-byte loads from any column (as the x gathers, whose vectors
// carry the same slack)
constexpr size_t kAggSlack = 64;

// Halo pack (distributed): up to 8 fields packed per launch.
struct PackField {
  const float* src;   // owned-base pointer of the field
  int comps;          // floats per cell
  uint32_t stage_off; // offset of this field's block in the stage buffer (floats)
};
struct PackArgs {
  PackField f[8];
  int nf;
  const int32_t* idx;  // [n] owned local rows to send
  uint32_t n;
  float* stage;
};

// r_m4 image of R (kernels.hip k_amg_restrict)
void build_r_m4(const std::vector<uint32_t>& r_row, const std::vector<uint32_t>& r_col, std::vector<int32_t>& out);

// Levels handled by the single-workgroup V-cycle tail kernel.
struct AmgTailLevel {
  AmgLevelDev L;
  float* x;
  float* xt;
  float* b;
  float* r;
};
constexpr int kMaxAmgLevels = 20;

// One tail level inside the LDS blob of k_amg_tail_blob (offsets in 32-bit
// words from the blob start, each array 16-byte aligned): off-diagonal CSR
// with u16 columns, diagonal data, P (agg, u16) and R (u16 CSR).
struct TailBlobLevel {
  uint32_t n, nc;
  uint32_t de, dv, rowoff, drank, val, col, agg, r_row, r_col;
  uint32_t maxlen;  // longest row (off-diagonal entries)
};

// ---------------- launch wrappers (kernels.hip) ----------------
void launch_prepare(const PrepareArgs& a, hipStream_t s);
// test mode (reference semantics): the reference's racy prepare with its 64-cell
// workgroups in order, d_p / grad_p in place (a.dp_out / a.gp_out = a.st's),
// then every non-owner face slot e takes -flux_s[mirror[e]] (mirror[e] < 0:
// owner or boundary slot, kept)
void launch_prepare_ordered(const PrepareArgs& a, const int32_t* mirror, uint32_t slots, hipStream_t s);
void launch_assemble(const AssembleArgs& a, hipStream_t s);
// writes per-block max bit patterns to blockmax[2*nb] and the final pair to maxbits[0..1]
// (and to host_out[0..1], a device view of pinned host memory, when non-null)
void launch_update_fields(uint32_t N, float alpha_u, float alpha_p, const float* x, float2* u,
                          float* p, uint32_t* blockmax, uint32_t* maxbits, uint32_t* host_out, hipStream_t s);
// unit partials (U chunks of 256 cells each) of dot(x, y) over 3-component cells
void launch_dot_partial(const float* x, const float* y, uint32_t N, uint32_t U, float* partial, hipStream_t s);
// Reference reduction order (test mode): partial[g] = the 64-wide halving tree
// of v[i] * v[i] over DOFs i in [64 g, 64 g + 64) of the 3N (norm_sq_partial,
// gmres_ops.wgsl:195-223); ng = ceil(n3 / 64) groups
void launch_ref_norm_partials(const float* v, uint32_t n3, float* partial, hipStream_t s);
// partial[ii * pstride + g] = the same tree of V_ii[i] * w[i], V_ii = binv[ii] *
// W_ii, ii = 0..j (calc_dots_cgs, gmres_cgs.wgsl:28-82)
void launch_ref_cgs_dots(const float* w, const float* basis, const float* binv, size_t stride, int j, uint32_t n3,
                         float* partial, uint32_t pstride, hipStream_t s);
// total of the reduction r (one vector): mode 1: out[0] = sqrt(total); mode 2:
// also *inv = 1.0f / sqrt (host-style) and g0 (if non-null) = sqrt
// g0 (mode 2): g0[0] = norm, g0[1..g_len) = 0; host_out (device view of pinned host memory, or null) = norm
void launch_reduce_final(const RedSrc& r, int mode, float* out, float* inv, float* g0, int g_len, float* host_out,
                         hipStream_t s);
// b != null: y = b - A x with the residual axpby's operations (1 * b + -1 * (A x))
// nt: the matrix and b are read with the nontemporal policy (kernels.hip ldx)
void launch_spmv(const CoupledMatrix& A, const float* x, float* y, hipStream_t s, const float* b = nullptr,
                 bool nt = false);
// basis: unnormalised W_i at basis + i*stride, scales binv[i]; unit partials
// partial[ii * np + k] of <w, V_ii>, ii = 0..j
// keep_bytes > 0: the last blocks (their j + 2 vectors within keep_bytes) read
// the basis with the default policy, for a top-down update (rev) after it
void launch_cgs_dots(const float* w, const float* basis, const float* binv, size_t stride, int j,
                     uint32_t N, uint32_t U, float* partial, uint32_t np, hipStream_t s, size_t keep_bytes = 0,
                     bool lat = false);
// H[j][ii] = total of vector ii of r (r.nvec = j + 1)
void launch_cgs_reduce(const RedSrc& r, int j, float* H, int m1, hipStream_t s);
// W_{j+1} = w - sum_i H[i,j] V_i  (written into basis slot j+1) + ||W_{j+1}||^2 unit partials
// fr != null: the CGS totals (H column j) reduced inside the update from the
// dots' unit partials (k_cgs_reduce not launched); only where
// cgs_reduce_fusable(*fr) holds -- one GPU, at most 256 padded units
void launch_cgs_update_norm(const float* w, float* basis, const float* binv, size_t stride, int j, float* H,
                            int m1, uint32_t N, uint32_t U, float* partial, hipStream_t s, bool rev = false,
                            bool ntb = true, const RedSrc* fr = nullptr, bool lat = false);
// small meshes (<= CFD_CGS_LAT_MAX_CELLS): the CGS dots / update in their
// latency form (several basis vectors per load round trip; same bits)
bool cgs_latency_form(uint32_t N);
bool cgs_reduce_fusable(const RedSrc& r);
// ||W_{j+1}|| = sqrt(total of r) -> H[j+1,j], binv[j+1]; Givens update of column j; resid_hist[j] = |g[j+1]|,
// also into host_resid[j] (device view of pinned host memory) when non-null
void launch_norm_givens(const RedSrc& r, int j, float* H, int m1, float* givens, float* g, float* binv,
                        float* resid_hist, float* host_resid, hipStream_t s);
// r_in = binv[j] * W_j
void launch_precond_predict(const CoupledMatrix& A, const float* w_in, const float* binv, int j,
                            const float* dinv_uv, const float* dinv_p, float* temp_p, float* p_sol,
                            float* p_prev, hipStream_t s, bool nt = false);
// one relax_pressure sweep, 4 rows per thread over the scalar ELL image viewed as
// an AmgLevelDev (val = the live scalar matrix, len / col16 / col32 incl. the
// diagonal, skipped by `drank`); rows [L.r0, L.r1) + [L.r2, L.r3)
void launch_relax_pressure4(const AmgLevelDev& L, const uint8_t* drank, const float* dinv_p, const float* temp_p,
                            const float* src, float* dst, hipStream_t s);
// all `iters` relax_pressure sweeps in one single-workgroup launch (p_sol / temp
// ping-pong as the per-sweep launches, the final iterates back in both); false
// when N > kRelaxFusedMaxRows or the ELL width is too wide for the register image
constexpr uint32_t kRelaxFusedMaxRows = 8191;  // two (N + 1)-float iterates in 64 KiB of LDS
bool launch_relax_pressure_fused(uint32_t N, uint32_t ld, uint32_t ws, const int32_t* col, const uint32_t* len,
                                 const float* sval, const float* dinv_p, const float* temp_p, float* p_sol,
                                 float* temp, uint32_t iters, hipStream_t s);
void launch_precond_correct(const CoupledMatrix& A, const float* w_in, const float* binv, int j,
                            const float* p_sol, const float* dinv_uv, float* z, hipStream_t s);
void launch_solve_triangular(const float* H, const float* g, float* y, int k, int m1,
                             hipStream_t s);
// lat: the latency form allowed (small meshes; false = the streaming form)
void launch_update_x(float* x, const float* z, size_t stride, const float* y, int k, size_t n,
                     hipStream_t s, bool lat = true);
// ev0/ev1 (optional): timing events recorded by the GPU at kernel start / end
// nt: the level matrix, b and the diagonal read with the nontemporal policy
void launch_amg_smooth(const AmgLevelDev& L, const float* x, const float* b, float* x_out,
                       hipStream_t s, hipEvent_t ev0 = nullptr, hipEvent_t ev1 = nullptr, bool nt = false);
// post-smoother with the prolongation fused: x_out = smooth(x + P xc), bit-identical
// to launch_amg_prolong(L, x, xc) then launch_amg_smooth(L, x, b, x_out), but x is
// only read (single-GPU / replicated levels: every column an owned row)
void launch_amg_smooth_prolong(const AmgLevelDev& L, const float* x, const float* xc, const float* b,
                               float* x_out, hipStream_t s);
// test mode (reference semantics): the reference's in-place smoother with its
// 64-row workgroups run in order (rows of a workgroup read before any writes)
void launch_amg_smooth_ordered(const AmgLevelDev& L, float* x, const float* b, hipStream_t s);
// pre-smoother of a level whose x is identically +0 (bit-identical to launch_amg_smooth then)
void launch_amg_smooth_zero(const AmgLevelDev& L, const float* b, float* x_out, hipStream_t s);
void launch_amg_residual(const AmgLevelDev& L, const float* x, const float* b, float* r,
                         hipStream_t s, bool nt = false);
// coarse_b = R r and coarse_x = 0 (the reference's separate `clear` pass fused); on a
// distributed coarse level also clears its ghosts: [-glo, 0) and [stride_c, stride_c + ghi)
// sm_out != null: instead of clearing coarse_x, write the coarse level's
// zero-x pre-smoother result (mix(0, (b - 0)/de, 0.8), de = sm_de) to sm_out.
// Coarse rows [I0, I1) only (I1 = 0: all L.nc); `ghosts` false: no ghost
// clearing (a distributed launch split around the residual halo).
void launch_amg_restrict(const AmgLevelDev& L, const float* r, float* coarse_b, float* coarse_x,
                         uint32_t stride_c, uint32_t glo, uint32_t ghi, hipStream_t s,
                         float* sm_out = nullptr, const float* sm_de = nullptr, uint32_t I0 = 0,
                         uint32_t I1 = 0, bool ghosts = true);
// V-cycle restricted to levels [first, nlev) of `tail` (device array), one workgroup:
// pre-smooth / residual / restrict+clear down, 10 coarsest sweeps, prolong / post-smooth up.
// Every level's x ends in tail[l].x (even sweep counts).
// lds_bytes > 0: the LDS-resident version (needs every tail vector in <= kTailLdsMax bytes)
constexpr size_t kTailLdsMax = 160 * 1024 - 1024;
void launch_amg_tail(const AmgTailLevel* tail, int first, int nlev, size_t lds_bytes, hipStream_t s);
// The LDS tail with the matrices in LDS too: `blob` (blob_words 32-bit words,
// a multiple of 4) is copied into LDS after the vectors (vec_floats floats);
// desc[l] describes level l (l in [first, nlev)).  lds_bytes = 4 * (vec_floats + blob_words).
void launch_amg_tail_blob(const AmgTailLevel* tail, const TailBlobLevel* desc, const uint32_t* blob,
                          uint32_t blob_words, uint32_t vec_floats, int first, int nlev, const float* b_first,
                          uint32_t n_first, hipStream_t s);
// fine rows [f0, f1) (multiples of 4 but f1 = L.n; f1 = 0: all)
// residual + restriction fused (k_amg_resrestrict; L.rr_agg > 0, replicated
// or single-GPU level): coarse_b = R (b - A x), coarse_x cleared or the
// coarse zero-x pre-smoother written to sm_out (as launch_amg_restrict)
void launch_amg_resrestrict(const AmgLevelDev& L, const float* x, const float* b, float* coarse_b, float* coarse_x,
                            float* sm_out, const float* sm_de, hipStream_t s);
// levels i (Lf: x, b) and i+1 (Lm) down-leg in one launch: writes level
// i+1's rhs bm and pre-smoothed x xm (as k_amg_resrestrict with sm_out), then
// level i+2's rhs cb and either its pre-smoothed x (sm_out, diagonal sm_de)
// or cx = 0 -- the bits of the two k_amg_resrestrict launches
// levels c (Lc: x xc, b bc; coarse x xcc of level c+1) and c-1 (Lf: x xf, b
// bf): writes only the fine level's post-smoothed x into xf_out -- the bits of
// the two k_amg_smooth<..., PRO> launches for the fine level
void launch_amg_prolong_smooth_pair(const AmgLevelDev& Lf, const AmgLevelDev& Lc, const AmgUpPairImage& P,
                                    const float* xf, const float* bf, float* xf_out, const float* xc,
                                    const float* bc, const float* xcc, hipStream_t s);
void launch_amg_resrestrict_pair(const AmgLevelDev& Lf, const AmgLevelDev& Lm, const AmgPairImage& P,
                                 const float* x, const float* b, float* bm, float* xm, float* cb, float* cx,
                                 float* sm_out, const float* sm_de, hipStream_t s);
void launch_amg_prolong(const AmgLevelDev& L, float* x, const float* coarse_x, hipStream_t s, uint32_t f0 = 0,
                        uint32_t f1 = 0, bool nt = false);
// Sets the tail kernels' dynamic-LDS attribute on `device` (once per device,
// thread-safe; throws on failure) and returns their LDS budget there:
// min(kTailLdsMax, the device's opt-in per-block LDS).  Call with `device` current.
size_t init_kernel_attributes(int device);
// check_evolution (coupled_solver.rs:501-580) statistics in the canonical order (f64):
// chunk partials partial[f * np + k], f = {evolution, sum_u, sum_v, sumsq_u, sumsq_v}
// The variance part reads record ((gbase + c) >> 2) - rec0 of `var` (stride bug, §0.1-12).
void launch_evolution_partial(StateView cur, StateView prev, int have_prev, uint32_t N,
                              StateView var, uint64_t gbase, uint64_t rec0, uint32_t U, double* partial, uint32_t np,
                              hipStream_t s);
// ---- distributed helpers ----
void launch_pack(const PackArgs& a, hipStream_t s);
// distributed: this rank's segment values out[v * maxseg + s] of nvec reductions
// from their unit partials part[v * np + k] (k < nunits local, G units per segment)
void launch_seg_reduce(const float* part, uint32_t np, uint32_t nchunks, uint32_t G, int nvec, float* out,
                       uint32_t maxseg, hipStream_t s);
void launch_seg_reduce_d(const double* part, uint32_t np, uint32_t nchunks, uint32_t G, int nvec, double* out,
                         uint32_t maxseg, hipStream_t s);
void launch_max_combine(const uint32_t* gathered, int R, uint32_t* out, uint32_t* host_out, hipStream_t s);
// out5[f] = total of the 5 check_evolution sums (r.nvec = 5)
void launch_evolution_final(const RedSrcD& r, double* out5, hipStream_t s);

}  // namespace cfd2
