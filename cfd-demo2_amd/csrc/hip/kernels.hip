// gfx950 (MI355X / CDNA4) kernels of the coupled FV step.
//
// Every kernel is HBM-bandwidth bound (<= 0.25 flop/B): face sweeps, SpMV on
// compressed 3x3 blocks, BLAS-1 with wavefront reductions, Jacobi smoothing,
// restriction and prolongation.  No MFMA: nothing here is a dense contraction.
// Arithmetic follows the reference WGSL operation-for-operation (file:line in
// each kernel) and is compiled with -ffp-contract=off, so results are
// bit-identical to the CPU oracle; reductions follow the canonical order of
// kernels.hpp (256 threads x 4 cells per chunk, halving tree).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <mutex>
#include <stdexcept>
#include <string>

#include "kernels.hpp"

namespace cfd2 {

namespace {

// Tuning constants below are plain numbers (A/B-tuned with
// tools/ab_variants.py); every compile-time switch between two code paths
// was removed once its A/B was decided (round 4; git history keeps the losers).
//
// One basis load in flight per wavefront in the CGS kernels (load_cells3 SER)
// on meshes of at least this many cells (per rank); below it, every load of a
// wavefront stays in flight together.  With ~15+ blocks per CU the serialised
// loads win (same-box A/B at C2: update 346 -> 295, dots 294 -> 281 us); with
// ~4 blocks per CU nothing hides a wavefront's one-at-a-time loads (C1: dots
// 41.8 -> 31.0, update 40.5 -> 36.2 us unserialised; profiles/r03/ab_log.md).
#ifndef CFD_CGS_SER_MIN_CELLS
#define CFD_CGS_SER_MIN_CELLS (1u << 22)
#endif

#ifndef CFD_RED_SEGS
#define CFD_RED_SEGS 4  // independent partial loads per lane in the finishing kernels
#endif
constexpr int kBlock = 256;

__device__ __forceinline__ float wsmoothstep(float lo, float hi, float x) {
  const float t = fminf(fmaxf((x - lo) / (hi - lo), 0.0f), 1.0f);
  return t * t * (3.0f - 2.0f * t);
}
__device__ __forceinline__ float wmix(float a, float b, float t) { return a * (1.0f - t) + b * t; }
__device__ __forceinline__ float safe_inverse(float v) {
  return fabsf(v) > 1e-14f ? 1.0f / v : 0.0f;
}

// Loads of a kernel's once-read streams (matrix slots, row headers, the rows'
// own operands) with the nontemporal policy (NT: global_load ... nt) or the
// default one.  NT is chosen per launch for the kernels that are the LAST
// readers of their matrix before it is evicted anyway, so its lines do not
// displace, in the 256 MB Infinity Cache, the vectors the next kernels read
// (Solver::nt_mask).  Same bits either way.
template <bool NT, class V>
__device__ __forceinline__ V ldx(const V* p) {
  if constexpr (!NT) {
    return *p;
  } else {
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
    // f4u / f2u sources are only 4-byte aligned: their loads keep that
    // alignment instead of the vector types' natural 16 / 8 bytes
    typedef unsigned int u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));
    typedef unsigned int u32x2a4 __attribute__((ext_vector_type(2), aligned(4)));
    V r;
    if constexpr (sizeof(V) == 16 && alignof(V) >= 16) {
      const u32x4 t = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
      __builtin_memcpy(&r, &t, 16);
    } else if constexpr (sizeof(V) == 16) {
      const u32x4a4 t = __builtin_nontemporal_load(reinterpret_cast<const u32x4a4*>(p));
      __builtin_memcpy(&r, &t, 16);
    } else if constexpr (sizeof(V) == 8 && alignof(V) >= 8) {
      const u32x2 t = __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(p));
      __builtin_memcpy(&r, &t, 8);
    } else if constexpr (sizeof(V) == 8) {
      const u32x2a4 t = __builtin_nontemporal_load(reinterpret_cast<const u32x2a4*>(p));
      __builtin_memcpy(&r, &t, 8);
    } else if constexpr (sizeof(V) == 4) {
      const uint32_t t = __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(p));
      __builtin_memcpy(&r, &t, 4);
    } else if constexpr (sizeof(V) == 2) {
      const uint16_t t = __builtin_nontemporal_load(reinterpret_cast<const uint16_t*>(p));
      __builtin_memcpy(&r, &t, 2);
    } else {
      static_assert(sizeof(V) == 1, "ldx: 1, 2, 4, 8 or 16 bytes");
      const uint8_t t = __builtin_nontemporal_load(reinterpret_cast<const uint8_t*>(p));
      __builtin_memcpy(&r, &t, 1);
    }
    return r;
  }
}
// typed views for ldx of an address inside an array of another element type
template <bool NT, class V, class T>
__device__ __forceinline__ V ldv(const T* p) {
  return ldx<NT>(reinterpret_cast<const V*>(p));
}

__device__ __forceinline__ float f4(const float4& v, int k) {
  return k == 0 ? v.x : k == 1 ? v.y : k == 2 ? v.z : v.w;
}
__device__ __forceinline__ uint32_t u4(const uchar4& v, int k) {
  return k == 0 ? v.x : k == 1 ? v.y : k == 2 ? v.z : v.w;
}
// aligned-slot rows (CoupledMatrix::lg): slots in use, and whether slot r
// holds an entry of row k of the thread's 4
__device__ __forceinline__ uint32_t lg_used(const ushort4& v, int k) {
  return (k == 0 ? v.x : k == 1 ? v.y : k == 2 ? v.z : v.w) & kLgUsedMask;
}
__device__ __forceinline__ bool lg_on(const ushort4& v, int k, uint32_t r) {
  const uint32_t w = k == 0 ? v.x : k == 1 ? v.y : k == 2 ? v.z : v.w;
  return r < (w & kLgUsedMask) && !((w >> 8 >> r) & 1u);
}

inline unsigned grid_for(size_t n) { return (unsigned)((n + kBlock - 1) / kBlock); }

// XCD-aware block -> tile remap (cdna_hip_programming.md T1): the dispatcher
// deals blocks round-robin over the 8 XCDs; remapping gives XCD k a contiguous
// range of rows, so the i +- n_y neighbour gathers of a structured-ish cut-cell
// mesh hit that XCD's L2.  Bijective for any grid size; a speed choice only.
// REV: each XCD walks its range from the top down.  Blocks are dispatched in
// blockIdx order, so a kernel launched right after a forward kernel over the
// same data starts on the rows whose lines that kernel touched last, which may
// still sit in the memory-side Infinity Cache (MALL, 256 MB, shared by all
// XCDs).  Order only: every row's arithmetic is unchanged.
template <bool REV = false>
__device__ __forceinline__ uint32_t xcd_block() {
  const uint32_t b = blockIdx.x, nb = gridDim.x;
  const uint32_t xcd = b & 7u, q = nb >> 3, r = nb & 7u;
  const uint32_t base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  if constexpr (REV) return base + ((xcd < r) ? q : q - 1u) - (b >> 3);
  return base + (b >> 3);
}
template <bool REV = false>
__device__ __forceinline__ uint32_t row_id() { return xcd_block<REV>() * kBlock + threadIdx.x; }

// Kernels that run top-down (xcd_block<true>) to reuse the Infinity Cache lines
// of the kernel before them (build-time tunables, tools/ab_variants.py).  Same-box
// A/B at C2 (profiles/r01/ab_reverse_order.txt): k_amg_residual, which follows
// the pre-smoother over the same level matrix, 83.1 -> 67.4 us at level 0 when
// the two sweep in opposite directions; k_spmv, which follows k_precond_correct
// over the same cval_g / column slots, 233.5 -> 223.1 us; 278.9 -> 273.5
// ms/step.  Round 3: the smoother top-down and the residual (and the fused
// residual + restriction) bottom-up instead -- the same alternation, and now
// each smoother also runs against the bottom-up kernel before it (the Schur
// prediction writing its b and x, the prolongation): level-0 smoother 77.7 ->
// 74.7 us, C2 -1.0 / -1.25 ms/step in two same-box pairs
// (profiles/r03/ab_rev_schur_early_c2.txt, ab_early_operands_c2.txt).  The CGS
// update after the dots gains nothing (its nontemporal basis reads do not stay
// in the MALL, and temporal ones cost 20 %), so the CGS kernels keep one direction.
constexpr bool kRevSpmv = true;       // k_spmv2: top-down, after the bottom-up Schur correction
constexpr bool kRevResidual = false;  // k_amg_residual / k_amg_resrestrict: bottom-up
constexpr bool kRevSmooth = true;     // k_amg_smooth: top-down

// First row of this thread's 4 in a launch over [r0, r1) and [r2, r3) (the
// second range lets a distributed rank process both boundary strips of a
// halo'd kernel in one launch); false: no rows for this thread.
template <bool REV = false>
__device__ __forceinline__ bool row_range(uint32_t r0, uint32_t r1, uint32_t r2, uint32_t r3, uint32_t& i0) {
  const uint32_t t = row_id<REV>(), na = (r1 - r0 + 3) / 4;
  if (t < na) {
    i0 = r0 + 4 * t;
    return i0 < r1;
  }
  i0 = r2 + 4 * (t - na);
  return i0 < r3;
}
inline unsigned rows2_grid(uint32_t r0, uint32_t r1, uint32_t r2, uint32_t r3) {
  const size_t t = (size_t)(r1 - r0 + 3) / 4 + (r3 > r2 ? (size_t)(r3 - r2 + 3) / 4 : 0);
  return (unsigned)((t + 255) / 256);
}

// ---- canonical reduction order (kernels.hpp: leaf / chunk / segment / total) ----
// Pairwise tree over the first `active` lanes of the wavefront (a power of
// two <= 64); lane 0 holds the root.  Lane l adds lane l + s at strides
// s = 1, 2, ...: at every level each surviving node is (left + right).
template <class T>
__device__ __forceinline__ T wave_tree(T v, uint32_t active = 64) {
  for (uint32_t st = 1; st < active; st <<= 1) v = v + __shfl_down(v, st);
  return v;
}
// chunk of this wavefront in a reduction kernel (4 chunks per 256-thread block)
__device__ __forceinline__ uint32_t red_chunk() { return blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6); }
__device__ __forceinline__ uint32_t red_lane() { return threadIdx.x & 63; }

// Segment values of U consecutive-in-steps segments s0, s0 + sstep, ... from
// chunk partials pv[k] (k < nchunks, missing chunks +0): lane l holds chunk
// slots [l K, l K + K) of the segment, K = min(4, G / 64) ... (G <= 256).
template <class T, int U>
__device__ __forceinline__ void seg_trees(const T* __restrict__ pv, uint32_t nchunks, uint32_t G, uint32_t s0,
                                          uint32_t sstep, uint32_t nseg, T out[U]) {
  const uint32_t lane = red_lane();
  const uint32_t K = G >= 256 ? 4u : (G >= 128 ? 2u : 1u);
  const uint32_t L = G / K;  // active lanes (power of two)
  T e[U][4];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint32_t sg = s0 + u * sstep;
    const uint64_t k0 = (uint64_t)sg * G + (uint64_t)lane * K;
    if constexpr (sizeof(T) == 4) {
      // 4 chunk slots in one 16-byte load (per-vector strides are multiples of 4)
      if (K == 4 && sg < nseg && k0 + 3 < nchunks) {
        const float4 q = *reinterpret_cast<const float4*>(pv + k0);
        e[u][0] = q.x;
        e[u][1] = q.y;
        e[u][2] = q.z;
        e[u][3] = q.w;
        continue;
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint64_t k = k0 + q;
      e[u][q] = (sg < nseg && lane < L && (uint32_t)q < K && k < nchunks) ? pv[k] : T(0);
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    T v;
    if (K == 4)
      v = (e[u][0] + e[u][1]) + (e[u][2] + e[u][3]);
    else if (K == 2)
      v = e[u][0] + e[u][1];
    else
      v = e[u][0];
    out[u] = wave_tree(v, L);
  }
}

__host__ __device__ __forceinline__ uint32_t pow2_ceil(uint32_t n) {
  uint32_t p = 1;
  while (p < n) p <<= 1;
  return p;
}

// Segment values of one vector's unit partials pv[0, nunits) into LDS a[0, P)
// (P = pow2 >= nseg; segments past nseg are +0): segment sg = pairwise tree over
// its GU unit values pv[sg GU ..] (missing units +0).  A group of LS = GU / K
// lanes serves one segment, each lane K = min(4, GU) consecutive units (one
// 16-byte load when K = 4), then the tree over the group's lanes.  A wavefront
// iterates as a whole, so every shuffle reads a live lane.
template <class T, int NT>
__device__ __forceinline__ void seg_values(const T* __restrict__ pv, uint32_t nunits, uint32_t GU, uint32_t nseg,
                                           uint32_t P, T* a) {
  const uint32_t K = GU >= 4 ? 4u : GU;
  const uint32_t LS = GU / K;
  const uint32_t slots = P * LS;  // a multiple of 64 when >= 64
  constexpr int R = CFD_RED_SEGS;  // independent loads in flight per lane
  for (uint32_t base = threadIdx.x & ~63u; base < slots; base += R * NT) {
    T e[R][4];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint32_t t = base + r * NT + red_lane();
      const uint32_t sg = t / LS;
      const uint64_t k0 = (uint64_t)sg * GU + (uint64_t)(t % LS) * K;
      if constexpr (sizeof(T) == 4) {
        if (K == 4 && sg < nseg && k0 + 3 < nunits) {
          const float4 q = *reinterpret_cast<const float4*>(pv + k0);
          e[r][0] = q.x;
          e[r][1] = q.y;
          e[r][2] = q.z;
          e[r][3] = q.w;
          continue;
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q)
        e[r][q] = (sg < nseg && (uint32_t)q < K && k0 + q < nunits) ? pv[k0 + q] : T(0);
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      T v = K == 4 ? (e[r][0] + e[r][1]) + (e[r][2] + e[r][3]) : (K == 2 ? e[r][0] + e[r][1] : e[r][0]);
      for (uint32_t st = 1; st < LS; st <<= 1) v = v + __shfl_down(v, st);
      const uint32_t t = base + r * NT + red_lane();
      if (t < slots && t % LS == 0) a[t / LS] = v;
    }
  }
}

// Pairwise tree over a[0, P) (P a power of two <= kRedMaxSegments): blocks of
// 64 by wavefront trees, then the <= 64 block values by one wavefront -- the
// same bits as halving level by level.  b needs 65 entries.  Every thread
// returns the total.
template <class T, int NT>
__device__ __forceinline__ T total_tree(const T* a, uint32_t P, T* b) {
  constexpr uint32_t NW = NT / 64;
  const uint32_t w = threadIdx.x >> 6, lane = red_lane();
  __syncthreads();  // a[] complete
  uint32_t Q = P;
  const T* src = a;
  if (P > 64) {
    for (uint32_t gi = w; gi < P / 64; gi += NW) {
      const T v = wave_tree(a[64 * gi + lane], 64);
      if (lane == 0) b[gi] = v;
    }
    __syncthreads();
    Q = P / 64;
    src = b;
  }
  if (w == 0) {
    const T v = wave_tree(lane < Q ? src[lane] : T(0), Q);
    if (lane == 0) b[64] = v;
  }
  __syncthreads();
  const T tot = b[64];
  __syncthreads();  // the caller may reuse the LDS
  return tot;
}

// The 64-wide halving tree of the reference's workgroup reductions (stride
// 32 .. 1: lane l adds lane l + stride, gmres_ops.wgsl:177-182) as one
// wavefront's shuffles -- the same pairs, lane 0 holds the result.
template <class T>
__device__ __forceinline__ T ref_tree64(T v) {
  for (int st = 32; st > 0; st >>= 1) v = v + __shfl_down(v, st);
  return v;
}

// Reference reduction order (RedSrcT::order, test mode): the total of vector v
// from the reference's 64-DOF group partials.  Every thread returns it.
template <class T, int NT>
__device__ __forceinline__ T ref_total(const RedSrcT<T>& r, uint32_t v, T* b) {
  const T* p = r.p + (size_t)v * r.stride;
  __syncthreads();
  if (r.order == 1) {  // reduce_final: one thread, the partials in order
    if (threadIdx.x == 0) {
      T s = T(0);
      for (uint32_t k = 0; k < r.nchunks; ++k) s += p[k];
      b[64] = s;
    }
  } else if (threadIdx.x < 64) {  // reduce_dots_cgs: strided lane sums, then the tree
    T s = T(0);
    for (uint32_t k = threadIdx.x; k < r.nchunks; k += 64) s += p[k];
    s = ref_tree64(s);
    if (threadIdx.x == 0) b[64] = s;
  }
  __syncthreads();
  const T tot = b[64];
  __syncthreads();  // the caller may reuse the LDS
  return tot;
}

// Total of vector v of reduction r by the whole block (NT threads): the
// segment values into LDS a[0, P) (+0 padding to P = pow2 >= nseg), then the
// pairwise tree over them.  Every thread returns the total.
template <class T, int NT>
__device__ __forceinline__ T red_total(const RedSrcT<T>& r, uint32_t v, T* a, T* b) {
  if (r.order) return ref_total<T, NT>(r, v, b);
  const uint32_t P = pow2_ceil(r.nseg);
  if (r.seg_src) {  // distributed: gathered segment values
    const size_t blk = (size_t)r.nvec * r.stride;
    for (uint32_t sg = threadIdx.x; sg < P; sg += NT) {
      T val = T(0);
      if (sg < r.nseg) {
        const uint32_t src = r.seg_src[sg];
        val = r.p[(size_t)(src >> 20) * blk + (size_t)v * r.stride + (src & 0xFFFFFu)];
      }
      a[sg] = val;
    }
  } else {  // one GPU: segment trees of the unit partials
    seg_values<T, NT>(r.p + (size_t)v * r.stride, r.nchunks, r.G, r.nseg, P, a);
  }
  return total_tree<T, NT>(a, P, b);
}
#ifndef CFD_RED_FINAL_THREADS
#define CFD_RED_FINAL_THREADS 1024
#endif
constexpr int kRedFinalThreads = CFD_RED_FINAL_THREADS;

// ---------------------------------------------------------------------------
// prepare_coupled.wgsl:63-348 — Rhie-Chow face flux, d_p, Green-Gauss grads.
// Snapshot semantics: reads st (pre-kernel), writes d_p/grad_p to dp_out/gp_out.
// prepare_cell: cell i's face fluxes (stored) and its new d_p, grad_p, grad_u,
// grad_v (returned; k_prepare stores them, k_prepare_ordered after a barrier)
__device__ __forceinline__ void prepare_cell(const PrepareArgs& a, uint32_t i, float& dp_new, float2& gp_new,
                                             float2& gu_new, float2& gv_new) {
  const uint32_t N = a.N;
  const cfd_constants c = a.c;
  const FaceSlots fs = a.fs;
  const float vol = a.vol[i];
  float diag_coeff = 0.0f;
  float time_coeff = vol * c.density / c.dt;
  if (c.time_scheme == 1u) {
    const float r = c.dt / c.dt_old;
    time_coeff = vol * c.density / c.dt * (1.0f + 2.0f * r) / (1.0f + r);
  }
  diag_coeff += time_coeff;
  const float2 uc = a.st.u[i];
  const float pc = a.st.p[i];
  const float dpc = a.st.dp[i];
  const float2 gpc = a.st.gp[i];
  float gpx = 0.0f, gpy = 0.0f, gux = 0.0f, guy = 0.0f, gvx = 0.0f, gvy = 0.0f;
  const uint32_t nf = fs.nface[i];
  for (uint32_t k = 0; k < nf; ++k) {
    const size_t e = (size_t)k * N + i;
    const uint32_t meta = fs.meta[e];
    const int32_t other = fs.other[e];
    const uint32_t bt = meta & kMetaBtypeMask;
    const bool own = (meta & kMetaOwner) != 0;
    const float area = fs.area[e];
    const float nx = fs.nx[e], ny = fs.ny[e];  // oriented out of this cell
    // stored face normal, then prepare's geometric re-orientation (wgsl:122-130)
    const float Nx = own ? nx : -nx, Ny = own ? ny : -ny;
    const bool flip = (meta & kMetaFluxFlip) != 0;
    const float nfx = flip ? -Nx : Nx, nfy = flip ? -Ny : Ny;
    float flux = 0.0f;
    float po_other = 0.0f;
    float2 uo = make_float2(0.0f, 0.0f);
    if (other != kNoCell) {
      const float2 u_oth = a.st.u[other];
      const float p_oth = a.st.p[other];
      const float dp_oth = a.st.dp[other];
      const float2 gp_oth = a.st.gp[other];
      uo = u_oth;
      po_other = p_oth;
      const float2 uow = own ? uc : u_oth, ung = own ? u_oth : uc;
      const float pow_ = own ? pc : p_oth, png = own ? p_oth : pc;
      const float dpow = own ? dpc : dp_oth, dpng = own ? dp_oth : dpc;
      const float2 gpow = own ? gpc : gp_oth, gpng = own ? gp_oth : gpc;
      const float lambda = fs.lam_f[e];
      const float ufx = lambda * uow.x + (1.0f - lambda) * ung.x;
      const float ufy = lambda * uow.y + (1.0f - lambda) * ung.y;
      const float dp_face = lambda * dpow + (1.0f - lambda) * dpng;
      const float gfx = lambda * gpow.x + (1.0f - lambda) * gpng.x;
      const float gfy = lambda * gpow.y + (1.0f - lambda) * gpng.y;
      const float dist = fs.dist_a[e];
      const float grad_p_n = gfx * nfx + gfy * nfy;
      const float p_grad_f = (png - pow_) / dist;
      const float rc_term = dp_face * area * (grad_p_n - p_grad_f);
      const float u_n = ufx * nfx + ufy * nfy;
      flux = c.density * (u_n * area + rc_term);
    } else if (bt == 1u) {
      const float ramp = wsmoothstep(0.0f, c.ramp_time, c.time);
      const float ubx = c.inlet_velocity * ramp, uby = 0.0f;
      flux = c.density * (ubx * nfx + uby * nfy) * area;
    } else if (bt == 2u) {
      const float u_n = uc.x * nfx + uc.y * nfy;  // boundary faces are owned by this cell
      const float raw = c.density * u_n * area;
      flux = fmaxf(0.0f, raw);
    }
    const float flux_out = own ? flux : -flux;
    a.flux_s[e] = flux_out;
    const float diff_coeff = c.viscosity * area / fs.dist_e[e];
    const float conv_diag = flux_out > 0.0f ? flux_out : 0.0f;
    if (other != kNoCell) {
      diag_coeff += diff_coeff + conv_diag;
    } else if (bt == 1u || bt == 3u) {
      diag_coeff += diff_coeff;
      if (flux_out > 0.0f) diag_coeff += flux_out;
    } else if (bt == 2u) {
      if (flux_out > 0.0f) diag_coeff += flux_out;
    }
    float vfp, vfu, vfv;
    if (other != kNoCell) {
      const float lp = fs.lam_s[e];
      vfp = lp * pc + (1.0f - lp) * po_other;
      if ((meta & kMetaDegen) == 0) {
        vfu = lp * uc.x + (1.0f - lp) * uo.x;
        vfv = lp * uc.y + (1.0f - lp) * uo.y;
      } else {
        vfu = 0.5f * (uc.x + uo.x);
        vfv = 0.5f * (uc.y + uo.y);
      }
    } else {
      vfp = (bt == 2u) ? 0.0f : pc;
      if (bt == 1u) {
        const float ramp = wsmoothstep(0.0f, c.ramp_time, c.time);
        vfu = c.inlet_velocity * ramp;
        vfv = 0.0f;
      } else if (bt == 3u) {
        vfu = 0.0f;
        vfv = 0.0f;
      } else {
        vfu = uc.x;
        vfv = uc.y;
      }
    }
    gpx += vfp * nx * area;
    gpy += vfp * ny * area;
    gux += vfu * nx * area;
    guy += vfu * ny * area;
    gvx += vfv * nx * area;
    gvy += vfv * ny * area;
  }
  dp_new = (fabsf(diag_coeff) > 1e-20f) ? vol / diag_coeff : 0.0f;
  gp_new = make_float2(gpx / vol, gpy / vol);
  gu_new = make_float2(gux / vol, guy / vol);
  gv_new = make_float2(gvx / vol, gvy / vol);
}
__global__ void __launch_bounds__(kBlock) k_prepare(PrepareArgs a) {
  const uint32_t i = row_id();
  if (i >= a.N) return;
  float dp;
  float2 gp, gu, gv;
  prepare_cell(a, i, dp, gp, gu, gv);
  a.dp_out[i] = dp;
  a.gp_out[i] = gp;
  a.grad_u[i] = gu;
  a.grad_v[i] = gv;
}
// The reference's RACY prepare (prepare_coupled.wgsl:140-143 vs :328-337)
// under one legal schedule (test mode, Solver::ref_racy; oracle
// kSemRacyPrepare): the 64-cell workgroups one after another, d_p / grad_p
// written in place (dp_out == st.dp, gp_out == st.gp), every cell of a
// workgroup reading before any writes -- later workgroups read the new values.
__global__ void __launch_bounds__(64) k_prepare_ordered(PrepareArgs a) {
  for (uint32_t b0 = 0; b0 < a.N; b0 += 64) {
    const uint32_t i = b0 + threadIdx.x;
    float dp = 0.0f;
    float2 gp = make_float2(0.0f, 0.0f), gu = gp, gv = gp;
    if (i < a.N) prepare_cell(a, i, dp, gp, gu, gv);
    __syncthreads();  // the workgroup's reads complete
    if (i < a.N) {
      a.dp_out[i] = dp;
      a.gp_out[i] = gp;
      a.grad_u[i] = gu;
      a.grad_v[i] = gv;
    }
    __syncthreads();  // visible to the next workgroup
  }
}
// the assembly reads fluxes[face] as the OWNER stored it (coupled_assembly_
// merged.wgsl:153): a non-owner slot takes -(owner's flux) -- the same bits as
// its own computation under snapshot reads, not under the racy ones
__global__ void __launch_bounds__(kBlock) k_flux_mirror(float* flux_s, const int32_t* mirror, uint32_t S) {
  const uint32_t e = blockIdx.x * kBlock + threadIdx.x;
  if (e >= S) return;
  const int32_t m = mirror[e];
  if (m >= 0) flux_s[e] = -flux_s[m];  // owner slots (m < 0) are only read
}

// coupled_assembly_merged.wgsl:70-463
__global__ void __launch_bounds__(kBlock) k_assemble(AssembleArgs a) {
  const uint32_t i = row_id();
  const uint32_t N = a.N;
  if (i >= N) return;
  const cfd_constants c = a.c;
  const FaceSlots fs = a.fs;
  const float vol = a.vol[i];
  float diag_uv = 0.0f;  // diag_u == diag_v (identical update sequence)
  float sdup = 0.0f, sdvp = 0.0f, sdpu = 0.0f, sdpv = 0.0f, sdpp = 0.0f;
  float rhs_u = 0.0f, rhs_v = 0.0f, rhs_p = 0.0f, sdiag = 0.0f;
  const float2 un = a.u_old[i];
  float coeff_time = vol * c.density / c.dt;
  float rtu = coeff_time * un.x, rtv = coeff_time * un.y;
  if (c.time_scheme == 1u) {
    const float dt = c.dt, dt_old = c.dt_old;
    const float r = dt / dt_old;
    const float2 unm1 = a.u_old_old[i];
    coeff_time = vol * c.density / dt * (1.0f + 2.0f * r) / (1.0f + r);
    const float fn = (1.0f + r);
    const float fnm1 = (r * r) / (1.0f + r);
    rtu = (vol * c.density / dt) * (fn * un.x - fnm1 * unm1.x);
    rtv = (vol * c.density / dt) * (fn * un.y - fnm1 * unm1.y);
  }
  diag_uv += coeff_time;
  rhs_u += rtu;
  rhs_v += rtv;
  const float dpc = a.st.dp[i];
  const float2 uc = a.st.u[i];
  const uint32_t nf = fs.nface[i];
  for (uint32_t k = 0; k < nf; ++k) {
    const size_t e = (size_t)k * N + i;
    const uint32_t meta = fs.meta[e];
    const int32_t other = fs.other[e];
    const uint32_t bt = meta & kMetaBtypeMask;
    const float area = fs.area[e];
    const float nx = fs.nx[e], ny = fs.ny[e];
    const float flux = a.flux_s[e];
    const float dist = fs.dist_a[e];
    const float diff_coeff = c.viscosity * area / dist;
    const float conv_diag = flux > 0.0f ? flux : 0.0f;
    const float conv_off = flux > 0.0f ? 0.0f : flux;
    if (other != kNoCell) {
      const uint32_t rank = (meta >> kMetaRankShift) & 0xFFu;
      const float dp_other = a.st.dp[other];
      const float coeff = -diff_coeff + conv_off;
      diag_uv += diff_coeff + conv_diag;
      if (c.scheme != 0u) {
        const float2 uo = a.st.u[other];
        float pu_u = uc.x, pu_v = uc.y;
        if (flux < 0.0f) {
          pu_u = uo.x;
          pu_v = uo.y;
        }
        float ph_u = pu_u, ph_v = pu_v;
        if (c.scheme == 1u) {
          if (flux > 0.0f) {
            const float2 gu = a.grad_u[i], gv = a.grad_v[i];
            const float rx = fs.rx[e], ry = fs.ry[e];
            ph_u = uc.x + (gu.x * rx + gu.y * ry);
            ph_v = uc.y + (gv.x * rx + gv.y * ry);
          } else {
            const float2 gu = a.grad_u[other], gv = a.grad_v[other];
            const float rx = fs.rox[e], ry = fs.roy[e];
            ph_u = uo.x + (gu.x * rx + gu.y * ry);
            ph_v = uo.y + (gv.x * rx + gv.y * ry);
          }
        } else if (c.scheme == 2u) {
          if (flux > 0.0f) {
            const float2 gu = a.grad_u[i], gv = a.grad_v[i];
            const float dx = fs.dvx[e], dy = fs.dvy[e];
            const float gtu = gu.x * dx + gu.y * dy, gtv = gv.x * dx + gv.y * dy;
            ph_u = 0.625f * uc.x + 0.375f * uo.x + 0.125f * gtu;
            ph_v = 0.625f * uc.y + 0.375f * uo.y + 0.125f * gtv;
          } else {
            const float2 gu = a.grad_u[other], gv = a.grad_v[other];
            const float dx = -fs.dvx[e], dy = -fs.dvy[e];  // center - other_center
            const float gtu = gu.x * dx + gu.y * dy, gtv = gv.x * dx + gv.y * dy;
            ph_u = 0.625f * uo.x + 0.375f * uc.x + 0.125f * gtu;
            ph_v = 0.625f * uo.y + 0.375f * uc.y + 0.125f * gtv;
          }
        }
        rhs_u -= flux * (ph_u - pu_u);
        rhs_v -= flux * (ph_v - pu_v);
      }
      const float lambda = fs.lam_s[e];
      const float oml = 1.0f - lambda;
      const float pgx = area * nx, pgy = area * ny;
      sdup += lambda * pgx;
      sdvp += lambda * pgy;
      const float dcx = nx * area, dcy = ny * area;
      sdpu += lambda * dcx;
      sdpv += lambda * dcy;
      const float dp_f = lambda * dpc + (1.0f - lambda) * dp_other;
      const float lapl = dp_f * area / dist;
      sdpp += lapl;
      const float scoeff = c.density * dp_f * area / dist;
      sdiag += scoeff;
      const size_t cslot = (size_t)((meta >> kMetaTSlotShift) & 0xFFu) * a.ld + i;
      a.cval_a[cslot] = make_float2(coeff, -lapl);
      a.cval_g[cslot] = make_float2(oml * pgx, oml * pgy);
      a.sval[(size_t)rank * a.ld + i] = -scoeff;
    } else if (bt == 1u) {
      const float ramp = wsmoothstep(0.0f, c.ramp_time, c.time);
      const float ubx = c.inlet_velocity * ramp, uby = 0.0f;
      diag_uv += diff_coeff;
      rhs_u += diff_coeff * ubx;
      rhs_v += diff_coeff * uby;
      if (flux > 0.0f) {
        diag_uv += flux;
      } else {
        rhs_u -= flux * ubx;
        rhs_v -= flux * uby;
      }
      sdup += area * nx;
      sdvp += area * ny;
      const float flux_bc = (ubx * nx + uby * ny) * area;
      rhs_p -= flux_bc;
    } else if (bt == 3u) {
      diag_uv += diff_coeff;
      sdup += area * nx;
      sdvp += area * ny;
    } else if (bt == 2u) {
      if (flux > 0.0f) diag_uv += flux;
      sdpu += nx * area;
      sdpv += ny * area;
      const float lapl = dpc * area / dist;
      sdpp += lapl;
      const float scoeff = c.density * dpc * area / dist;
      sdiag += scoeff;
    }
  }
  const size_t cdslot = (size_t)a.cslot_diag[i] * a.ld + i;
  a.cval_a[cdslot] = make_float2(diag_uv, 0.0f + sdpp);
  a.cval_g[cdslot] = make_float2(sdup, sdvp);
  a.cdiag2[i] = make_float2(sdpu, sdpv);
  a.sval[(size_t)a.srank_diag[i] * a.ld + i] = sdiag;
  a.rhs[3 * (size_t)i + 0] = rhs_u;
  a.rhs[3 * (size_t)i + 1] = rhs_v;
  a.rhs[3 * (size_t)i + 2] = rhs_p;
  a.dinv_uv[i] = safe_inverse(diag_uv);
  a.dinv_p[i] = safe_inverse(sdiag);
}

// update_fields_from_coupled.wgsl:45-98.  The reference folds max|du|, max|dp|
// with one atomicMax per workgroup into a single word; here each block writes
// the max of its bit patterns (order-independent) and k_maxdiff_final folds
// them, avoiding ~40k same-address atomics per call.
__global__ void __launch_bounds__(kBlock) k_update_fields(uint32_t N, float alpha_u, float alpha_p,
                                                          const float* __restrict__ x, float2* u,
                                                          float* p, uint32_t* blockmax) {
  __shared__ uint32_t su[4], sp[4];
  const uint32_t lb = xcd_block();
  const uint32_t i = lb * kBlock + threadIdx.x;
  uint32_t bu = 0, bp = 0;
  if (i < N) {
    const float un = x[3 * (size_t)i], vn = x[3 * (size_t)i + 1], pn = x[3 * (size_t)i + 2];
    const float2 uo = u[i];
    const float po = p[i];
    const float ux = uo.x + alpha_u * (un - uo.x);
    const float uy = uo.y + alpha_u * (vn - uo.y);
    const float pu = po + alpha_p * (pn - po);
    u[i] = make_float2(ux, uy);
    p[i] = pu;
    const float du = fmaxf(fabsf(ux - uo.x), fabsf(uy - uo.y));
    const float dp = fabsf(pu - po);
    bu = __float_as_uint(du);
    bp = __float_as_uint(dp);
  }
  for (int o = 32; o >= 1; o >>= 1) {
    bu = max(bu, (uint32_t)__shfl_xor((int)bu, o));
    bp = max(bp, (uint32_t)__shfl_xor((int)bp, o));
  }
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    su[wv] = bu;
    sp[wv] = bp;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    blockmax[2 * lb] = max(max(su[0], su[1]), max(su[2], su[3]));
    blockmax[2 * lb + 1] = max(max(sp[0], sp[1]), max(sp[2], sp[3]));
  }
}

__global__ void __launch_bounds__(kBlock) k_maxdiff_final(const uint32_t* __restrict__ blockmax,
                                                          uint32_t nb, uint32_t* maxbits, uint32_t* host_out) {
  __shared__ uint32_t su[4], sp[4];
  uint32_t bu = 0, bp = 0;
  for (uint32_t q = threadIdx.x; q < nb; q += kBlock) {
    const uint2 v = *reinterpret_cast<const uint2*>(blockmax + 2 * (size_t)q);
    bu = max(bu, v.x);
    bp = max(bp, v.y);
  }
  for (int o = 32; o >= 1; o >>= 1) {
    bu = max(bu, (uint32_t)__shfl_xor((int)bu, o));
    bp = max(bp, (uint32_t)__shfl_xor((int)bp, o));
  }
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    su[wv] = bu;
    sp[wv] = bp;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    maxbits[0] = max(max(su[0], su[1]), max(su[2], su[3]));
    maxbits[1] = max(max(sp[0], sp[1]), max(sp[2], sp[3]));
    if (host_out) {  // mapped pinned host memory: the host's lagged read needs no copy
      host_out[0] = maxbits[0];
      host_out[1] = maxbits[1];
    }
  }
}

__device__ __forceinline__ void load12(const float* p, float v[12]) {  // 3 float4 = 4 rows x (u,v,p)
  const float4 a = *reinterpret_cast<const float4*>(p);
  const float4 b = *reinterpret_cast<const float4*>(p + 4);
  const float4 c = *reinterpret_cast<const float4*>(p + 8);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  v[8] = c.x; v[9] = c.y; v[10] = c.z; v[11] = c.w;
}
__device__ __forceinline__ void store12(float* p, const float v[12]) {
  *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
  *reinterpret_cast<float4*>(p + 8) = make_float4(v[8], v[9], v[10], v[11]);
}

// 3-component cell vectors in the reduction kernels (kernels.hpp: the cell
// term of a dot is (x_u y_u + x_v y_v) + x_p y_p).  Block b covers the 4
// chunks of cells [1024 b, 1024 b + 1024); lane l of wavefront w holds cell
// c_q = 1024 b + 256 q + 64 w + l of chunk q (q = 0..3), its 3 floats by one
// 12-byte access, so the block's 4 wavefronts read one chunk together (768
// contiguous bytes per instruction).  A chunk value is the pairwise tree over
// its 256 cells: each wavefront's 64 (a quarter, wave_tree), then the 4
// quarters (quarter_chunk).  Cells past N: 0.  SER: every load completes
// before the next issues -- for these kernels, which stream up to 51 vectors
// at once, measured faster than keeping a wavefront's loads in flight
// together (same-box A/B at C2: CGS update 349 -> 294 us, dots 300 -> 289).
__device__ __forceinline__ size_t cell_qb(uint32_t b, uint32_t q) {
  return (size_t)b * 1024u + 256u * q + (threadIdx.x & ~63u) + red_lane();
}
__device__ __forceinline__ size_t cell_q(uint32_t q) { return cell_qb(blockIdx.x, q); }
template <bool FULL, bool NT = false, bool SER = false>
__device__ __forceinline__ void load_cells3(const float* p, uint32_t N, float v[4][3], uint32_t b = ~0u) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const size_t c = cell_qb(b == ~0u ? blockIdx.x : b, q);
    if (FULL || c < N) {
#pragma unroll
      for (int e = 0; e < 3; ++e) {
        if constexpr (NT)
          v[q][e] = __builtin_nontemporal_load(p + 3 * c + e);
        else
          v[q][e] = p[3 * c + e];
      }
      if constexpr (SER) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      v[q][0] = v[q][1] = v[q][2] = 0.0f;
    }
  }
}
template <bool FULL, bool NT = true>
__device__ __forceinline__ void store_cells3_stream(float* p, uint32_t N, const float v[4][3], uint32_t b = ~0u) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const size_t c = cell_qb(b == ~0u ? blockIdx.x : b, q);
    if (FULL || c < N) {
#pragma unroll
      for (int e = 0; e < 3; ++e) {
        if constexpr (NT)
          __builtin_nontemporal_store(v[q][e], p + 3 * c + e);
        else
          p[3 * c + e] = v[q][e];
      }
    }
  }
}
__device__ __forceinline__ float cell_dot3(const float a[3], const float b[3]) {
  return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2];
}
// wave_tree(v, 64) without LDS traffic: strides 1..8 by DPP row shifts (lane
// l adds lane l + s of its row of 16; only lanes whose chain stays inside the
// row are read), strides 16 and 32 from the row roots by lane reads -- the
// same additions in the same order.  Valid in every lane.
template <int S>
__device__ __forceinline__ float row_down(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x100 + S, 0xF, 0xF, true));
}
__device__ __forceinline__ float wave_tree64(float v) {
  v = v + row_down<1>(v);
  v = v + row_down<2>(v);
  v = v + row_down<4>(v);
  v = v + row_down<8>(v);
  const float r0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
  const float r1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16));
  const float r2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
  const float r3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48));
  return (r0 + r1) + (r2 + r3);
}
// quarters of the block's chunks: lds[4 q + w] = wave_tree of wavefront w's
// cell terms t[q] (written by lane 0)
__device__ __forceinline__ void quarter_trees(const float t[4], float* lds) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float r = wave_tree64(t[q]);
    if (red_lane() == 0) lds[4 * q + (threadIdx.x >> 6)] = r;
  }
}
// chunk q's value from its 4 quarter values (pairwise)
__device__ __forceinline__ float quarter_chunk(const float* l, int q) {
  return (l[4 * q] + l[4 * q + 1]) + (l[4 * q + 2] + l[4 * q + 3]);
}
// Units of the block's 4 chunk values l[0..3] (kernels.hpp): unit u of U chunks
// = the pairwise tree over them
template <class T>
__device__ __forceinline__ T unit_value(const T* l, uint32_t U, uint32_t u) {
  if (U == 4) return (l[0] + l[1]) + (l[2] + l[3]);
  if (U == 2) return l[2 * u] + l[2 * u + 1];
  return l[u];
}
// ... from the 16 quarter values ql[4 q + w] of the block's chunks
__device__ __forceinline__ float unit_value_q(const float* ql, uint32_t U, uint32_t u) {
  float l[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) l[q] = quarter_chunk(ql, q);
  return unit_value(l, U, u);
}
// the block's chunks are all inside the mesh
__device__ __forceinline__ bool block_full(uint32_t N, uint32_t b = ~0u) {
  return (size_t)((b == ~0u ? blockIdx.x : b) + 1) * 4u * kRedChunkCells <= N;
}

// unit partials of dot(x, y) over 3-component cells
__global__ void __launch_bounds__(kBlock) k_dot_partial(const float* __restrict__ x,
                                                        const float* __restrict__ y, uint32_t N, uint32_t U,
                                                        float* partial) {
  __shared__ float lds[16];
  float a[4][3], b[4][3], t[4];
  load_cells3<false>(x, N, a);
  load_cells3<false>(y, N, b);
#pragma unroll
  for (int q = 0; q < 4; ++q) t[q] = cell_dot3(a[q], b[q]);
  quarter_trees(t, lds);
  __syncthreads();
  const uint32_t UB = 4 / U, unit = blockIdx.x * UB + threadIdx.x;
  if (threadIdx.x < UB && (size_t)unit * U * kRedChunkCells < N) partial[unit] = unit_value_q(lds, U, threadIdx.x);
}

// Reference-order group partials (test mode, launch_ref_norm_partials /
// launch_ref_cgs_dots): one wavefront per 64-DOF group, four per block.
__global__ void __launch_bounds__(256) k_ref_norm_partials(const float* __restrict__ v, uint32_t n3,
                                                          float* partial, uint32_t ng) {
  const uint32_t g = blockIdx.x * 4 + (threadIdx.x >> 6), l = threadIdx.x & 63;
  const size_t i = (size_t)g * 64 + l;
  float x = 0.0f;
  if (i < n3) {
    const float a = v[i];
    x = a * a;  // norm_sq_partial: val * val
  }
  x = ref_tree64(x);
  if (l == 0 && g < ng) partial[g] = x;
}
__global__ void __launch_bounds__(256) k_ref_cgs_dots(const float* __restrict__ w, const float* __restrict__ basis,
                                                     const float* __restrict__ binv, size_t stride, uint32_t n3,
                                                     float* partial, uint32_t pstride, uint32_t ng) {
  const uint32_t g = blockIdx.x * 4 + (threadIdx.x >> 6), l = threadIdx.x & 63, ii = blockIdx.y;
  const size_t i = (size_t)g * 64 + l;
  float x = 0.0f;
  if (i < n3) {
    const float vv = binv[ii] * basis[(size_t)ii * stride + i];  // V_ii as the reference's scale stored it
    x = vv * w[i];                                               // calc_dots_cgs: v * w_val
  }
  x = ref_tree64(x);
  if (l == 0 && g < ng) partial[(size_t)ii * pstride + g] = x;
}

// norm outputs of a finished dot: mode 1: out = sqrt(s); mode 2: also inv, g0
__device__ __forceinline__ void norm_out(float s, int mode, float* out, float* inv, float* g0, float* host_out) {
  const float nrm = sqrtf(s);
  out[0] = nrm;
  if (host_out) host_out[0] = nrm;  // mapped pinned host memory: the host's read needs no copy
  if (mode == 2) {
    inv[0] = 1.0f / nrm;  // host-side `1.0 / residual_norm` (coupled_solver_fgmres.rs:1872)
    if (g0) g0[0] = nrm;
  }
}

// g_len > 0 (mode 2): g = [||r||, 0, ..., 0] of length g_len (the zero fill of
// coupled_solver_fgmres.rs:1880-1890 done here instead of a separate fill)
__global__ void __launch_bounds__(kRedFinalThreads) k_reduce_final(RedSrc r, int mode, float* out, float* inv,
                                                                   float* g0, int g_len, float* host_out) {
  __shared__ float la[kRedMaxSegments], lb[65];
  const float s = red_total<float, kRedFinalThreads>(r, 0, la, lb);
  if (g0)
    for (int k = 1 + (int)threadIdx.x; k < g_len; k += kRedFinalThreads) g0[k] = 0.0f;
  if (threadIdx.x == 0) norm_out(s, mode, out, inv, g0, host_out);
}

// Gathers of the row kernels.  Unused ELL slots and padding rows hold the
// row's own (valid) index, so a gather can be issued unconditionally
// (ALWAYS): no branch per load; the value of an unused slot is never consumed
// (every accumulation skips r >= len), so results are unchanged.  Same-box
// A/B (round 1, C2): k_amg_smooth 84 -> 81 us; k_amg_residual keeps the
// predicated form on its MODE 0 levels.
template <bool ALWAYS = false>
__device__ __forceinline__ float gat(bool on, const float* p) {
  if constexpr (ALWAYS) {
    (void)on;
    return *p;
  } else {
    return on ? *p : 0.0f;
  }
}

// Vector gathers: the columns of one slot for consecutive rows are, for
// every interior row of a face stencil, consecutive cells (c, c+1, ...): one
// 16-byte load (dword-aligned: gfx950 global loads need only 4-byte alignment
// for multi-dword accesses) fetches them all, and only threads whose slot is
// not consecutive (boundary / cut cells) issue the per-row loads.  Cuts the
// gather instructions per wave ~4x for scalar vectors (the row kernels are
// VMEM-issue bound: SQ_WAIT_INST_ANY ~0.5-0.7 of wave cycles,
// tools/gpu_sq.sh; round 1: level-0 smoother 84 -> 78 us, Schur predict
// 198 -> 185, correct 166 -> 159).  Every vector read this way has >= 64
// floats of padding past its last (ghost) entry.
typedef float f4u __attribute__((ext_vector_type(4), aligned(4)));
typedef float f2u __attribute__((ext_vector_type(2), aligned(4)));
__device__ __forceinline__ f2u ld2u(const float* p) { return *reinterpret_cast<const f2u*>(p); }
__device__ __forceinline__ f4u ld4u(const float* p) { return *reinterpret_cast<const f4u*>(p); }
__device__ __forceinline__ bool consec4(const int c[4]) {
  return c[1] == c[0] + 1 && c[2] == c[0] + 2 && c[3] == c[0] + 3;
}


// Slot-group sizes of the coupled row kernels (all loads of a group are
// issued before the first use).  Build-time tunables (tools/ab_variants.py).
#ifndef CFD_SPMV_U
#define CFD_SPMV_U 4
#endif
#ifndef CFD_PREDICT_U
#define CFD_PREDICT_U 4
#endif
#ifndef CFD_CORRECT_U
#define CFD_CORRECT_U 4
#endif

// Slot loads of the row kernels are unconditional: slot r reads ELL slot
// min(r, ws - 1) (ws = the matrix's ELL width, kernel-uniform), which always
// exists; unused slots hold value 0 and the row's own column, and every
// accumulation skips r >= len, so results are unchanged.  Without a branch
// per slot the compiler issues a whole group's matrix loads back to back
// (a predicated load per slot made it wait for each slot's column load
// before issuing the next slot), and the first group does not wait for the
// row lengths.  The first group (U1) is sized to cover a whole interior row
// (5 entries of a quad cell's coupled row).
// SpMV: the first slot group's cval_a / cval_g loads are issued with the row
// headers, before the wait for them (C2 216 -> 197 us; the same for the
// Schur prediction lost 150 -> 158 us: profiles/r03/ab_coupled_pre_c2.txt;
// the regular rows' x gathers issued speculatively as well gained nothing
// more, 198 -> 200 us: ab_spmv_spec_c2.txt)
#ifndef CFD_SPMV_U1
#define CFD_SPMV_U1 5
#endif

// The coupled row kernels (SpMV, Schur predict / correct) take 2 cells (6
// rows) per thread: half the registers per slot group of the 4-cell form
// (102 instead of 196 VGPRs: 4 wavefronts per SIMD instead of 2), one 16-byte
// load per slot array; same-box A/B at C2 (round 2): SpMV 225.8 -> 218.0 us.
template <bool REV = false>
__device__ __forceinline__ bool row_range2(uint32_t r0, uint32_t r1, uint32_t r2, uint32_t r3, uint32_t& i0) {
  const uint32_t t = row_id<REV>(), na = (r1 - r0 + 1) / 2;
  if (t < na) {
    i0 = r0 + 2 * t;
    return i0 < r1;
  }
  i0 = r2 + 2 * (t - na);
  return i0 < r3;
}
inline unsigned rows2x_grid(uint32_t r0, uint32_t r1, uint32_t r2, uint32_t r3) {
  const size_t t = (size_t)(r1 - r0 + 1) / 2 + (r3 > r2 ? (size_t)(r3 - r2 + 1) / 2 : 0);
  return (unsigned)((t + 255) / 256);
}
// the two rows' columns of slot offset `off`
template <bool D16, bool NT = false>
__device__ __forceinline__ void ccols2(const CoupledMatrix& A, size_t off, uint32_t i0, int c[2]) {
  if constexpr (D16) {
    const short2 d = ldv<NT, short2>(A.col16 + off);
    c[0] = (int)i0 + (int)d.x;
    c[1] = (int)i0 + 1 + (int)d.y;
  } else {
    const int2 q = ldv<NT, int2>(A.col + off);
    c[0] = q.x;
    c[1] = q.y;
  }
}
__device__ __forceinline__ bool lg2_on(uint32_t w, uint32_t r) { return r < (w & kLgUsedMask) && !((w >> 8 >> r) & 1u); }
// REG (first slot group of a wave of regular rows, r0 = 0): columns
// row + tmode[slot] (no column loads), and the two rows' x entries are six
// consecutive floats (one 16-byte + one 8-byte gather)
// PRE: the group's cval_a / cval_g slots were loaded by the caller (first
// group: issued right after the row headers, before the wait for them)
template <bool D16, int U, bool REG = false, bool PRE = false, bool NT = false>
__device__ __forceinline__ void spmv2_group(const CoupledMatrix& A, const float* __restrict__ x, uint32_t i0,
                                            uint32_t r0, uint32_t rmax, const uint32_t lw[2], const uint32_t dr[2],
                                            const float2 d2[2], float su[2], float sv[2], float sp[2],
                                            const float4* pa = nullptr, const float4* pg = nullptr) {
  float4 a[U], g[U];
  int c[U][2];
  float xg[U][2][3];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const size_t off = (size_t)min(r0 + u, rmax) * A.ld + i0;
    if constexpr (PRE) {
      a[u] = pa[u];
      g[u] = pg[u];
    } else {
      a[u] = ldv<NT, float4>(A.cval_a + off);
      g[u] = ldv<NT, float4>(A.cval_g + off);
    }
    if constexpr (REG) {
      c[u][0] = (int)i0 + A.tmode[u];
      c[u][1] = c[u][0] + 1;
    } else {
      ccols2<D16, NT>(A, off, i0, c[u]);
    }
  }
  if constexpr (REG) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const float* b = x + 3 * (ptrdiff_t)c[u][0];
      const f4u q0 = ld4u(b);
      const f2u q1 = ld2u(b + 4);
      xg[u][0][0] = q0.x;
      xg[u][0][1] = q0.y;
      xg[u][0][2] = q0.z;
      xg[u][1][0] = q0.w;
      xg[u][1][1] = q1.x;
      xg[u][1][2] = q1.y;
    }
  } else {
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const ptrdiff_t j = 3 * (ptrdiff_t)c[u][k];
        xg[u][k][0] = x[j];
        xg[u][k][1] = x[j + 1];
        xg[u][k][2] = x[j + 2];
      }
  }
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const uint32_t r = r0 + u;
      if (!lg2_on(lw[k], r)) continue;
      const bool dg = (r == dr[k]);
      const float uu = k ? a[u].z : a[u].x, pp = k ? a[u].w : a[u].y;
      const float up = k ? g[u].z : g[u].x, vp = k ? g[u].w : g[u].y;
      const float pu = dg ? d2[k].x : up, pv = dg ? d2[k].y : vp;
      const float xu = xg[u][k][0], xv = xg[u][k][1], xp = xg[u][k][2];
      su[k] += uu * xu;
      su[k] += 0.0f * xv;
      su[k] += up * xp;
      sv[k] += 0.0f * xu;
      sv[k] += uu * xv;
      sv[k] += vp * xp;
      sp[k] += pu * xu;
      sp[k] += pv * xv;
      sp[k] += pp * xp;
    }
}
// the two rows' slot headers (u16) and diagonal slots (u8).  Packing both
// into one u32 per row (one load fewer) lost at C2: SpMV 208 -> 213, Schur
// prediction 155 -> 160 us (profiles/r03/ab_log.md) -- 2 bytes more per row
// cost more than the instruction saved.
template <bool NT = false>
__device__ __forceinline__ void row2_headers(const CoupledMatrix& A, uint32_t i0, uint32_t lw[2], uint32_t dr[2]) {
  const ushort2 lg = ldv<NT, ushort2>(A.lg + i0);
  const uchar2 drr = ldv<NT, uchar2>(A.drank + i0);
  lw[0] = lg.x;
  lw[1] = lg.y;
  dr[0] = drr.x;
  dr[1] = drr.y;
}
// b != null: y = 1 * b + -1 * (A x), the residual's axpby (gmres_ops.wgsl:108-117)
// applied to each output element as it is stored (compute_residual_into: the
// product itself is not needed)
template <bool D16, bool NT>
__global__ void __launch_bounds__(kBlock) k_spmv2(CoupledMatrix A, const float* __restrict__ x,
                                                  float* __restrict__ y, const float* __restrict__ b) {
  constexpr int U = CFD_SPMV_U, U1 = CFD_SPMV_U1;
  uint32_t i0;
  if (!row_range2<kRevSpmv>(A.r0, A.r1, A.r2, A.r3, i0)) return;
  uint32_t lw[2], dr[2];
  row2_headers<NT>(A, i0, lw, dr);
  const float4 dd = ldv<NT, float4>(A.cdiag2 + i0);
  const float2 d2[2] = {make_float2(dd.x, dd.y), make_float2(dd.z, dd.w)};
  const uint32_t maxlen = max(lw[0] & kLgUsedMask, lw[1] & kLgUsedMask);
  float su[2] = {0.0f, 0.0f}, sv[2] = {0.0f, 0.0f}, sp[2] = {0.0f, 0.0f};
  // the first slot group's values issued with the row headers (see CFD_SPMV_U1)
  float4 pa[U1], pg[U1];
#pragma unroll
  for (int u = 0; u < U1; ++u) {
    const size_t off = (size_t)min((uint32_t)u, (uint32_t)A.ws - 1u) * A.ld + i0;
    pa[u] = ldv<NT, float4>(A.cval_a + off);
    pg[u] = ldv<NT, float4>(A.cval_g + off);
  }
  if (A.reg && A.ws <= U1 && __all((lw[0] & lw[1] & kLgRegular) != 0u))  // ws <= U1: the only group
    spmv2_group<D16, U1, true, true, NT>(A, x, i0, 0, (uint32_t)A.ws - 1u, lw, dr, d2, su, sv, sp, pa, pg);
  else
    spmv2_group<D16, U1, false, true, NT>(A, x, i0, 0, (uint32_t)A.ws - 1u, lw, dr, d2, su, sv, sp, pa, pg);
  for (uint32_t r0 = U1; r0 < maxlen; r0 += U)
    spmv2_group<D16, U, false, false, NT>(A, x, i0, r0, maxlen - 1u, lw, dr, d2, su, sv, sp);
  float* yo = y + 3 * (size_t)i0;  // 8-byte aligned (i0 even)
  typedef float f2v __attribute__((ext_vector_type(2)));
  if (b) {
    const float* bo = b + 3 * (size_t)i0;
    const f4u b4 = ldv<NT, f4u>(bo);
    const f2u b2 = ldv<NT, f2u>(bo + 4);
    *reinterpret_cast<f4u*>(yo) = f4u{1.0f * b4.x + -1.0f * su[0], 1.0f * b4.y + -1.0f * sv[0],
                                      1.0f * b4.z + -1.0f * sp[0], 1.0f * b4.w + -1.0f * su[1]};
    *reinterpret_cast<f2v*>(yo + 4) = f2v{1.0f * b2.x + -1.0f * sv[1], 1.0f * b2.y + -1.0f * sp[1]};
    return;
  }
  *reinterpret_cast<f4u*>(yo) = f4u{su[0], sv[0], sp[0], su[1]};
  *reinterpret_cast<f2v*>(yo + 4) = f2v{sv[1], sp[1]};
}

// calc_dots_cgs (gmres_cgs.wgsl:28-82): partial[ii * np + unit] = <w, V_ii>, ii = 0..j,
// V_ii = binv[ii] * W_ii, in the cell layout of load_cells3; quarter values
// ql[16 ii + 4 q + w] in LDS, units at the end.
template <bool FULL, bool SER, bool NTB = true>
__device__ __forceinline__ void cgs_dots_cells(const float* __restrict__ w, const float* __restrict__ basis,
                                               const float* __restrict__ binv, size_t stride, int j, uint32_t N,
                                               float* ql) {
  float wv[4][3];
  load_cells3<FULL>(w, N, wv);
  for (int ii = 0; ii <= j; ++ii) {
    const float sc = binv[ii];
    float v[4][3], t[4];
    load_cells3<FULL, NTB, SER>(basis + (size_t)ii * stride, N, v);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
#pragma unroll
      for (int e = 0; e < 3; ++e) v[q][e] = sc * v[q][e];
      t[q] = cell_dot3(wv[q], v[q]);
    }
    quarter_trees(t, ql + 16 * ii);
  }
}
template <bool SER>
__global__ void __launch_bounds__(kBlock) k_cgs_dots(const float* __restrict__ w,
                                                     const float* __restrict__ basis,
                                                     const float* __restrict__ binv, size_t stride,
                                                     int j, uint32_t N, uint32_t U, float* partial, uint32_t np,
                                                     uint32_t tb) {
  __shared__ float ql[16 * 64];
  // blocks from tb on read the basis with the default policy: their lines stay
  // in the Infinity Cache for the update, which walks the blocks top-down
  if (blockIdx.x < tb) {
    if (block_full(N))
      cgs_dots_cells<true, SER>(w, basis, binv, stride, j, N, ql);
    else
      cgs_dots_cells<false, SER>(w, basis, binv, stride, j, N, ql);
  } else {
    if (block_full(N))
      cgs_dots_cells<true, SER, false>(w, basis, binv, stride, j, N, ql);
    else
      cgs_dots_cells<false, SER, false>(w, basis, binv, stride, j, N, ql);
  }
  __syncthreads();
  const uint32_t UB = 4 / U;
  for (uint32_t idx = threadIdx.x; idx < (uint32_t)(j + 1) * UB; idx += kBlock) {
    const uint32_t ii = idx / UB, u = idx % UB, unit = blockIdx.x * UB + u;
    if ((size_t)unit * U * kRedChunkCells < N) partial[(size_t)ii * np + unit] = unit_value_q(ql + 16 * ii, U, u);
  }
}

// Latency form of the CGS passes for small meshes (round 5): with a few
// blocks on a mostly idle chip each basis vector's loads are a dependent
// round trip of their own when the loop over ii issues one vector at a time,
// so C0's dots / update ran ≈ 10 / 12 us for ≈ 1 us of bytes.  Here KB
// vectors are loaded together before any of them is used, and the dots are
// spread over blockIdx.y (KB vectors per block, w read by each): the same
// cell terms, quarter trees and unit values per vector and chunk, the update's
// corrections accumulated in ii order as before.
#ifndef CFD_CGS_LAT_MAX_CELLS
#define CFD_CGS_LAT_MAX_CELLS (1u << 17)
#endif
constexpr int kCgsLatDots = 4, kCgsLatUpdate = 20;
template <bool FULL, int KB>
__device__ __forceinline__ void cgs_dots_cells_batch(const float* __restrict__ w, const float* __restrict__ basis,
                                                     const float* __restrict__ binv, size_t stride, int ii0, int j,
                                                     uint32_t N, float* ql) {
  float wv[4][3], v[KB][4][3];
  load_cells3<FULL>(w, N, wv);
#pragma unroll
  for (int k = 0; k < KB; ++k) load_cells3<FULL>(basis + (size_t)min(ii0 + k, j) * stride, N, v[k]);
#pragma unroll
  for (int k = 0; k < KB; ++k) {
    if (ii0 + k > j) break;
    const float sc = binv[ii0 + k];
    float t[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
#pragma unroll
      for (int e = 0; e < 3; ++e) v[k][q][e] = sc * v[k][q][e];
      t[q] = cell_dot3(wv[q], v[k][q]);
    }
    quarter_trees(t, ql + 16 * k);
  }
}
__global__ void __launch_bounds__(kBlock) k_cgs_dots_lat(const float* __restrict__ w,
                                                         const float* __restrict__ basis,
                                                         const float* __restrict__ binv, size_t stride, int j,
                                                         uint32_t N, uint32_t U, float* partial, uint32_t np) {
  constexpr int KB = kCgsLatDots;
  __shared__ float ql[16 * KB];
  const int ii0 = (int)blockIdx.y * KB;
  if (block_full(N))
    cgs_dots_cells_batch<true, KB>(w, basis, binv, stride, ii0, j, N, ql);
  else
    cgs_dots_cells_batch<false, KB>(w, basis, binv, stride, ii0, j, N, ql);
  __syncthreads();
  const uint32_t UB = 4 / U, nk = (uint32_t)min(KB, j + 1 - ii0);
  for (uint32_t idx = threadIdx.x; idx < nk * UB; idx += kBlock) {
    const uint32_t k = idx / UB, u = idx % UB, unit = blockIdx.x * UB + u;
    if ((size_t)unit * U * kRedChunkCells < N) partial[(size_t)(ii0 + k) * np + unit] = unit_value_q(ql + 16 * k, U, u);
  }
}

// reduce_dots_cgs (gmres_cgs.wgsl:86-120): H[j][ii] for ii = blockIdx.x
__global__ void __launch_bounds__(kRedFinalThreads) k_cgs_reduce(RedSrc r, int j, float* H, int m1) {
  __shared__ float la[kRedMaxSegments], lb[65];
  const int ii = blockIdx.x;
  const float s = red_total<float, kRedFinalThreads>(r, (uint32_t)ii, la, lb);
  if (threadIdx.x == 0) H[(size_t)j * m1 + ii] = s;
}

// update_w_cgs (gmres_cgs.wgsl:125-166) fused with the ||w||^2 unit partial; the
// updated w is written straight into basis slot j+1 (unnormalised, see binv).
// NTB: nontemporal basis loads and store of the new vector (the default);
// false when the whole basis stays in the caches (small meshes, see
// launch_cgs_update_norm)
template <bool FULL, bool SER, bool NTB>
__device__ __forceinline__ void cgs_update_cells(const float* __restrict__ w, float* basis, size_t stride, int j,
                                                 const float* hcol, const float* scol, uint32_t N, float t[4],
                                                 uint32_t b) {
  float corr[4][3] = {};
  for (int ii = 0; ii <= j; ++ii) {
    const float h = hcol[ii], sc = scol[ii];
    float v[4][3];
    load_cells3<FULL, NTB, SER>(basis + (size_t)ii * stride, N, v, b);
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int e = 0; e < 3; ++e) corr[q][e] += h * (sc * v[q][e]);
  }
  float wn[4][3];
  load_cells3<FULL>(w, N, wn, b);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
#pragma unroll
    for (int e = 0; e < 3; ++e) wn[q][e] = wn[q][e] - corr[q][e];
    t[q] = cell_dot3(wn[q], wn[q]);
  }
  store_cells3_stream<FULL, NTB>(basis + (size_t)(j + 1) * stride, N, wn, b);
}
// k_cgs_reduce's totals computed by every block of the update for itself (one
// GPU, at most 256 padded units: meshes up to ≈ 260 k cells).  The canonical
// total of a vector (red_total: segment trees of GU units, then the tree over
// the P segment values) is the pairwise tree over its unit partials padded
// with +0 to T = P GU values; here L = T / K lanes hold K = min(4, T)
// consecutive units each and a lane tree finishes it -- the same tree.  All
// (j + 1) L lane slots are loaded before any tree (RB rounds of the block in
// flight).  hcol[ii] = the total of vector ii.
template <int NT = kBlock>
__device__ __forceinline__ void cgs_reduce_local(const RedSrc& r, int j, float* hcol) {
  const uint32_t T = pow2_ceil(r.nseg) * r.G, K = T >= 4 ? 4u : T, L = T / K;
  const uint32_t slots = (uint32_t)(j + 1) * L;
  constexpr int RB = NT >= 1024 ? 1 : 4;  // 1,024 threads: one slot each per round (registers)
  for (uint32_t base = 0; base < slots; base += RB * NT) {
    float e[RB][4];
#pragma unroll
    for (int rr = 0; rr < RB; ++rr) {
      const uint32_t sl = base + rr * NT + threadIdx.x;
      const uint32_t ii = sl / L, k0 = (sl % L) * K;
      const float* pv = r.p + (size_t)ii * r.stride;
      if (K == 4 && sl < slots && k0 + 3 < r.nchunks) {  // stride and k0 multiples of 4
        const float4 q = *reinterpret_cast<const float4*>(pv + k0);
        e[rr][0] = q.x;
        e[rr][1] = q.y;
        e[rr][2] = q.z;
        e[rr][3] = q.w;
        continue;
      }
#pragma unroll
      for (uint32_t q = 0; q < 4; ++q) e[rr][q] = (sl < slots && q < K && k0 + q < r.nchunks) ? pv[k0 + q] : 0.0f;
    }
#pragma unroll
    for (int rr = 0; rr < RB; ++rr) {
      float v = K == 4 ? (e[rr][0] + e[rr][1]) + (e[rr][2] + e[rr][3]) : (K == 2 ? e[rr][0] + e[rr][1] : e[rr][0]);
      for (uint32_t st = 1; st < L; st <<= 1) v = v + __shfl_down(v, st);
      const uint32_t sl = base + rr * NT + threadIdx.x;
      if (sl < slots && sl % L == 0) hcol[sl / L] = v;
    }
  }
}

// FR: the CGS totals reduced in the kernel (cgs_reduce_local from the dots'
// unit partials fr; block 0 stores the Hessenberg column) instead of by
// k_cgs_reduce -- one launch fewer per FGMRES iteration on small meshes
template <bool SER, bool NTB = true, bool FR = false>
__global__ void __launch_bounds__(kBlock) k_cgs_update_norm(const float* __restrict__ w,
                                                            float* basis,
                                                            const float* __restrict__ binv,
                                                            size_t stride, int j,
                                                            float* __restrict__ H, int m1,
                                                            uint32_t N, uint32_t U, float* partial, int rev,
                                                            RedSrc fr) {
  __shared__ float hcol[64], scol[64], ql[16];
  const uint32_t b = rev ? gridDim.x - 1u - blockIdx.x : blockIdx.x;  // rev: top-down (after the dots)
  if constexpr (FR) {
    if (threadIdx.x <= (unsigned)j) scol[threadIdx.x] = binv[threadIdx.x];
    cgs_reduce_local(fr, j, hcol);
    __syncthreads();
    if (blockIdx.x == 0 && threadIdx.x <= (unsigned)j) H[(size_t)j * m1 + threadIdx.x] = hcol[threadIdx.x];
  } else {
    if (threadIdx.x <= (unsigned)j) {
      hcol[threadIdx.x] = H[(size_t)j * m1 + threadIdx.x];
      scol[threadIdx.x] = binv[threadIdx.x];
    }
    __syncthreads();
  }
  float t[4];
  if (block_full(N, b))
    cgs_update_cells<true, SER, NTB>(w, basis, stride, j, hcol, scol, N, t, b);
  else
    cgs_update_cells<false, SER, NTB>(w, basis, stride, j, hcol, scol, N, t, b);
  quarter_trees(t, ql);
  __syncthreads();
  const uint32_t UB = 4 / U, unit = b * UB + threadIdx.x;
  if (threadIdx.x < UB && (size_t)unit * U * kRedChunkCells < N) partial[unit] = unit_value_q(ql, U, threadIdx.x);
}

// Latency form of the update (small meshes, see k_cgs_dots_lat): blocks of
// 1,024 threads, one cell per thread -- thread t of block b holds cell
// 1024 b + t, so wavefront t / 64 holds quarter (t / 64) % 4 of chunk t / 256,
// the cells of load_cells3's quarter -- and the first kCgsLatUpdate basis
// vectors (3 floats each) loaded with w before the Hessenberg column is
// known (with FR, while the totals are reduced): one round trip for
// j < kCgsLatUpdate.  Corrections accumulated in ii order, the same norm
// quarter trees and unit values as k_cgs_update_norm.
template <bool FR>
__global__ void __launch_bounds__(1024) k_cgs_update_norm_lat(const float* __restrict__ w, float* basis,
                                                              const float* __restrict__ binv, size_t stride, int j,
                                                              float* __restrict__ H, int m1, uint32_t N, uint32_t U,
                                                              float* partial, RedSrc fr) {
  constexpr int KB = kCgsLatUpdate;
  __shared__ float hcol[64], scol[64], ql[16];
  const uint32_t t = threadIdx.x;
  const size_t c = (size_t)blockIdx.x * 1024u + t;
  const bool in = c < N;
  const size_t cc = in ? c : 0;
  float wn[3], v[KB][3];
#pragma unroll
  for (int e = 0; e < 3; ++e) wn[e] = w[3 * cc + e];
#pragma unroll
  for (int k = 0; k < KB; ++k)
#pragma unroll
    for (int e = 0; e < 3; ++e) v[k][e] = basis[(size_t)min(k, j) * stride + 3 * cc + e];
  if (t <= (unsigned)j) scol[t] = binv[t];
  if constexpr (FR) {
    cgs_reduce_local<1024>(fr, j, hcol);
  } else {
    if (t <= (unsigned)j) hcol[t] = H[(size_t)j * m1 + t];
  }
  __syncthreads();
  if constexpr (FR) {
    if (blockIdx.x == 0 && t <= (unsigned)j) H[(size_t)j * m1 + t] = hcol[t];
  }
  float corr[3] = {0.0f, 0.0f, 0.0f};
#pragma unroll
  for (int k = 0; k < KB; ++k) {
    if (k <= j) {  // predicated, not a break: v stays in registers
      const float h = hcol[k], sc = scol[k];
#pragma unroll
      for (int e = 0; e < 3; ++e) corr[e] += h * (sc * v[k][e]);
    }
  }
  for (int ii0 = KB; ii0 <= j; ii0 += KB) {  // j >= KB: further batches
#pragma unroll
    for (int k = 0; k < KB; ++k)
#pragma unroll
      for (int e = 0; e < 3; ++e) v[k][e] = basis[(size_t)min(ii0 + k, j) * stride + 3 * cc + e];
#pragma unroll
    for (int k = 0; k < KB; ++k) {
      if (ii0 + k <= j) {
        const float h = hcol[ii0 + k], sc = scol[ii0 + k];
#pragma unroll
        for (int e = 0; e < 3; ++e) corr[e] += h * (sc * v[k][e]);
      }
    }
  }
  float tq = 0.0f;  // cells past N: 0 (load_cells3's zero cells)
  if (in) {
#pragma unroll
    for (int e = 0; e < 3; ++e) wn[e] = wn[e] - corr[e];
    tq = cell_dot3(wn, wn);
#pragma unroll
    for (int e = 0; e < 3; ++e) basis[(size_t)(j + 1) * stride + 3 * c + e] = wn[e];
  }
  const float r = wave_tree64(tq);
  if (red_lane() == 0) ql[t >> 6] = r;
  __syncthreads();
  const uint32_t UB = 4 / U, unit = blockIdx.x * UB + t;
  if (t < UB && (size_t)unit * U * kRedChunkCells < N) partial[unit] = unit_value_q(ql, U, t);
}

// reduce_final_and_finish_norm (gmres_ops.wgsl:270-293) + update_hessenberg_givens
// (gmres_logic.wgsl:24-76).
__global__ void __launch_bounds__(kRedFinalThreads) k_norm_givens(RedSrc r, int j, float* H, int m1,
                                                                  float* givens, float* g, float* binv,
                                                                  float* resid_hist, float* host_resid) {
  __shared__ float la[kRedMaxSegments], lb[65];
  // Hessenberg column j and the rotations so far, staged in LDS by the block
  // (issued before the reduction): the serial Givens chain then makes LDS
  // round trips instead of dependent global ones
  float* Hc = H + (size_t)j * m1;
  float hv = 0.0f, gva = 0.0f, gvb = 0.0f;
  const uint32_t t = threadIdx.x;
  if (t <= (uint32_t)j) hv = Hc[t];
  if (t < (uint32_t)j) {
    gva = givens[2 * t];
    gvb = givens[2 * t + 1];
  }
  const float s = red_total<float, kRedFinalThreads>(r, 0, la, lb);  // ends with a barrier
  float* hc = la;         // [j + 2]
  float* gv = la + 128;   // [2 j]
  if (t <= (uint32_t)j) hc[t] = hv;
  if (t < (uint32_t)j) {
    gv[2 * t] = gva;
    gv[2 * t + 1] = gvb;
  }
  __syncthreads();
  if (t != 0) return;
  // norm_givens_out's operations, on the staged values
  const float norm = sqrtf(s);
  hc[j + 1] = norm;
  binv[j + 1] = norm > 1e-20f ? 1.0f / norm : 0.0f;
  for (int ii = 0; ii < j; ++ii) {
    const float hij = hc[ii], hi1j = hc[ii + 1];
    const float cc = gv[2 * ii], ss = gv[2 * ii + 1];
    hc[ii] = cc * hij + ss * hi1j;
    hc[ii + 1] = -ss * hij + cc * hi1j;
  }
  const float hjj = hc[j], hj1j = hc[j + 1];
  float cc = 1.0f, ss = 0.0f;
  const float rho = sqrtf(hjj * hjj + hj1j * hj1j);
  if (fabsf(rho) > 1e-20f) {
    cc = hjj / rho;
    ss = hj1j / rho;
  }
  givens[2 * j] = cc;
  givens[2 * j + 1] = ss;
  hc[j] = rho;
  hc[j + 1] = 0.0f;
  for (int ii = 0; ii <= j + 1; ++ii) Hc[ii] = hc[ii];
  const float gj = g[j], gj1 = g[j + 1];
  g[j] = cc * gj + ss * gj1;
  const float gn = -ss * gj + cc * gj1;
  g[j + 1] = gn;
  resid_hist[j] = fabsf(gn);
  // the host's lag-model read (coupled_solver.rs:326-435): written straight into
  // pinned host memory, so no copy is enqueued per iteration
  if (host_resid) host_resid[0] = fabsf(gn);
}

#ifndef CFD_PREDICT_U1
#define CFD_PREDICT_U1 5
#endif

// Every relax_pressure sweep of one preconditioner application in ONE
// workgroup (small meshes, N < 8192): the p_iters launches of k_relax_pressure4
// (64 at the reference's 8 k-cell benchmark mesh, each a ~4.6 us launch for a
// few microseconds of work) become one kernel.  Thread t owns rows t + 1024 k;
// its rows' off-diagonal entries (values + LDS byte addresses of their
// columns, compacted in slot order: the diagonal is skipped as in
// k_relax_pressure4), temp_p and dinv_p live in registers for all sweeps; the
// two ping-pong iterates live in LDS (P = p_sol at byte 0, T = temp at byte
// 32768: a sweep's source buffer is an immediate offset; unit-stride rows keep
// the neighbour reads free of bank conflicts).  Sweep s reads the iterate
// written by sweep s-1 (P for even s, T for odd) and writes the other buffer,
// exactly the launch sequence's src/dst alternation; one barrier per sweep
// orders it.  Unused entries point at a zero row with value +0: they add
// +0 * +0 = +0 to sigma, which starts at +0 and so is never -0 (a
// round-to-nearest sum is -0 only if both operands are), hence sigma + +0 ==
// sigma bit for bit -- the f32 result of k_relax_pressure4, without a compare
// and select per entry.
constexpr int kRelaxThreads = 1024;
template <int RPT, int OD>
__global__ void __launch_bounds__(kRelaxThreads) k_relax_pressure_fused(uint32_t N, uint32_t ld,
                                                                      const int32_t* __restrict__ col,
                                                                      const uint32_t* __restrict__ len,
                                                                      const float* __restrict__ sval,
                                                                      const float* __restrict__ dinv_p,
                                                                      const float* __restrict__ temp_p,
                                                                      float* p_sol, float* temp, uint32_t iters) {
  extern __shared__ float relax_lds[];  // P [0, 8192), T [8192, 16384); row N of each = +0
  char* base = reinterpret_cast<char*>(relax_lds);
  constexpr uint32_t kT = 4u * kRelaxFusedMaxRows + 4u;  // byte offset of T (32768)
  const uint32_t t = threadIdx.x;
  float dv[RPT], tp[RPT], v[RPT][OD];
  // own rows of both iterates (P: own[0], T: own[1]) also live in registers:
  // a sweep's mix operand (the destination's previous value, written by this
  // thread two sweeps earlier) is read from them, not from LDS
  float own[2][RPT];
  uint32_t ad[RPT][OD];
#pragma unroll
  for (int k = 0; k < RPT; ++k) {
    const uint32_t i = t + (uint32_t)k * kRelaxThreads;
    dv[k] = tp[k] = own[0][k] = own[1][k] = 0.0f;
#pragma unroll
    for (int e = 0; e < OD; ++e) {
      v[k][e] = 0.0f;
      ad[k][e] = 4u * N;  // the zero row
    }
    if (i < N) {
      own[0][k] = relax_lds[i] = p_sol[i];
      own[1][k] = relax_lds[kT / 4 + i] = temp[i];
      dv[k] = dinv_p[i];
      tp[k] = temp_p[i];
      const uint32_t l = len[i];
      int e = 0;
#pragma unroll
      for (int r = 0; r <= OD; ++r) {  // <= OD off-diagonals + the diagonal
        if ((uint32_t)r < l) {
          const size_t slot = (size_t)r * ld + i;
          const int32_t cc = col[slot];
          if (cc != (int32_t)i) {
            // e only ever increases by one: a static select chain keeps v / ad in registers
#pragma unroll
            for (int q = 0; q < OD; ++q)
              if (q == e) {
                v[k][q] = sval[slot];
                ad[k][q] = 4u * (uint32_t)cc;
              }
            ++e;
          }
        }
      }
    }
  }
  if (t == 0) relax_lds[N] = relax_lds[kT / 4 + N] = 0.0f;
  __syncthreads();
  // SRC = byte offset of the source iterate (0: P, kT: T)
  auto sweep = [&](auto src_off) {
    constexpr uint32_t SRC = decltype(src_off)::value, DST = kT - SRC;
    constexpr int DI = DST == 0 ? 0 : 1;
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
      // rows past N compute on the zero row: +0 entries, dv = tp = own = +0, so
      // they write mix(+0, +0, 1.2) = +0 back into it (branch-free sweep)
      const uint32_t i = min(t + (uint32_t)k * kRelaxThreads, N);
      float sigma = 0.0f;
#pragma unroll
      for (int e = 0; e < OD; ++e) sigma += v[k][e] * *reinterpret_cast<const float*>(base + ad[k][e] + SRC);
      const float hat_x = dv[k] * (tp[k] - sigma);
      // own row: only this thread touches it in this sweep
      own[DI][k] = wmix(own[DI][k], hat_x, 1.2f);
      *reinterpret_cast<float*>(base + 4u * i + DST) = own[DI][k];
    }
    __syncthreads();
  };
  uint32_t s = 0;
  for (; s + 1 < iters; s += 2) {
    sweep(std::integral_constant<uint32_t, 0u>{});
    sweep(std::integral_constant<uint32_t, kT>{});
  }
  if (s < iters) sweep(std::integral_constant<uint32_t, 0u>{});
#pragma unroll
  for (int k = 0; k < RPT; ++k) {
    const uint32_t i = t + (uint32_t)k * kRelaxThreads;
    if (i < N) {
      p_sol[i] = own[0][k];
      temp[i] = own[1][k];
    }
  }
}

#ifndef CFD_CORRECT_U1
#define CFD_CORRECT_U1 5
#endif

// ---- Schur predict / correct, 2 cells per thread ----
// The row operands of the Schur kernels are loaded with the row header, not
// after the slot loop: the prediction's dinv_p, the correction's V_j,
// dinv_uv and own p_sol -- one dependent round trip fewer per wave.
// Same-box A/B at C2 (profiles/r03/ab_rev_schur_early_c2.txt): prediction
// 152.3 -> 144.9, correction 135.8 -> 132.4 us, 254.8 -> 253.1 ms/step;
// C1 39.95 -> 39.22.
template <bool D16, int U, bool REG = false, bool NT = false>  // REG: see spmv2_group
__device__ __forceinline__ void predict2_group(const CoupledMatrix& A, const float* __restrict__ w_in, float sc,
                                               const float* __restrict__ dinv_uv, uint32_t i0, uint32_t r0,
                                               uint32_t rmax, const uint32_t lw[2], const uint32_t dr[2],
                                               const float2 d2[2], float rhs[2]) {
  float4 g[U];
  int c[U][2];
  float gd[U][2], gu[U][2], gv[U][2];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const size_t off = (size_t)min(r0 + u, rmax) * A.ld + i0;
    g[u] = ldv<NT, float4>(A.cval_g + off);
    if constexpr (REG) {
      c[u][0] = (int)i0 + A.tmode[u];
      c[u][1] = c[u][0] + 1;
    } else {
      ccols2<D16, NT>(A, off, i0, c[u]);
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {  // 2 consecutive cells: 8 + 24 bytes
    const f2u d = ld2u(dinv_uv + c[u][0]);
    const float* b = w_in + 3 * (ptrdiff_t)c[u][0];
    const f4u q0 = ld4u(b);
    const f2u q1 = ld2u(b + 4);
    gd[u][0] = d.x;
    gd[u][1] = d.y;
    gu[u][0] = q0.x;
    gv[u][0] = q0.y;
    gu[u][1] = q0.w;
    gv[u][1] = q1.x;
  }
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (c[u][1] != c[u][0] + 1) {
      const ptrdiff_t j = 3 * (ptrdiff_t)c[u][1];
      gd[u][1] = dinv_uv[c[u][1]];
      gu[u][1] = w_in[j];
      gv[u][1] = w_in[j + 1];
    }
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const uint32_t r = r0 + u;
      if (!lg2_on(lw[k], r)) continue;
      const bool dg = (r == dr[k]);
      const float gx = k ? g[u].z : g[u].x, gy = k ? g[u].w : g[u].y;
      const float pu = dg ? d2[k].x : gx, pv = dg ? d2[k].y : gy;
      const float ru = sc * gu[u][k], rv = sc * gv[u][k];
      const float zu = ru * gd[u][k];
      const float zv = rv * gd[u][k];
      rhs[k] -= pu * zu;
      rhs[k] -= pv * zv;
    }
}
template <bool D16, bool NT>
__global__ void __launch_bounds__(kBlock) k_precond_predict2(CoupledMatrix A, const float* __restrict__ w_in,
                                                             const float* __restrict__ binv, int jv,
                                                             const float* __restrict__ dinv_uv,
                                                             const float* __restrict__ dinv_p, float* temp_p,
                                                             float* p_sol, float* p_prev) {
  constexpr int U = CFD_PREDICT_U, U1 = CFD_PREDICT_U1;
  uint32_t i0;
  if (!row_range2(A.r0, A.r1, A.r2, A.r3, i0)) return;
  const float sc = binv[jv];
  const float* wb = w_in + 3 * (size_t)i0;
  const f4u wa = ld4u(wb);
  const f2u wc = ld2u(wb + 4);
  float rhs[2] = {sc * wa.z, sc * wc.y};
  uint32_t lw[2], dr[2];
  row2_headers<NT>(A, i0, lw, dr);
  const float4 dd = ldv<NT, float4>(A.cdiag2 + i0);
  const float2 d2[2] = {make_float2(dd.x, dd.y), make_float2(dd.z, dd.w)};
  const float2 dp = ldv<NT, float2>(dinv_p + i0);
  const uint32_t maxlen = max(lw[0] & kLgUsedMask, lw[1] & kLgUsedMask);
  if (A.reg && A.ws <= U1 && __all((lw[0] & lw[1] & kLgRegular) != 0u))  // ws <= U1: the only group
    predict2_group<D16, U1, true, NT>(A, w_in, sc, dinv_uv, i0, 0, (uint32_t)A.ws - 1u, lw, dr, d2, rhs);
  else
    predict2_group<D16, U1, false, NT>(A, w_in, sc, dinv_uv, i0, 0, (uint32_t)A.ws - 1u, lw, dr, d2, rhs);
  for (uint32_t r0 = U1; r0 < maxlen; r0 += U)
    predict2_group<D16, U, false, NT>(A, w_in, sc, dinv_uv, i0, r0, maxlen - 1u, lw, dr, d2, rhs);
  *reinterpret_cast<float2*>(temp_p + i0) = make_float2(rhs[0], rhs[1]);
  *reinterpret_cast<float2*>(p_sol + i0) = make_float2(dp.x * rhs[0], dp.y * rhs[1]);
  if (p_prev) *reinterpret_cast<float2*>(p_prev + i0) = make_float2(0.0f, 0.0f);
}
template <bool D16, int U, bool REG = false>  // REG: see spmv2_group
__device__ __forceinline__ void correct2_group(const CoupledMatrix& A, const float* __restrict__ p_sol, uint32_t i0,
                                               uint32_t r0, uint32_t rmax, const uint32_t lw[2], float cu[2],
                                               float cv[2]) {
  float4 g[U];
  int c[U][2];
  float pj[U][2];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const size_t off = (size_t)min(r0 + u, rmax) * A.ld + i0;
    g[u] = *reinterpret_cast<const float4*>(A.cval_g + off);
    if constexpr (REG) {
      c[u][0] = (int)i0 + A.tmode[u];
      c[u][1] = c[u][0] + 1;
    } else {
      ccols2<D16>(A, off, i0, c[u]);
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const f2u q = ld2u(p_sol + c[u][0]);
    pj[u][0] = q.x;
    pj[u][1] = q.y;
  }
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (c[u][1] != c[u][0] + 1) pj[u][1] = p_sol[c[u][1]];
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      if (!lg2_on(lw[k], r0 + u)) continue;
      cu[k] += (k ? g[u].z : g[u].x) * pj[u][k];
      cv[k] += (k ? g[u].w : g[u].y) * pj[u][k];
    }
}
template <bool D16>
__global__ void __launch_bounds__(kBlock) k_precond_correct2(CoupledMatrix A, const float* __restrict__ w_in,
                                                             const float* __restrict__ binv, int jv,
                                                             const float* __restrict__ p_sol,
                                                             const float* __restrict__ dinv_uv,
                                                             float* __restrict__ z) {
  constexpr int U = CFD_CORRECT_U, U1 = CFD_CORRECT_U1;
  uint32_t i0;
  if (!row_range2(A.r0, A.r1, A.r2, A.r3, i0)) return;
  const ushort2 lg = *reinterpret_cast<const ushort2*>(A.lg + i0);
  // the row pair's own operands issued with the header (no round trip after the slots)
  const float sc = binv[jv];
  const float* wb = w_in + 3 * (size_t)i0;
  const f4u wa = ld4u(wb);
  const f2u wc = ld2u(wb + 4);
  const float2 du = *reinterpret_cast<const float2*>(dinv_uv + i0);
  const float2 ps = *reinterpret_cast<const float2*>(p_sol + i0);
  const uint32_t lw[2] = {lg.x, lg.y};
  const uint32_t maxlen = max(lw[0] & kLgUsedMask, lw[1] & kLgUsedMask);
  float cu[2] = {0.0f, 0.0f}, cv[2] = {0.0f, 0.0f};
  if (A.reg && A.ws <= U1 && __all((lw[0] & lw[1] & kLgRegular) != 0u))  // ws <= U1: the only group
    correct2_group<D16, U1, true>(A, p_sol, i0, 0, (uint32_t)A.ws - 1u, lw, cu, cv);
  else
    correct2_group<D16, U1>(A, p_sol, i0, 0, (uint32_t)A.ws - 1u, lw, cu, cv);
  for (uint32_t r0 = U1; r0 < maxlen; r0 += U) correct2_group<D16, U>(A, p_sol, i0, r0, maxlen - 1u, lw, cu, cv);
  const float wo[6] = {wa.x, wa.y, wa.z, wa.w, wc.x, wc.y};
  const float dk[2] = {du.x, du.y}, pk[2] = {ps.x, ps.y};
  float o[6];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const float ru = sc * wo[3 * k], rv = sc * wo[3 * k + 1];
    const float zu = dk[k] * ru, zv = dk[k] * rv;
    o[3 * k] = zu - dk[k] * cu[k];
    o[3 * k + 1] = zv - dk[k] * cv[k];
    o[3 * k + 2] = pk[k];
  }
  float* zo = z + 3 * (size_t)i0;
  typedef float f2v __attribute__((ext_vector_type(2)));
  *reinterpret_cast<f4u*>(zo) = f4u{o[0], o[1], o[2], o[3]};
  *reinterpret_cast<f2v*>(zo + 4) = f2v{o[4], o[5]};
}

// solve_triangular (gmres_logic.wgsl:78-104), single lane
// H's first k columns and g are staged in LDS by the whole block, then one
// lane runs the reference's back substitution from LDS (the same operations
// in the same order; every H / y access was a dependent global round trip)
__global__ void __launch_bounds__(256) k_solve_triangular(const float* H, const float* g, float* y, int k, int m1) {
  __shared__ float hs[64 * 64], gs[64], ys[64];
  for (int e = threadIdx.x; e < k * m1; e += blockDim.x) hs[e] = H[e];
  if (threadIdx.x < (unsigned)k) gs[threadIdx.x] = g[threadIdx.x];
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int li = 0; li < k; ++li) {
      const int i = k - 1 - li;
      float sum = gs[i];
      // unrolled: the LDS loads of 8 terms issue together, only the
      // subtractions form the chain (same operations, same order)
#pragma unroll 8
      for (int jj = i + 1; jj < k; ++jj) sum -= hs[jj * m1 + i] * ys[jj];
      const float diag = hs[i * m1 + i];
      ys[i] = (fabsf(diag) > 1e-12f) ? sum / diag : 0.0f;
    }
  }
  __syncthreads();
  if (threadIdx.x < (unsigned)k) y[threadIdx.x] = ys[threadIdx.x];
}

// the preconditioned vectors Z_i are read once per restart cycle here (nontemporal)
__device__ __forceinline__ float4 ld4_upd(const float* p) { return ldv<true, float4>(p); }
template <bool SER>
__device__ __forceinline__ void upd_wait() {
  if constexpr (SER) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// basis_size x axpy_from_y (gmres_ops.wgsl:96-105) fused: x = y_i * z_i + x, i ascending
// SER: one Z load in flight per thread, on meshes of at least
// CFD_CGS_SER_MIN_CELLS cells (A/B C2: 614 -> 583 us)
template <bool SER>
__global__ void __launch_bounds__(kBlock) k_update_x(float* x, const float* __restrict__ z,
                                                     size_t stride, const float* __restrict__ y,
                                                     int k, size_t n) {
  const size_t e = 4 * ((size_t)blockIdx.x * kBlock + threadIdx.x);
  if (e >= n) return;
  if (e + 3 < n) {  // 4 elements per thread, 16-byte loads (slots are 256-byte aligned)
    float4 xv = *reinterpret_cast<const float4*>(x + e);
    int ii = 0;
    for (; ii + 1 < k; ii += 2) {
      const float4 z0 = ld4_upd(z + (size_t)ii * stride + e);
      upd_wait<SER>();
      const float4 z1 = ld4_upd(z + (size_t)(ii + 1) * stride + e);
      upd_wait<SER>();
      const float y0 = y[ii], y1 = y[ii + 1];
      xv.x = y0 * z0.x + xv.x;
      xv.y = y0 * z0.y + xv.y;
      xv.z = y0 * z0.z + xv.z;
      xv.w = y0 * z0.w + xv.w;
      xv.x = y1 * z1.x + xv.x;
      xv.y = y1 * z1.y + xv.y;
      xv.z = y1 * z1.z + xv.z;
      xv.w = y1 * z1.w + xv.w;
    }
    if (ii < k) {
      const float4 z0 = ld4_upd(z + (size_t)ii * stride + e);
      const float y0 = y[ii];
      xv.x = y0 * z0.x + xv.x;
      xv.y = y0 * z0.y + xv.y;
      xv.z = y0 * z0.z + xv.z;
      xv.w = y0 * z0.w + xv.w;
    }
    *reinterpret_cast<float4*>(x + e) = xv;
    return;
  }
  for (size_t f = e; f < n; ++f) {
    float xv = x[f];
    for (int ii = 0; ii < k; ++ii) xv = y[ii] * z[(size_t)ii * stride + f] + xv;
    x[f] = xv;
  }
}

// Latency form (small meshes, as the CGS passes': k_cgs_dots_lat): 16 of the
// Z vectors' loads issued per round trip instead of 2, the updates applied in
// ascending i as above -- same operations.
__global__ void __launch_bounds__(kBlock) k_update_x_lat(float* x, const float* __restrict__ z, size_t stride,
                                                         const float* __restrict__ y, int k, size_t n) {
  constexpr int KB = 16;
  const size_t e = 4 * ((size_t)blockIdx.x * kBlock + threadIdx.x);
  if (e >= n) return;
  if (e + 3 < n) {
    float4 xv = *reinterpret_cast<const float4*>(x + e);
    for (int ii0 = 0; ii0 < k; ii0 += KB) {
      float4 zb[KB];
#pragma unroll
      for (int q = 0; q < KB; ++q) zb[q] = *reinterpret_cast<const float4*>(z + (size_t)min(ii0 + q, k - 1) * stride + e);
#pragma unroll
      for (int q = 0; q < KB; ++q) {
        if (ii0 + q < k) {
          const float yq = y[ii0 + q];
          xv.x = yq * zb[q].x + xv.x;
          xv.y = yq * zb[q].y + xv.y;
          xv.z = yq * zb[q].z + xv.z;
          xv.w = yq * zb[q].w + xv.w;
        }
      }
    }
    *reinterpret_cast<float4*>(x + e) = xv;
    return;
  }
  for (size_t f = e; f < n; ++f) {
    float xv = x[f];
    for (int ii = 0; ii < k; ++ii) xv = y[ii] * z[(size_t)ii * stride + f] + xv;
    x[f] = xv;
  }
}

// ------------------------------- AMG ---------------------------------------
// Each thread owns 4 consecutive rows: b, x, de and every ELL slot are one
// 16-byte load per thread (coalesced 1 KiB per wavefront), column deltas are
// 8 bytes per slot, lengths 4 bytes; only the x gathers are scalar.
template <bool D16, bool NT = false>
__device__ __forceinline__ void load_cols4(const AmgLevelDev& L, size_t off, uint32_t i0,
                                           int c[4]) {
  if constexpr (D16) {
    const short4 d = ldv<NT, short4>(L.col16 + off);
    c[0] = (int)i0 + (int)d.x;
    c[1] = (int)i0 + 1 + (int)d.y;
    c[2] = (int)i0 + 2 + (int)d.z;
    c[3] = (int)i0 + 3 + (int)d.w;
  } else {
    const int4 q = ldv<NT, int4>(L.col32 + off);
    c[0] = q.x;
    c[1] = q.y;
    c[2] = q.z;
    c[3] = q.w;
  }
}

// Slots are processed in groups of kU with every load of the group issued
// before the first use (val/col, then the x gathers): ~kU x more memory-level
// parallelism per wave than a slot-at-a-time loop.  Accumulation order per
// row is unchanged (slot order).  kU = 2 since round 3: same-box A/B over
// kU = 1..4 (profiles/r03/ab_amg_u_c1.txt, _c2.txt) C1 42.90 -> 42.25 ms,
// C2 260.8 -> 259.5 ms/step; the 5 M-row level 1 (7 slots) gains most
// (residual 57.3 -> 51.3 us), level 0 (5 slots) is flat.
#ifndef CFD_AMG_U
#define CFD_AMG_U 2
#endif
constexpr int kU = CFD_AMG_U;

// MODE 1 (level 0 of a quad mesh, small latency-bound levels): slot loads
// unconditional, clamped to rmax, the first group peeled so its loads do not
// wait for the row lengths, gathers unconditional (vector gathers).  MODE 0
// (the big coarse levels, whose row lengths vary): every slot load predicated
// on the thread's longest row (avoids reading the padding of short rows);
// peeled loads with predicated gathers were slower there (A/B level 1: 62
// vs 57 us).
typedef int i4u __attribute__((ext_vector_type(4), aligned(4)));

// The prolongation prolongate_op (amg.wgsl:56-75) of a fine row f, applied to
// its value as it is read: x'[f] = x[f] + (0 + 1 * xc[agg[f]]) -- the two f32
// roundings of k_amg_prolong (0 + v turns -0 into +0, the add follows).
__device__ __forceinline__ float prolonged(float xf, float xcv) { return xf + (0.0f + 1.0f * xcv); }

// PRO: every gathered x value is the prolonged one (k_amg_smooth<..., true>):
// agg is gathered with the same columns as x (a 16-byte load where x is), then
// the coarse values -- one more dependent round trip instead of a launch.
template <bool D16, int MODE, bool ALWAYS = false, bool PRO = false, bool NT = false>
__device__ __forceinline__ void gather_group(const AmgLevelDev& L, const float* __restrict__ x,
                                             uint32_t i0, uint32_t r0, uint32_t rmax, const uchar4 ln,
                                             float4 v[kU], float xg[kU][4],
                                             const float* __restrict__ xc = nullptr) {
  int c[kU][4];
#pragma unroll
  for (int u = 0; u < kU; ++u) {
    if (MODE != 0 || r0 + u <= rmax) {
      const size_t off = (size_t)min(r0 + u, rmax) * L.stride + i0;
      v[u] = ldv<NT, float4>(L.val + off);
      load_cols4<D16, NT>(L, off, i0, c[u]);
    } else {
      v[u] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
#pragma unroll
      for (int k = 0; k < 4; ++k) c[u][k] = (int)i0 + k;
    }
  }
  [[maybe_unused]] int ag[kU][4];
  if constexpr (ALWAYS && MODE == 1) {
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const f4u q = ld4u(x + c[u][0]);
      xg[u][0] = q.x;
      xg[u][1] = q.y;
      xg[u][2] = q.z;
      xg[u][3] = q.w;
      if constexpr (PRO) {
        const i4u a = *reinterpret_cast<const i4u*>(L.agg + c[u][0]);
        ag[u][0] = a.x;
        ag[u][1] = a.y;
        ag[u][2] = a.z;
        ag[u][3] = a.w;
      }
    }
#pragma unroll
    for (int u = 0; u < kU; ++u)
      if (!consec4(c[u])) {
#pragma unroll
        for (int k = 1; k < 4; ++k) {
          xg[u][k] = x[c[u][k]];
          if constexpr (PRO) ag[u][k] = (int)L.agg[c[u][k]];
        }
      }
  } else {
#pragma unroll
    for (int u = 0; u < kU; ++u)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        xg[u][k] = gat<ALWAYS && MODE == 1>(r0 + u < u4(ln, k), x + c[u][k]);
        // unused slots hold the row's own (valid) column: agg of a real or padding row
        if constexpr (PRO) ag[u][k] = (int)L.agg[c[u][k]];
      }
  }
  if constexpr (PRO) {
    float cv[kU][4];
#pragma unroll
    for (int u = 0; u < kU; ++u)
#pragma unroll
      for (int k = 0; k < 4; ++k) cv[u][k] = xc[ag[u][k]];
#pragma unroll
    for (int u = 0; u < kU; ++u)
#pragma unroll
      for (int k = 0; k < 4; ++k) xg[u][k] = prolonged(xg[u][k], cv[u][k]);
  }
}

// smooth_op (amg.wgsl:24-50) restated out-of-place: x_out = mix(x, (b - sigma)/diag, 0.8).
// PRO (post-smoother of a single-GPU / replicated level): the prolongation
// from the coarse level xc that precedes it (k_amg_prolong) is applied to
// every x value as it is read, so x' = x + P xc is never stored -- the same
// f32 operations per value, one launch and one pass over x / agg fewer.
// smooth4: the 4 rows i0..i0+3
// The row operands (b, x, diagonal) are loaded after the slot loop (loading
// them with the row lengths was inside the noise, round 3); in the fused
// post-smoother the row's own prolongation term (agg -> x_c) comes after the
// slots as well (before them: +0.1 ... +0.5 us on every C1 level).
template <bool D16, int MODE, bool PRO = false, bool NT = false>
__device__ __forceinline__ float4 smooth4(const AmgLevelDev& L, const float* __restrict__ x,
                                          const float* __restrict__ b, uint32_t i0,
                                          const float* __restrict__ xc = nullptr) {
  const uchar4 ln = ldv<NT, uchar4>(L.len + i0);
  const uint32_t maxlen = max(max(ln.x, ln.y), max(ln.z, ln.w));
  float sg[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  auto step = [&](uint32_t r0, uint32_t rmax) {
    float4 v[kU];
    float xg[kU][4];
    gather_group<D16, MODE, true, PRO, NT>(L, x, i0, r0, rmax, ln, v, xg, xc);
#pragma unroll
    for (int u = 0; u < kU; ++u)
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (r0 + u < u4(ln, k)) sg[k] += f4(v[u], k) * xg[u][k];
  };
  if constexpr (MODE != 0) {
    // first slot group peeled: its loads (clamped to the ELL width) do not wait for the lengths
    step(0, (uint32_t)max(L.w, 1) - 1u);
    for (uint32_t r0 = kU; r0 < maxlen; r0 += kU) step(r0, maxlen - 1u);
  } else {
    for (uint32_t r0 = 0; r0 < maxlen; r0 += kU) step(r0, maxlen - 1u);
  }
  const float4 bb = ldv<NT, float4>(b + i0);
  float4 xx = *reinterpret_cast<const float4*>(x + i0);
  const float4 dd = ldv<NT, float4>(L.de + i0);
  if constexpr (PRO) {  // the row's own value, as k_amg_prolong (padding rows get + 0)
    float pc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    const int4 ag = *reinterpret_cast<const int4*>(L.agg + i0);
    pc[0] += 1.0f * xc[ag.x];
    if (i0 + 1 < L.n) pc[1] += 1.0f * xc[ag.y];
    if (i0 + 2 < L.n) pc[2] += 1.0f * xc[ag.z];
    if (i0 + 3 < L.n) pc[3] += 1.0f * xc[ag.w];
    xx.x += pc[0];
    xx.y += pc[1];
    xx.z += pc[2];
    xx.w += pc[3];
  }
  float4 o;
  o.x = wmix(xx.x, (bb.x - sg[0]) / dd.x, 0.8f);
  o.y = wmix(xx.y, (bb.y - sg[1]) / dd.y, 0.8f);
  o.z = wmix(xx.z, (bb.z - sg[2]) / dd.z, 0.8f);
  o.w = wmix(xx.w, (bb.w - sg[3]) / dd.w, 0.8f);
  return o;
}
// The level's fields the sweep needs first (row lengths, slot values and
// columns, the row ranges, ELL stride and width) and x, b lead the argument
// list: those 16 dwords arrive preloaded in SGPRs (kernarg preload, §4), so
// the first loads wait for no kernarg round trip; the rest of the level
// image comes with L.
template <bool D16, int MODE, bool PRO = false, bool NT = false>
__global__ void __launch_bounds__(kBlock) k_amg_smooth(const uint8_t* len, const float* val, const void* col,
                                                       uint32_t r0, uint32_t r1, uint32_t r2, uint32_t r3,
                                                       uint32_t stride, int w, const float* __restrict__ x,
                                                       const float* __restrict__ b, float* __restrict__ x_out,
                                                       AmgLevelDev L, const float* __restrict__ xc) {
  uint32_t i0;
  if (!row_range<kRevSmooth>(r0, r1, r2, r3, i0)) return;
  AmgLevelDev Lk = L;
  Lk.len = len;
  Lk.val = val;
  if constexpr (D16)
    Lk.col16 = static_cast<const int16_t*>(col);
  else
    Lk.col32 = static_cast<const int32_t*>(col);
  Lk.r0 = r0;
  Lk.r1 = r1;
  Lk.r2 = r2;
  Lk.r3 = r3;
  Lk.stride = stride;
  Lk.w = w;
  *reinterpret_cast<float4*>(x_out + i0) = smooth4<D16, MODE, PRO, NT>(Lk, x, b, i0, xc);
}
// The reference's IN-PLACE smooth_op (amg.wgsl:24-50) under one legal
// schedule (test mode, Solver::ref_inplace; oracle kSemInplaceSmoother): the
// 64-row workgroups one after another, every row of a workgroup reading x
// before any of them writes -- so rows of earlier workgroups are read new.
// One block walks the row blocks in order; its 16 threads take 4 rows each
// (smooth4: the same operations as k_amg_smooth).
template <bool D16, int MODE>
__global__ void __launch_bounds__(16) k_amg_smooth_ordered(AmgLevelDev L, float* x, const float* __restrict__ b) {
  for (uint32_t b0 = 0; b0 < L.n; b0 += 64) {
    const uint32_t i0 = b0 + 4 * threadIdx.x;
    float4 o = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    if (i0 < L.n) o = smooth4<D16, MODE>(L, x, b, i0);
    __syncthreads();  // the workgroup's reads complete
    if (i0 < L.n) *reinterpret_cast<float4*>(x + i0) = o;
    __syncthreads();  // visible to the next workgroup's reads
  }
}

// the leading arguments of k_amg_smooth from a level image
#define CFD_AMG_HEAD(L) \
  (L).len, (L).val, ((L).use16 ? (const void*)(L).col16 : (const void*)(L).col32), (L).r0, (L).r1, (L).r2, (L).r3, \
      (L).stride, (L).w

// smooth_op on a level whose x is identically +0 (every coarse level's
// pre-smoother: restrict just cleared it): sigma = +0, so the sweep is the
// elementwise x_out = mix(+0, (b - 0)/diag, 0.8) -- the same f32 operations
// as k_amg_smooth without reading the matrix.
__global__ void __launch_bounds__(kBlock) k_amg_smooth_zero(AmgLevelDev L, const float* __restrict__ b,
                                                            float* __restrict__ x_out) {
  const uint32_t i0 = 4 * row_id();
  if (i0 >= L.n) return;
  const float4 bb = *reinterpret_cast<const float4*>(b + i0);
  const float4 dd = *reinterpret_cast<const float4*>(L.de + i0);
  float4 o;
  o.x = wmix(0.0f, (bb.x - 0.0f) / dd.x, 0.8f);
  o.y = wmix(0.0f, (bb.y - 0.0f) / dd.y, 0.8f);
  o.z = wmix(0.0f, (bb.z - 0.0f) / dd.z, 0.8f);
  o.w = wmix(0.0f, (bb.w - 0.0f) / dd.w, 0.8f);
  *reinterpret_cast<float4*>(x_out + i0) = o;
}

// residual part of restrict_residual (amg.wgsl:80-111): r = b - A x over the full
// row in column order, the diagonal inserted at its rank.
template <bool D16, int MODE, bool NT = false>
__device__ __forceinline__ float4 residual4(const AmgLevelDev& L, const float* __restrict__ x,
                                            const float* __restrict__ b, uint32_t i0) {
  const uchar4 ln = ldv<NT, uchar4>(L.len + i0);
  const uchar4 dr = ldv<NT, uchar4>(L.drank + i0);
  const float4 xx = *reinterpret_cast<const float4*>(x + i0);
  const float4 dv = ldv<NT, float4>(L.dv + i0);
  const uint32_t maxlen = max(max(ln.x, ln.y), max(ln.z, ln.w));
  float ax[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  auto step = [&](uint32_t r0, uint32_t rmax) {
    float4 v[kU];
    float xg[kU][4];
    gather_group<D16, MODE, true, false, NT>(L, x, i0, r0, rmax, ln, v, xg);
#pragma unroll
    for (int u = 0; u < kU; ++u)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t r = r0 + u;
        if (r == u4(dr, k)) ax[k] += f4(dv, k) * f4(xx, k);
        if (r < u4(ln, k)) ax[k] += f4(v[u], k) * xg[u][k];
      }
  };
  uint32_t r0 = 0;
  if constexpr (MODE != 0) {
    step(0, (uint32_t)max(L.w, 1) - 1u);  // peeled first group (see k_amg_smooth)
    r0 = kU;
  }
  for (; r0 < maxlen; r0 += kU) step(r0, maxlen - 1u);
  // a diagonal ranked after every visited slot (rank = len >= r0) comes last
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (u4(dr, k) >= r0) ax[k] += f4(dv, k) * f4(xx, k);
  const float4 bb = ldv<NT, float4>(b + i0);
  float4 o;
  o.x = bb.x - ax[0];
  o.y = bb.y - ax[1];
  o.z = bb.z - ax[2];
  o.w = bb.w - ax[3];
  return o;
}
template <bool D16, int MODE, bool NT = false>
__global__ void __launch_bounds__(kBlock) k_amg_residual(AmgLevelDev L, const float* __restrict__ x,
                                                         const float* __restrict__ b, float* __restrict__ rr) {
  uint32_t i0;
  if (!row_range<kRevResidual>(L.r0, L.r1, L.r2, L.r3, i0)) return;
  *reinterpret_cast<float4*>(rr + i0) = residual4<D16, MODE, NT>(L, x, b, i0);
}

// relax_pressure (schur_precond.wgsl:52-90) on large meshes, 4 rows per thread
// over the scalar ELL image (16-bit column deltas, u8 lengths / diagonal ranks,
// the AMG row kernels' slot groups and vector gathers): the diagonal sits in
// the slots and is skipped by its rank, every other entry is summed in slot
// order -- the reference's f32 operations (omega = 1.2, the live scalar
// matrix), row for row.
template <bool D16>
__global__ void __launch_bounds__(kBlock) k_relax_pressure4(AmgLevelDev L, const uint8_t* __restrict__ drank,
                                                            const float* __restrict__ dinv_p,
                                                            const float* __restrict__ temp_p,
                                                            const float* __restrict__ src, float* dst) {
  uint32_t i0;
  if (!row_range(L.r0, L.r1, L.r2, L.r3, i0)) return;
  const uchar4 ln = *reinterpret_cast<const uchar4*>(L.len + i0);
  const uchar4 dr = *reinterpret_cast<const uchar4*>(drank + i0);
  const uint32_t maxlen = max(max(ln.x, ln.y), max(ln.z, ln.w));
  float sg[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  auto step = [&](uint32_t r0, uint32_t rmax) {
    float4 v[kU];
    float xg[kU][4];
    gather_group<D16, 1, true>(L, src, i0, r0, rmax, ln, v, xg);
#pragma unroll
    for (int u = 0; u < kU; ++u)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t r = r0 + u;
        if (r < u4(ln, k) && r != u4(dr, k)) sg[k] += f4(v[u], k) * xg[u][k];
      }
  };
  step(0, (uint32_t)max(L.w, 1) - 1u);  // peeled first group: its loads do not wait for the lengths
  for (uint32_t r0 = kU; r0 < maxlen; r0 += kU) step(r0, maxlen - 1u);
  const float4 dp = *reinterpret_cast<const float4*>(dinv_p + i0);
  const float4 tp = *reinterpret_cast<const float4*>(temp_p + i0);
  const float4 old = *reinterpret_cast<const float4*>(dst + i0);
  const float d[4] = {dp.x, dp.y, dp.z, dp.w}, b[4] = {tp.x, tp.y, tp.z, tp.w}, o[4] = {old.x, old.y, old.z, old.w};
  float y[4];
#pragma unroll
  for (int k = 0; k < 4; ++k)  // padding rows (i >= n) keep their value
    y[k] = (i0 + k < L.n) ? wmix(o[k], d[k] * (b[k] - sg[k]), 1.2f) : o[k];
  *reinterpret_cast<float4*>(dst + i0) = make_float4(y[0], y[1], y[2], y[3]);
}

// coarse value I of the restriction: sum_{f in R row I, ascending} 1.0 * r[f]
__device__ __forceinline__ float restrict_sum(const AmgLevelDev& L, const float* __restrict__ r, uint32_t I) {
  float sum = 0.0f;
  if (L.r_m4) {
    // the first 4 members in one 16-byte load, then their values
    const int4 m = L.r_m4[I];
    const bool over = m.w < -1;  // more than 4 members: member 3 stored as -2 - f
    const int f[4] = {m.x, m.y, m.z, over ? -2 - m.w : m.w};
    float v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = r[max(f[q], 0)];
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (f[q] >= 0) sum += 1.0f * v[q];
    if (over)  // the members after the fourth, in ascending order
      for (uint32_t k = L.r_row[I] + 4; k < L.r_row[I + 1]; ++k) sum += 1.0f * r[L.r_col[k]];
  } else {
    // members fetched 4 at a time (indices clamped to the row's last member,
    // unused values skipped): one round trip for the indices and one for the
    // values per 4 members instead of one dependent pair per member
    const uint32_t k0 = L.r_row[I], k1 = L.r_row[I + 1];
    for (uint32_t k = k0; k < k1; k += 4) {
      uint32_t f[4];
      float v[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) f[q] = L.r_col[min(k + q, k1 - 1)];
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = r[f[q]];
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (k + q < k1) sum += 1.0f * v[q];
    }
  }
  return sum;
}

// restriction part: coarse_b[I] = sum_{f in R row I, ascending} 1.0 * r[f];
// also clears the coarse solution (amg.rs:721-725 `clear`, fused), including
// its ghost entries [-glo, 0) and [stride_c, stride_c + ghi) on a distributed level
__global__ void __launch_bounds__(kBlock) k_amg_restrict(AmgLevelDev L, const float* __restrict__ r,
                                                         float* __restrict__ cb,
                                                         float* __restrict__ cx, uint32_t stride_c,
                                                         uint32_t glo, uint32_t ghi,
                                                         float* __restrict__ sm_out,
                                                         const float* __restrict__ sm_de, uint32_t I0,
                                                         uint32_t I1) {
  const uint32_t I = I0 + row_id();
  if (I < I1) {
    // the coarse diagonal loaded with the members (no round trip after the sum)
    const float dec = sm_out ? sm_de[I] : 1.0f;
    const float sum = restrict_sum(L, r, I);
    cb[I] = sum;
    if (sm_out)  // the coarse level's zero-x pre-smoother fused (k_amg_smooth_zero)
      sm_out[I] = wmix(0.0f, (sum - 0.0f) / dec, 0.8f);
    else
      cx[I] = 0.0f;
    return;
  }
  if (sm_out) return;
  const uint32_t g = I - I1;
  if (g < glo)
    cx[-1 - (int)g] = 0.0f;
  else if (g < glo + ghi)
    cx[stride_c + (g - glo)] = 0.0f;
}

// Residual (amg.wgsl:80-111) and restriction (:114-120) of a single-GPU or
// replicated level in one kernel: a block owns aggregates [I0, I1) (L.rr_agg
// per block); its threads compute the residuals of those aggregates' members,
// rows r_col[p] for p in [r_row[I0], r_row[I1]), one row per thread, into
// LDS in member order; then thread t sums aggregate I0 + t's members in
// ascending order.  Every row's residual accumulates as in k_amg_residual
// (slots below the diagonal's rank, the diagonal, the rest) and every coarse
// value as in k_amg_restrict (0 + r_1 + r_2 ...): the same f32 operations.
// Saves the residual vector's store and the restriction's gathers of it, and
// one launch per level.  Bottom-up (kRevResidual), after the top-down smoother.
template <bool D16>
__global__ void __launch_bounds__(kBlock) k_amg_resrestrict(AmgLevelDev L, const float* __restrict__ x,
                                                            const float* __restrict__ b, float* __restrict__ cb,
                                                            float* __restrict__ cx, float* __restrict__ sm_out,
                                                            const float* __restrict__ sm_de) {
  __shared__ float rl[kRRCap];
  const uint32_t I0 = xcd_block<kRevResidual>() * L.rr_agg;
  if (I0 >= L.nc) return;
  const uint32_t I1 = min(I0 + L.rr_agg, L.nc);
  const uint32_t p0 = L.r_row[I0], p1 = L.r_row[I1];
  const uint32_t w = (uint32_t)max(L.w, 1);
  // this thread's aggregate's member range and coarse diagonal, loaded before
  // the residual phase (no dependent round trips after the barrier)
  [[maybe_unused]] uint32_t mk0 = 0, mk1 = 0;
  [[maybe_unused]] float dec = 1.0f;
  if (I0 + threadIdx.x < I1) {
    mk0 = L.r_row[I0 + threadIdx.x];
    mk1 = L.r_row[I0 + threadIdx.x + 1];
    if (sm_out) dec = sm_de[I0 + threadIdx.x];
  }
  for (uint32_t p = p0 + threadIdx.x; p < p1; p += kBlock) {
    const uint32_t f = L.r_col[p];
    const uint32_t len = L.len[f], dr = L.drank[f];
    const float xf = x[f], dvf = L.dv[f];
    float ax = 0.0f;
    uint32_t r0 = 0;
    for (; r0 < len; r0 += 4) {
      float v[4], xg[4];
      int c[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const size_t off = (size_t)min(r0 + u, w - 1u) * L.stride + f;
        v[u] = L.val[off];
        c[u] = D16 ? (int)f + (int)L.col16[off] : L.col32[off];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) xg[u] = x[c[u]];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const uint32_t r = r0 + u;
        if (r == dr) ax += dvf * xf;
        if (r < len) ax += v[u] * xg[u];
      }
    }
    if (dr >= r0) ax += dvf * xf;  // a diagonal ranked after every visited slot comes last
    rl[p - p0] = b[f] - ax;
  }
  __syncthreads();
  const uint32_t t = threadIdx.x;
  if (I0 + t >= I1) return;
  const uint32_t I = I0 + t;
  float sum = 0.0f;
  for (uint32_t k = mk0; k < mk1; ++k) sum += 1.0f * rl[k - p0];
  cb[I] = sum;
  if (sm_out)  // the coarse level's zero-x pre-smoother fused (k_amg_smooth_zero)
    sm_out[I] = wmix(0.0f, (sum - 0.0f) / dec, 0.8f);
  else
    cx[I] = 0.0f;
}

// The up-leg of two adjacent single-GPU / replicated levels (c, c-1) in one
// launch (AmgUpPairImage, kernels.hpp): phase 1 smooths the level-c rows T
// the block needs with their prolongation from level c+1 applied to every
// read (k_amg_smooth<..., PRO>'s operations: x' = x + (0 + 1 x_c+1[agg]),
// sigma over the off-diagonals in slot order, mix(x', (b - sigma) / de,
// 0.8)) into LDS; phase 2 smooths the block's fine rows the same way with
// x_f + (0 + 1 x_c[agg]) read from that LDS image.  The fine rows' slots,
// columns, local indices and x gathers are loaded before phase 1.
template <bool D16F, bool D16C>
__global__ void __launch_bounds__(kUpPairRows) k_amg_prolong_smooth_pair(AmgLevelDev Lf, AmgLevelDev Lc,
                                                                       AmgUpPairImage P,
                                                                       const float* __restrict__ xf,
                                                                       const float* __restrict__ bf,
                                                                       float* __restrict__ xf_out,
                                                                       const float* __restrict__ xc,
                                                                       const float* __restrict__ bc,
                                                                       const float* __restrict__ xcc) {
  __shared__ float xs[kUpPairCap];
  const uint32_t blk = xcd_block<kRevSmooth>();
  if (blk >= P.nblocks) return;
  const uint32_t t = threadIdx.x;
  const uint32_t f = blk * kUpPairRows + t;
  const bool own = f < Lf.n;
  // fine row operands (independent of phase 1)
  constexpr int W = kPairW;
  uint32_t flen = 0, flo = 0;
  float fx = 0.0f, fb = 0.0f, fde = 1.0f;
  float fv[W], fg[W];
  uint32_t fl[W];
  const uint32_t wf = (uint32_t)max(Lf.w, 1);
  if (own) {
    flen = Lf.len[f];
    flo = P.lto[f];
    fx = xf[f];
    fb = bf[f];
    fde = Lf.de[f];
#pragma unroll
    for (int r = 0; r < W; ++r) {
      const size_t off = (size_t)min((uint32_t)r, wf - 1u) * Lf.stride + f;
      fv[r] = Lf.val[off];
      fl[r] = P.lt[off];
      const int c = D16F ? (int)f + (int)Lf.col16[off] : Lf.col32[off];
      fg[r] = xf[c];
    }
  }
  // phase 1: post-smoothed level-c rows of T (prolongation from c+1 in the reads)
  const uint32_t t0 = P.tb[blk], nt = P.tb[blk + 1] - t0;
  const uint32_t wc = (uint32_t)max(Lc.w, 1);
  for (uint32_t q = t; q < nt; q += kUpPairRows) {
    const uint32_t g = P.t[t0 + q];
    const uint32_t len = Lc.len[g];
    float sg = 0.0f;
    for (uint32_t r = 0; r < len; ++r) {
      const size_t off = (size_t)min(r, wc - 1u) * Lc.stride + g;
      const int c = D16C ? (int)g + (int)Lc.col16[off] : Lc.col32[off];
      const float xg = prolonged(xc[c], xcc[Lc.agg[c]]);
      sg += Lc.val[off] * xg;
    }
    float xx = xc[g];
    float pc = 0.0f;
    pc += 1.0f * xcc[Lc.agg[g]];
    xx += pc;
    xs[q] = wmix(xx, (bc[g] - sg) / Lc.de[g], 0.8f);
  }
  __syncthreads();
  // phase 2: the block's fine rows, x_f + P x_c read through the LDS image
  if (!own) return;
  float sg = 0.0f;
  for (uint32_t r = 0; r < flen; ++r) {
    float v, xg;
    if (r < (uint32_t)W) {
      v = fv[r];
      xg = prolonged(fg[r], xs[fl[r]]);
    } else {
      const size_t off = (size_t)r * Lf.stride + f;
      const int c = D16F ? (int)f + (int)Lf.col16[off] : Lf.col32[off];
      v = Lf.val[off];
      xg = prolonged(xf[c], xs[P.lt[off]]);
    }
    sg += v * xg;
  }
  float pc = 0.0f;
  pc += 1.0f * xs[flo];
  fx += pc;
  xf_out[f] = wmix(fx, (fb - sg) / fde, 0.8f);
}

// The down-leg of two adjacent single-GPU / replicated levels (i, i+1) in one
// launch (AmgPairImage, kernels.hpp): the two k_amg_resrestrict launches'
// arithmetic, operation for operation.  Phase 1: one level-i member residual
// per thread (k_amg_resrestrict's loop) into LDS; phase 2: every S row's rhs
// (0 + r_1 + r_2 ... in R order) and its zero-x pre-smoother
// mix(0, (b - 0) / de, 0.8), the block's own rows stored; phase 3: the level-
// (i+1) residual of the block's rows from the LDS values (diagonal at its rank
// among the off-diagonals, as k_amg_resrestrict); phase 4: the level-(i+2)
// rhs per aggregate and its pre-smoother (or x = 0).  The level-(i+1) slots,
// row headers and the aggregate ranges are loaded before phase 1, so the
// second level costs LDS round trips only; the ring rows' level-i residuals
// are the redundant work (amg_fusion_ratio.py).
template <bool D16, uint32_t NTH>
__global__ void __launch_bounds__(NTH) k_amg_resrestrict_pair(AmgLevelDev Lf, AmgLevelDev Lm,
                                                                     AmgPairImage P, const float* __restrict__ x,
                                                                     const float* __restrict__ b,
                                                                     float* __restrict__ bm, float* __restrict__ xm,
                                                                     float* __restrict__ cb, float* __restrict__ cx,
                                                                     float* __restrict__ sm_out,
                                                                     const float* __restrict__ sm_de) {
  __shared__ float rl[NTH];  // level-i residuals of the block's f rows
  __shared__ float bs[NTH];  // level-(i+1) rhs of the block's s rows
  __shared__ float xs[NTH];  // their pre-smoothed x
  __shared__ float r2[NTH];  // level-(i+1) residuals of the block's own rows
  const uint32_t blk = xcd_block<kRevResidual>();
  if (blk >= P.nblocks) return;
  const uint32_t t = threadIdx.x;
  const uint32_t s0 = P.sb[blk], s1 = P.sb[blk + 1];
  const uint32_t J0 = P.jb[blk], J1 = P.jb[blk + 1];
  const uint32_t m0 = Lm.r_row[J0], nm = Lm.r_row[J1] - m0;
  const uint32_t fb = P.fo[s0], fe = P.fo[s1];
  // phase-2 / phase-3 / phase-4 operands, independent of phase 1
  uint32_t sr = 0, k0 = 0, k1 = 0, mlen = 0, mdr = 0, a0 = 0, a1 = 0;
  float des = 1.0f, mdv = 0.0f, dec = 1.0f;
  float mv[kPairW];
  uint32_t mc[kPairW];
  if (s0 + t < s1) {
    sr = P.s[s0 + t];
    k0 = P.fo[s0 + t];
    k1 = P.fo[s0 + t + 1];
    des = Lm.de[sr];
  }
  if (t < nm) {
    mlen = Lm.len[sr];
    mdr = Lm.drank[sr];
    mdv = Lm.dv[sr];
    const uint32_t wm = (uint32_t)max(Lm.w, 1);
#pragma unroll
    for (int r = 0; r < kPairW; ++r) {
      const size_t off = (size_t)min((uint32_t)r, wm - 1u) * Lm.stride + sr;
      mv[r] = Lm.val[off];
      mc[r] = P.lc[off];
    }
  }
  if (J0 + t < J1) {
    a0 = Lm.r_row[J0 + t];
    a1 = Lm.r_row[J0 + t + 1];
    if (sm_out) dec = sm_de[J0 + t];
  }
  // phase 1: level-i residuals (k_amg_resrestrict's row loop)
  const uint32_t w = (uint32_t)max(Lf.w, 1);
  for (uint32_t p = fb + t; p < fe; p += NTH) {
    const uint32_t f = P.f[p];
    const uint32_t len = Lf.len[f], dr = Lf.drank[f];
    const float xf = x[f], dvf = Lf.dv[f];
    float ax = 0.0f;
    uint32_t r0 = 0;
    for (; r0 < len; r0 += 4) {
      float v[4], xg[4];
      int c[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const size_t off = (size_t)min(r0 + u, w - 1u) * Lf.stride + f;
        v[u] = Lf.val[off];
        c[u] = D16 ? (int)f + (int)Lf.col16[off] : Lf.col32[off];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) xg[u] = x[c[u]];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const uint32_t r = r0 + u;
        if (r == dr) ax += dvf * xf;
        if (r < len) ax += v[u] * xg[u];
      }
    }
    if (dr >= r0) ax += dvf * xf;
    rl[p - fb] = b[f] - ax;
  }
  __syncthreads();
  // phase 2: level-(i+1) rhs (restriction) and zero-x pre-smoother of every s row
  if (s0 + t < s1) {
    float sum = 0.0f;
    for (uint32_t k = k0; k < k1; ++k) sum += 1.0f * rl[k - fb];
    const float xv = wmix(0.0f, (sum - 0.0f) / des, 0.8f);
    bs[t] = sum;
    xs[t] = xv;
    if (t < nm) {  // the block's own rows (every level-(i+1) row is one block's)
      bm[sr] = sum;
      xm[sr] = xv;
    }
  }
  __syncthreads();
  // phase 3: level-(i+1) residual of the block's rows
  if (t < nm) {
    const float xf = xs[t];
    float ax = 0.0f;
    uint32_t r = 0;
    for (; r < mlen; ++r) {
      float v;
      uint32_t c;
      if (r < (uint32_t)kPairW) {
        v = mv[r];
        c = mc[r];
      } else {
        const size_t off = (size_t)r * Lm.stride + sr;
        v = Lm.val[off];
        c = P.lc[off];
      }
      if (r == mdr) ax += mdv * xf;
      ax += v * xs[c];
    }
    if (mdr >= r) ax += mdv * xf;  // a diagonal ranked after every off-diagonal comes last
    r2[t] = bs[t] - ax;
  }
  __syncthreads();
  // phase 4: level-(i+2) rhs (restriction) and its pre-smoother / cleared x
  if (J0 + t < J1) {
    const uint32_t J = J0 + t;
    float sum = 0.0f;
    for (uint32_t k = a0; k < a1; ++k) sum += 1.0f * r2[k - m0];
    cb[J] = sum;
    if (sm_out)
      sm_out[J] = wmix(0.0f, (sum - 0.0f) / dec, 0.8f);
    else
      cx[J] = 0.0f;
  }
}

// prolongate_op (amg.wgsl:56-75): x += (0 + 1 * xc[agg]), 4 rows per thread.
// agg is a signed local index on a distributed level (aggregates seeded on a
// lower rank are ghosts of xc below 0).
template <bool NT>
__global__ void __launch_bounds__(kBlock) k_amg_prolong(AmgLevelDev L, float* __restrict__ x,
                                                        const float* __restrict__ xc, uint32_t f0, uint32_t f1) {
  const uint32_t i0 = f0 + 4 * row_id();
  if (i0 >= f1) return;
  float4 xx = *reinterpret_cast<const float4*>(x + i0);
  const int4 ag = ldv<NT, int4>(L.agg + i0);
  float c0 = 0.0f, c1 = 0.0f, c2 = 0.0f, c3 = 0.0f;  // padding rows (>= n) get 0
  c0 += 1.0f * xc[ag.x];
  if (i0 + 1 < L.n) c1 += 1.0f * xc[ag.y];
  if (i0 + 2 < L.n) c2 += 1.0f * xc[ag.z];
  if (i0 + 3 < L.n) c3 += 1.0f * xc[ag.w];
  xx.x += c0;
  xx.y += c1;
  xx.z += c2;
  xx.w += c3;
  *reinterpret_cast<float4*>(x + i0) = xx;
}

// ---- single-row helpers for the one-workgroup kernels (small levels) ----
__device__ __forceinline__ int col_at(const AmgLevelDev& L, size_t off, uint32_t i) {
  return L.use16 ? (int)i + (int)L.col16[off] : L.col32[off];
}
__device__ __forceinline__ float smooth_row(const AmgLevelDev& L, const float* x, const float* b,
                                            uint32_t i) {
  float sigma = 0.0f;
  const uint32_t len = L.len16 ? (uint32_t)L.len16[i] : (uint32_t)L.len[i];
  for (uint32_t r = 0; r < len; ++r) {
    const size_t off = (size_t)r * L.stride + i;
    sigma += L.val[off] * x[col_at(L, off, i)];
  }
  return wmix(x[i], (b[i] - sigma) / L.de[i], 0.8f);
}
__device__ __forceinline__ float residual_row(const AmgLevelDev& L, const float* x, const float* b,
                                              uint32_t i) {
  const uint32_t len = L.len16 ? (uint32_t)L.len16[i] : (uint32_t)L.len[i];
  const uint32_t dr = L.drank16 ? (uint32_t)L.drank16[i] : (uint32_t)L.drank[i];
  float ax = 0.0f;
  for (uint32_t r = 0; r <= len; ++r) {
    if (r == dr) ax += L.dv[i] * x[i];
    if (r == len) break;
    const size_t off = (size_t)r * L.stride + i;
    ax += L.val[off] * x[col_at(L, off, i)];
  }
  return b[i] - ax;
}

// One workgroup runs the V-cycle over the small levels [first, nlev): every
// phase of amg.rs:666-770 with a workgroup barrier instead of a kernel boundary.
// Each level does an even number of out-of-place sweeps, so the pre-smoother
// goes x -> xt, the post-smoother xt -> x and the coarsest solve ends in x,
// exactly the host-side ping-pong of Solver::amg_smooth.
__global__ void __launch_bounds__(1024) k_amg_tail(const AmgTailLevel* __restrict__ tail, int first,
                                                   int nlev) {
  const uint32_t t = threadIdx.x, nt = blockDim.x;
  for (int l = first; l + 1 < nlev; ++l) {
    const AmgTailLevel T = tail[l];
    for (uint32_t i = t; i < T.L.n; i += nt) T.xt[i] = smooth_row(T.L, T.x, T.b, i);
    __syncthreads();
    for (uint32_t i = t; i < T.L.n; i += nt) T.r[i] = residual_row(T.L, T.xt, T.b, i);
    __syncthreads();
    float* cb = tail[l + 1].b;
    float* cx = tail[l + 1].x;
    for (uint32_t I = t; I < T.L.nc; I += nt) {
      float sum = 0.0f;
      for (uint32_t k = T.L.r_row[I]; k < T.L.r_row[I + 1]; ++k) sum += 1.0f * T.r[T.L.r_col[k]];
      cb[I] = sum;
      cx[I] = 0.0f;
    }
    __syncthreads();
  }
  {
    const AmgTailLevel T = tail[nlev - 1];
    for (int s = 0; s < 10; ++s) {
      const float* xin = (s & 1) ? T.xt : T.x;
      float* xout = (s & 1) ? T.x : T.xt;
      for (uint32_t i = t; i < T.L.n; i += nt) xout[i] = smooth_row(T.L, xin, T.b, i);
      __syncthreads();
    }
  }
  for (int l = nlev - 2; l >= first; --l) {
    const AmgTailLevel T = tail[l];
    const float* xc = tail[l + 1].x;
    for (uint32_t i = t; i < T.L.n; i += nt) {
      float corr = 0.0f;
      corr += 1.0f * xc[T.L.agg[i]];
      T.xt[i] += corr;
    }
    __syncthreads();
    for (uint32_t i = t; i < T.L.n; i += nt) T.x[i] = smooth_row(T.L, T.xt, T.b, i);
    __syncthreads();
  }
}

// The same V-cycle tail with every vector of the tail levels in LDS (x, xt,
// b, r per level; the matrices stay in L2): each phase is one global-latency
// round (matrix row) + LDS gathers + a barrier.  Entry: b of `first` in global
// memory, x of every tail level known zero (cleared by the restriction), so
// each pre-smoother is the elementwise zero-x sweep.  Exit: x of `first`
// written back for the host-side prolongation.
__device__ __forceinline__ uint32_t r4(uint32_t n) { return (n + 3) & ~3u; }

__global__ void __launch_bounds__(1024) k_amg_tail_lds(const AmgTailLevel* __restrict__ tail, int first,
                                                       int nlev) {
  extern __shared__ float sm[];
  const uint32_t t = threadIdx.x, nt = blockDim.x;
  auto base = [&](int l) {
    uint32_t o = 0;
    for (int k = first; k < l; ++k) o += 4 * r4(tail[k].L.n);
    return sm + o;
  };
  {
    const AmgTailLevel T = tail[first];
    float* B0 = base(first) + 2 * r4(T.L.n);
    for (uint32_t i = t; i < T.L.n; i += nt) B0[i] = T.b[i];
  }
  __syncthreads();
  for (int l = first; l + 1 < nlev; ++l) {
    const AmgLevelDev L = tail[l].L;
    const uint32_t nr = r4(L.n);
    float* X = base(l);
    float* XT = X + nr;
    float* B = XT + nr;
    float* Rr = B + nr;
    for (uint32_t i = t; i < L.n; i += nt) XT[i] = wmix(0.0f, (B[i] - 0.0f) / L.de[i], 0.8f);
    __syncthreads();
    for (uint32_t i = t; i < L.n; i += nt) Rr[i] = residual_row(L, XT, B, i);
    __syncthreads();
    float* CB = base(l + 1) + 2 * r4(tail[l + 1].L.n);
    for (uint32_t I = t; I < L.nc; I += nt) {
      float sum = 0.0f;
      for (uint32_t k = L.r_row[I]; k < L.r_row[I + 1]; ++k) sum += 1.0f * Rr[L.r_col[k]];
      CB[I] = sum;
    }
    __syncthreads();
  }
  {
    const AmgLevelDev L = tail[nlev - 1].L;
    const uint32_t nr = r4(L.n);
    float* X = base(nlev - 1);
    float* XT = X + nr;
    float* B = XT + nr;
    for (int s = 0; s < 10; ++s) {
      if (s == 0) {
        for (uint32_t i = t; i < L.n; i += nt) XT[i] = wmix(0.0f, (B[i] - 0.0f) / L.de[i], 0.8f);
      } else {
        const float* xin = (s & 1) ? XT : X;
        float* xout = (s & 1) ? X : XT;
        for (uint32_t i = t; i < L.n; i += nt) xout[i] = smooth_row(L, xin, B, i);
      }
      __syncthreads();
    }
  }
  for (int l = nlev - 2; l >= first; --l) {
    const AmgLevelDev L = tail[l].L;
    const uint32_t nr = r4(L.n);
    float* X = base(l);
    float* XT = X + nr;
    float* B = XT + nr;
    const float* XC = base(l + 1);
    for (uint32_t i = t; i < L.n; i += nt) {
      float corr = 0.0f;
      corr += 1.0f * XC[L.agg[i]];
      XT[i] += corr;
    }
    __syncthreads();
    for (uint32_t i = t; i < L.n; i += nt) X[i] = smooth_row(L, XT, B, i);
    __syncthreads();
  }
  const AmgTailLevel T = tail[first];
  const float* X0 = base(first);
  for (uint32_t i = t; i < T.L.n; i += nt) T.x[i] = X0[i];
}


// The LDS tail with every matrix of the tail levels in LDS as well (the blob
// built once by the host from the level images: off-diagonal CSR with u16
// columns, dv/de, drank, P and R).  Each phase is then LDS reads + one
// barrier instead of a global (L2) round trip per matrix slot.  Same row
// arithmetic, in the same order, as smooth_row / residual_row.
// The zero-x pre-smoother is fused with the residual, and the prolongation
// with the post-smoother (two barriers fewer per level, round 3).
__global__ void __launch_bounds__(1024) k_amg_tail_blob(const AmgTailLevel* __restrict__ tail,
                                                        const TailBlobLevel* __restrict__ desc,
                                                        const uint32_t* __restrict__ blob, uint32_t blob_words,
                                                        uint32_t vec_floats, int first, int nlev,
                                                        const float* __restrict__ b_first, uint32_t n_first) {
  extern __shared__ float sm[];
  const uint32_t t = threadIdx.x, nt = blockDim.x;
  uint32_t* bw = reinterpret_cast<uint32_t*>(sm + vec_floats);
  auto base = [&](int l) {
    uint32_t o = 0;
    for (int k = first; k < l; ++k) o += 4 * r4(desc[k].n);
    return sm + o;
  };
  {
    // every global load of the blob and of b issued before the first LDS
    // store: one memory round trip instead of one per 16 KiB pass (the blob
    // is cold in HBM after the fine levels' sweeps: C2 25.2 -> 23.9 us,
    // profiles/r03/ab_tail_occ_c2.txt).  The launch is always
    // 1024 threads; blob and b together fit in kTailLdsMax (16 B per row of
    // b's level alone), so KB / KV loads per thread cover both.
    constexpr uint32_t NT = 1024, KB = (uint32_t)((kTailLdsMax / 16 + NT - 1) / NT), KV = KB;
    // b and n of the first level as kernel arguments: no dependent load of
    // the level descriptors before the b loads
    const uint32_t n = n_first;
    const float* gb = b_first;
    uint4 v[KB];
    float bv[KV];
    // clamped, unconditional loads (guarded ones put v[] in scratch)
#pragma unroll
    for (uint32_t k = 0; k < KB; ++k)
      v[k] = *reinterpret_cast<const uint4*>(blob + min(4 * (t + k * NT), blob_words - 4));
#pragma unroll
    for (uint32_t k = 0; k < KV; ++k) bv[k] = gb[min(t + k * NT, n - 1)];
    // pin the loaded registers here so that the compiler cannot sink each
    // load into its guarded store below (load -> wait -> store per pass)
#pragma unroll
    for (uint32_t k = 0; k < KB; ++k) asm volatile("" : "+v"(v[k].x), "+v"(v[k].y), "+v"(v[k].z), "+v"(v[k].w));
#pragma unroll
    for (uint32_t k = 0; k < KV; ++k) asm volatile("" : "+v"(bv[k]));
#pragma unroll
    for (uint32_t k = 0; k < KB; ++k) {
      const uint32_t w = 4 * (t + k * NT);
      if (w < blob_words) *reinterpret_cast<uint4*>(bw + w) = v[k];
    }
    float* B0 = base(first) + 2 * r4(n);
#pragma unroll
    for (uint32_t k = 0; k < KV; ++k)
      if (t + k * NT < n) B0[t + k * NT] = bv[k];
  }
  __syncthreads();
  auto fw = [&](uint32_t off) { return reinterpret_cast<const float*>(bw + off); };
  auto hw = [&](uint32_t off) { return reinterpret_cast<const uint16_t*>(bw + off); };
  auto smooth = [&](const TailBlobLevel& D, const float* xin, const float* B, uint32_t i) {
    const uint32_t* ro = bw + D.rowoff;
    const float* val = fw(D.val);
    const uint16_t* col = hw(D.col);
    float sigma = 0.0f;
    for (uint32_t e = ro[i]; e < ro[i + 1]; ++e) sigma += val[e] * xin[col[e]];
    return wmix(xin[i], (B[i] - sigma) / fw(D.de)[i], 0.8f);
  };
  for (int l = first; l + 1 < nlev; ++l) {
    const TailBlobLevel D = desc[l];
    const uint32_t nr = r4(D.n);
    float* X = base(l);
    float* XT = X + nr;
    float* B = XT + nr;
    float* Rr = B + nr;
    const float* de = fw(D.de);
    // zero-x pre-smoother and residual in one phase: a neighbour's smoothed
    // value is recomputed from its b and diagonal (the same operations as
    // the sweep), the row's own is stored for the up-sweep
    const uint32_t* ro = bw + D.rowoff;
    const float* val = fw(D.val);
    const float* dv = fw(D.dv);
    const uint16_t* col = hw(D.col);
    const uint8_t* drank = reinterpret_cast<const uint8_t*>(bw + D.drank);
    for (uint32_t i = t; i < D.n; i += nt) {
      const float xti = wmix(0.0f, (B[i] - 0.0f) / de[i], 0.8f);
      XT[i] = xti;
      const uint32_t e0 = ro[i], len = ro[i + 1] - e0, dr = drank[i];
      float ax = 0.0f;
      for (uint32_t r = 0; r <= len; ++r) {
        if (r == dr) ax += dv[i] * xti;
        if (r == len) break;
        const uint32_t j = col[e0 + r];
        ax += val[e0 + r] * wmix(0.0f, (B[j] - 0.0f) / de[j], 0.8f);
      }
      Rr[i] = B[i] - ax;
    }
    __syncthreads();
    float* CB = base(l + 1) + 2 * r4(desc[l + 1].n);
    {
      const uint16_t* rrow = hw(D.r_row);
      const uint16_t* rcol = hw(D.r_col);
      for (uint32_t I = t; I < D.nc; I += nt) {
        float sum = 0.0f;
        for (uint32_t k = rrow[I]; k < rrow[I + 1]; ++k) sum += 1.0f * Rr[rcol[k]];
        CB[I] = sum;
      }
    }
    __syncthreads();
  }
  {
    const TailBlobLevel D = desc[nlev - 1];
    const uint32_t nr = r4(D.n);
    float* X = base(nlev - 1);
    float* XT = X + nr;
    float* B = XT + nr;
    const float* de = fw(D.de);
    if (D.maxlen == 0) {
      // coarsest level without off-diagonal entries (C1: 829 rows): every
      // sweep is row-local, so each thread runs its row's 10 sweeps in
      // registers with no barrier in between -- the operations of smooth()
      // with sigma = +0 in the same order (bit-identical; (b - 0) / d is the
      // same value in every sweep)
      for (uint32_t i = t; i < D.n; i += nt) {
        const float q = (B[i] - 0.0f) / de[i];
        float xp = wmix(0.0f, q, 0.8f), xq = xp;
        for (int s = 1; s < 10; ++s) {
          xq = xp;
          xp = wmix(xq, q, 0.8f);
        }
        XT[i] = xq;  // sweep 8 (even sweeps write XT)
        X[i] = xp;   // sweep 9
      }
      __syncthreads();
    } else {
      for (int s = 0; s < 10; ++s) {
        if (s == 0) {
          for (uint32_t i = t; i < D.n; i += nt) XT[i] = wmix(0.0f, (B[i] - 0.0f) / de[i], 0.8f);
        } else {
          const float* xin = (s & 1) ? XT : X;
          float* xout = (s & 1) ? X : XT;
          for (uint32_t i = t; i < D.n; i += nt) xout[i] = smooth(D, xin, B, i);
        }
        __syncthreads();
      }
    }
  }
  for (int l = nlev - 2; l >= first; --l) {
    const TailBlobLevel D = desc[l];
    const uint32_t nr = r4(D.n);
    float* X = base(l);
    float* XT = X + nr;
    float* B = XT + nr;
    const float* XC = base(l + 1);
    const uint16_t* agg = hw(D.agg);
    // prolongation and post-smoother in one phase: every value the sweep
    // reads is prolonged as it is read (k_amg_smooth<..., PRO>'s rule)
    const uint32_t* ro = bw + D.rowoff;
    const float* val = fw(D.val);
    const uint16_t* col = hw(D.col);
    const float* de = fw(D.de);
    for (uint32_t i = t; i < D.n; i += nt) {
      float sigma = 0.0f;
      for (uint32_t e = ro[i]; e < ro[i + 1]; ++e) {
        const uint32_t j = col[e];
        sigma += val[e] * prolonged(XT[j], XC[agg[j]]);
      }
      X[i] = wmix(prolonged(XT[i], XC[agg[i]]), (B[i] - sigma) / de[i], 0.8f);
    }
    __syncthreads();
  }
  const float* X0 = base(first);
  float* gx = tail[first].x;
  for (uint32_t i = t; i < desc[first].n; i += nt) gx[i] = X0[i];
}

// ---------------------- check_evolution statistics --------------------------
// AoS view of the reference FluidState (coupled_solver.rs:504 reads the 32-byte
// records as a flat f32 array): record r = {u.x, u.y, p, d_p, gp.x, gp.y, 0, 0}.
__device__ __forceinline__ void view_pair(const StateView& v, uint32_t rec, int pair, float* a,
                                          float* b) {
  if (pair == 0) {
    const float2 u = v.u[rec];
    *a = u.x;
    *b = u.y;
  } else if (pair == 1) {
    *a = v.p[rec];
    *b = v.dp[rec];
  } else if (pair == 2) {
    const float2 gp = v.gp[rec];
    *a = gp.x;
    *b = gp.y;
  } else {
    *a = 0.0f;
    *b = 0.0f;
  }
}

// `var` + (gbase, rec0): the records the variance part reads -- the record of
// global index gbase + c is ((gbase + c) >> 2) - rec0 in `var` (on one GPU:
// var = cur, gbase = rec0 = 0; distributed: records fetched from their owners).
// Leaves per cell: evolution = the 8 squared differences added in field order
// (u.x, u.y, p, d_p, grad_p.x, grad_p.y, and the unused grad_component pair,
// which is 0 - 0), then u, v, u^2, v^2 of the (stride-bug) variance record;
// chunk partials partial[f * np + k] in the canonical tree order.
__global__ void __launch_bounds__(kBlock) k_evolution_partial(StateView cur, StateView prev,
                                                              int have_prev, uint32_t N,
                                                              StateView var, uint64_t gbase,
                                                              uint64_t rec0, uint32_t U, double* partial,
                                                              uint32_t np) {
  __shared__ double lds[5 * 4];
  const uint32_t k = red_chunk();
  const uint32_t c0 = k * kRedChunkCells + 4 * red_lane();
  double lf[5][4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint32_t c = c0 + q;
    double evo = 0.0, a_d = 0.0, b_d = 0.0;
    if (c < N) {
      if (have_prev) {
        bool first = true;
        for (int pr = 0; pr < 4; ++pr) {
          float a0, b0, a1, b1;
          view_pair(cur, c, pr, &a0, &b0);
          view_pair(prev, c, pr, &a1, &b1);
          const float da = a0 - a1, db = b0 - b1;
          const double ta = (double)(da * da), tb = (double)(db * db);
          evo = first ? ta : evo + ta;
          evo = evo + tb;
          first = false;
        }
      }
      float a, b;
      const uint64_t gi = gbase + c;
      view_pair(var, (uint32_t)((gi >> 2) - rec0), (int)(gi & 3), &a, &b);
      a_d = (double)a;
      b_d = (double)b;
    }
    lf[0][q] = evo;
    lf[1][q] = a_d;
    lf[2][q] = b_d;
    lf[3][q] = a_d * a_d;
    lf[4][q] = b_d * b_d;
  }
#pragma unroll
  for (int f = 0; f < 5; ++f) {
    const double r = wave_tree((lf[f][0] + lf[f][1]) + (lf[f][2] + lf[f][3]));
    if (red_lane() == 0) lds[4 * f + (threadIdx.x >> 6)] = r;
  }
  __syncthreads();
  const uint32_t UB = 4 / U;
  if (threadIdx.x < 5 * UB) {
    const uint32_t f = threadIdx.x / UB, u = threadIdx.x % UB, unit = blockIdx.x * UB + u;
    if ((size_t)unit * U * kRedChunkCells < N && unit < np) partial[(size_t)f * np + unit] = unit_value(lds + 4 * f, U, u);
  }
}

__global__ void __launch_bounds__(kRedFinalThreads) k_evolution_final(RedSrcD r, double* out5) {
  __shared__ double la[kRedMaxSegments], lb[65];
  for (int f = 0; f < 5; ++f) {
    const double t = red_total<double, kRedFinalThreads>(r, (uint32_t)f, la, lb);
    if (threadIdx.x == 0) out5[f] = t;
  }
}

// ------------------------- distributed helpers ------------------------------
// Halo pack: for every field f, stage[off_f + k*comps_f + c] = src_f[idx[k]*comps_f + c]
// (idx = owned rows the peers need, concatenated per peer, ascending global id).
__global__ void __launch_bounds__(kBlock) k_pack(PackArgs a) {
  const uint32_t k = blockIdx.x * kBlock + threadIdx.x;
  if (k >= a.n) return;
  const int32_t i = a.idx[k];
  for (int f = 0; f < a.nf; ++f) {
    const PackField F = a.f[f];
    for (int c = 0; c < F.comps; ++c)
      a.stage[F.stage_off + (size_t)k * F.comps + c] = F.src[(ptrdiff_t)i * F.comps + c];
  }
}

// Distributed: this rank's segment values of nvec reductions, one wavefront
// per segment: out[v * maxseg + s] (blockIdx.y = v).
template <class T>
__global__ void __launch_bounds__(kBlock) k_seg_reduce(const T* __restrict__ part, uint32_t np, uint32_t nchunks,
                                                       uint32_t G, T* out, uint32_t maxseg) {
  const uint32_t sg = blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
  const uint32_t v = blockIdx.y;
  const uint32_t nsl = (nchunks + G - 1) / G;
  T o[1];
  seg_trees<T, 1>(part + (size_t)v * np, nchunks, G, sg, 0, nsl, o);
  if (red_lane() == 0 && sg < maxseg) out[(size_t)v * maxseg + sg] = o[0];
}

// max over ranks of the (u, p) max-diff bit patterns
__global__ void k_max_combine(const uint32_t* __restrict__ gathered, int R, uint32_t* out, uint32_t* host_out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  uint32_t bu = 0, bp = 0;
  for (int r = 0; r < R; ++r) {
    bu = max(bu, gathered[2 * r]);
    bp = max(bp, gathered[2 * r + 1]);
  }
  out[0] = bu;
  out[1] = bp;
  if (host_out) {
    host_out[0] = bu;
    host_out[1] = bp;
  }
}

}  // namespace

// ------------------------------- launchers ----------------------------------
void launch_prepare(const PrepareArgs& a, hipStream_t s) {
  if (a.N) hipLaunchKernelGGL(k_prepare, dim3(grid_for(a.N)), dim3(kBlock), 0, s, a);
}
void launch_prepare_ordered(const PrepareArgs& a, const int32_t* mirror, uint32_t slots, hipStream_t s) {
  if (!a.N) return;
  hipLaunchKernelGGL(k_prepare_ordered, dim3(1), dim3(64), 0, s, a);
  hipLaunchKernelGGL(k_flux_mirror, dim3((slots + kBlock - 1) / kBlock), dim3(kBlock), 0, s, a.flux_s, mirror, slots);
}
void launch_assemble(const AssembleArgs& a, hipStream_t s) {
  if (a.N) hipLaunchKernelGGL(k_assemble, dim3(grid_for(a.N)), dim3(kBlock), 0, s, a);
}
void launch_update_fields(uint32_t N, float au, float ap, const float* x, float2* u, float* p,
                          uint32_t* blockmax, uint32_t* maxbits, uint32_t* host_out, hipStream_t s) {
  if (!N) return;
  const unsigned nb = grid_for(N);
  hipLaunchKernelGGL(k_update_fields, dim3(nb), dim3(kBlock), 0, s, N, au, ap, x, u, p, blockmax);
  hipLaunchKernelGGL(k_maxdiff_final, dim3(1), dim3(kBlock), 0, s, blockmax, nb, maxbits, host_out);
}
inline unsigned red_blocks(uint32_t N) {  // 4 chunks of 256 cells per 256-thread block
  const unsigned nch = (N + kRedChunkCells - 1) / kRedChunkCells;
  return (nch + 3) / 4;
}
void launch_dot_partial(const float* x, const float* y, uint32_t N, uint32_t U, float* partial, hipStream_t s) {
  if (N) hipLaunchKernelGGL(k_dot_partial, dim3(red_blocks(N)), dim3(kBlock), 0, s, x, y, N, U, partial);
}
void launch_ref_norm_partials(const float* v, uint32_t n3, float* partial, hipStream_t s) {
  const uint32_t ng = (n3 + 63) / 64;
  if (ng) hipLaunchKernelGGL(k_ref_norm_partials, dim3((ng + 3) / 4), dim3(256), 0, s, v, n3, partial, ng);
}
void launch_ref_cgs_dots(const float* w, const float* basis, const float* binv, size_t stride, int j, uint32_t n3,
                         float* partial, uint32_t pstride, hipStream_t s) {
  const uint32_t ng = (n3 + 63) / 64;
  if (ng)
    hipLaunchKernelGGL(k_ref_cgs_dots, dim3((ng + 3) / 4, (unsigned)(j + 1)), dim3(256), 0, s, w, basis, binv, stride,
                       n3, partial, pstride, ng);
}
void launch_reduce_final(const RedSrc& r, int mode, float* out, float* inv, float* g0, int g_len, float* host_out,
                         hipStream_t s) {
  hipLaunchKernelGGL(k_reduce_final, dim3(1), dim3(kRedFinalThreads), 0, s, r, mode, out, inv, g0, g_len,
                     host_out);
}
void launch_spmv(const CoupledMatrix& A, const float* x, float* y, hipStream_t s, const float* b, bool nt) {
  if (A.r1 <= A.r0 && A.r3 <= A.r2) return;
  const unsigned nb = rows2x_grid(A.r0, A.r1, A.r2, A.r3);
  auto fn = A.use16 ? (nt ? k_spmv2<true, true> : k_spmv2<true, false>)
                    : (nt ? k_spmv2<false, true> : k_spmv2<false, false>);
  hipLaunchKernelGGL(fn, dim3(nb), dim3(kBlock), 0, s, A, x, y, b);
}
bool cgs_latency_form(uint32_t N) { return N <= CFD_CGS_LAT_MAX_CELLS; }
void launch_cgs_dots(const float* w, const float* basis, const float* binv, size_t stride, int j, uint32_t N,
                     uint32_t U, float* partial, uint32_t np, hipStream_t s, size_t keep_bytes, bool lat) {
  if (!N) return;
  const uint32_t nb = red_blocks(N);
  if (lat) {
    if (!cgs_latency_form(N)) throw std::logic_error("launch_cgs_dots: latency form past its size limit");
    hipLaunchKernelGGL(k_cgs_dots_lat, dim3(nb, (unsigned)(j + kCgsLatDots) / kCgsLatDots), dim3(kBlock), 0, s, w,
                       basis, binv, stride, j, N, U, partial, np);
    return;
  }
  // the last blocks whose basis lines (j + 1 vectors + w, 12 B per cell each) fit keep_bytes
  const size_t keep_blocks = keep_bytes / ((size_t)(j + 2) * 12u * 1024u);
  const uint32_t tb = keep_blocks >= nb ? 0u : nb - (uint32_t)keep_blocks;
  if (N >= CFD_CGS_SER_MIN_CELLS)
    hipLaunchKernelGGL(k_cgs_dots<true>, dim3(nb), dim3(kBlock), 0, s, w, basis, binv, stride, j, N, U,
                       partial, np, tb);
  else
    hipLaunchKernelGGL(k_cgs_dots<false>, dim3(nb), dim3(kBlock), 0, s, w, basis, binv, stride, j, N, U,
                       partial, np, tb);
}
void launch_cgs_reduce(const RedSrc& r, int j, float* H, int m1, hipStream_t s) {
  hipLaunchKernelGGL(k_cgs_reduce, dim3(j + 1), dim3(kRedFinalThreads), 0, s, r, j, H, m1);
}
bool cgs_reduce_fusable(const RedSrc& r) {
  return !r.seg_src && (uint64_t)pow2_ceil(r.nseg) * r.G <= 256u;
}
void launch_cgs_update_norm(const float* w, float* basis, const float* binv, size_t stride, int j, float* H,
                            int m1, uint32_t N, uint32_t U, float* partial, hipStream_t s, bool rev, bool ntb,
                            const RedSrc* fr, bool lat) {
  if (!N) return;
  const bool ser = N >= CFD_CGS_SER_MIN_CELLS;
  if (fr && (ser || !cgs_reduce_fusable(*fr)))
    throw std::logic_error("launch_cgs_update_norm: fused CGS reduction past its size limit");
  if (lat && !cgs_latency_form(N)) throw std::logic_error("launch_cgs_update_norm: latency form past its size limit");
  if (lat) {  // default-policy loads and store (ntb and rev do not apply)
    hipLaunchKernelGGL(fr ? k_cgs_update_norm_lat<true> : k_cgs_update_norm_lat<false>, dim3((N + 1023) / 1024),
                       dim3(1024), 0, s, w, basis, binv, stride, j, H, m1, N, U, partial, fr ? *fr : RedSrc{});
    return;
  }
  auto fn = fr  ? (ntb ? k_cgs_update_norm<false, true, true> : k_cgs_update_norm<false, false, true>)
          : ser ? (ntb ? k_cgs_update_norm<true, true> : k_cgs_update_norm<true, false>)
                : (ntb ? k_cgs_update_norm<false, true> : k_cgs_update_norm<false, false>);
  hipLaunchKernelGGL(fn, dim3(red_blocks(N)), dim3(kBlock), 0, s, w, basis, binv, stride, j, H, m1, N, U, partial,
                     rev ? 1 : 0, fr ? *fr : RedSrc{});
}
void launch_norm_givens(const RedSrc& r, int j, float* H, int m1, float* givens, float* g, float* binv,
                        float* resid_hist, float* host_resid, hipStream_t s) {
  hipLaunchKernelGGL(k_norm_givens, dim3(1), dim3(kRedFinalThreads), 0, s, r, j, H, m1, givens, g, binv,
                     resid_hist, host_resid);
}
void launch_precond_predict(const CoupledMatrix& A, const float* w_in, const float* binv, int j,
                            const float* dinv_uv, const float* dinv_p, float* temp_p, float* p_sol,
                            float* p_prev, hipStream_t s, bool nt) {
  if (A.r1 <= A.r0 && A.r3 <= A.r2) return;
  const unsigned nb = rows2x_grid(A.r0, A.r1, A.r2, A.r3);
  auto fn = A.use16 ? (nt ? k_precond_predict2<true, true> : k_precond_predict2<true, false>)
                    : (nt ? k_precond_predict2<false, true> : k_precond_predict2<false, false>);
  hipLaunchKernelGGL(fn, dim3(nb), dim3(kBlock), 0, s, A, w_in, binv, j, dinv_uv, dinv_p, temp_p, p_sol, p_prev);
}
void launch_relax_pressure4(const AmgLevelDev& L, const uint8_t* drank, const float* dinv_p, const float* temp_p,
                            const float* src, float* dst, hipStream_t s) {
  if (L.r1 <= L.r0 && L.r3 <= L.r2) return;
  const unsigned nb = rows2_grid(L.r0, L.r1, L.r2, L.r3);
  if (L.use16)
    hipLaunchKernelGGL(k_relax_pressure4<true>, dim3(nb), dim3(kBlock), 0, s, L, drank, dinv_p, temp_p, src, dst);
  else
    hipLaunchKernelGGL(k_relax_pressure4<false>, dim3(nb), dim3(kBlock), 0, s, L, drank, dinv_p, temp_p, src, dst);
}
bool launch_relax_pressure_fused(uint32_t N, uint32_t ld, uint32_t ws, const int32_t* col, const uint32_t* len,
                                 const float* sval, const float* dinv_p, const float* temp_p, float* p_sol,
                                 float* temp, uint32_t iters, hipStream_t s) {
  if (N == 0 || N > kRelaxFusedMaxRows || iters == 0) return false;
  const size_t lds = 2 * ((size_t)kRelaxFusedMaxRows + 1) * sizeof(float);  // 64 KiB
  const dim3 g(1), b(kRelaxThreads);
  // ws = widest row incl. the diagonal: at most ws - 1 off-diagonal entries per row
#define CFD_RELAX_FUSED_CASE(RPT, OD)                                                                         \
  if (N <= (uint32_t)(RPT) * kRelaxThreads && ws <= (uint32_t)(OD) + 1u) {                                    \
    hipLaunchKernelGGL((k_relax_pressure_fused<RPT, OD>), g, b, lds, s, N, ld, col, len, sval, dinv_p, temp_p, \
                       p_sol, temp, iters);                                                                   \
    return true;                                                                                              \
  }
  CFD_RELAX_FUSED_CASE(1, 15)  // register budget at 1024 threads: 128 VGPRs (the 8 x 4 case spills 16)
  CFD_RELAX_FUSED_CASE(2, 15)
  CFD_RELAX_FUSED_CASE(4, 9)
  CFD_RELAX_FUSED_CASE(8, 4)
#undef CFD_RELAX_FUSED_CASE
  return false;
}
void launch_precond_correct(const CoupledMatrix& A, const float* w_in, const float* binv, int j,
                            const float* p_sol, const float* dinv_uv, float* z, hipStream_t s) {
  if (A.r1 <= A.r0 && A.r3 <= A.r2) return;
  const unsigned nb = rows2x_grid(A.r0, A.r1, A.r2, A.r3);
  if (A.use16)
    hipLaunchKernelGGL(k_precond_correct2<true>, dim3(nb), dim3(kBlock), 0, s, A, w_in, binv, j, p_sol, dinv_uv, z);
  else
    hipLaunchKernelGGL(k_precond_correct2<false>, dim3(nb), dim3(kBlock), 0, s, A, w_in, binv, j, p_sol, dinv_uv, z);
}
void launch_solve_triangular(const float* H, const float* g, float* y, int k, int m1, hipStream_t s) {
  if (k > 64 || m1 > 64) throw std::invalid_argument("solve_triangular: basis larger than 64");
  hipLaunchKernelGGL(k_solve_triangular, dim3(1), dim3(256), 0, s, H, g, y, k, m1);
}
void launch_update_x(float* x, const float* z, size_t stride, const float* y, int k, size_t n,
                     hipStream_t s, bool lat) {
  if (!n) return;
  if (lat && n / 3 <= CFD_CGS_LAT_MAX_CELLS && k > 2) {
    hipLaunchKernelGGL(k_update_x_lat, dim3(grid_for((n + 3) / 4)), dim3(kBlock), 0, s, x, z, stride, y, k, n);
    return;
  }
  if (n / 3 >= CFD_CGS_SER_MIN_CELLS)
    hipLaunchKernelGGL(k_update_x<true>, dim3(grid_for((n + 3) / 4)), dim3(kBlock), 0, s, x, z, stride, y, k, n);
  else
    hipLaunchKernelGGL(k_update_x<false>, dim3(grid_for((n + 3) / 4)), dim3(kBlock), 0, s, x, z, stride, y, k, n);
}
// instance for a level: 16/32-bit columns x load mode (see gather_group) x load policy
#define CFD_AMG_INSTANCE(kern, L, ...)                                                  \
  ((L).use16 ? ((L).full ? kern<true, 1, __VA_ARGS__> : kern<true, 0, __VA_ARGS__>) \
             : ((L).full ? kern<false, 1, __VA_ARGS__> : kern<false, 0, __VA_ARGS__>))

void launch_amg_smooth(const AmgLevelDev& L, const float* x, const float* b, float* x_out, hipStream_t s,
                       hipEvent_t ev0, hipEvent_t ev1, bool nt) {
  if (L.r1 <= L.r0 && L.r3 <= L.r2) return;
  const unsigned nb = rows2_grid(L.r0, L.r1, L.r2, L.r3);
  auto fn = nt ? CFD_AMG_INSTANCE(k_amg_smooth, L, false, true) : CFD_AMG_INSTANCE(k_amg_smooth, L, false, false);
  if (ev0)  // timed launch: events recorded by the GPU at kernel start / end
    hipExtLaunchKernelGGL(fn, dim3(nb), dim3(kBlock), 0, s, ev0, ev1, 0, CFD_AMG_HEAD(L), x, b, x_out, L,
                          (const float*)nullptr);
  else
    hipLaunchKernelGGL(fn, dim3(nb), dim3(kBlock), 0, s, CFD_AMG_HEAD(L), x, b, x_out, L, (const float*)nullptr);
}
void launch_amg_smooth_ordered(const AmgLevelDev& L, float* x, const float* b, hipStream_t s) {
  if (L.n == 0) return;
  auto fn = L.use16 ? (L.full ? k_amg_smooth_ordered<true, 1> : k_amg_smooth_ordered<true, 0>)
                    : (L.full ? k_amg_smooth_ordered<false, 1> : k_amg_smooth_ordered<false, 0>);
  hipLaunchKernelGGL(fn, dim3(1), dim3(16), 0, s, L, x, b);
}
void launch_amg_smooth_prolong(const AmgLevelDev& L, const float* x, const float* xc, const float* b, float* x_out,
                               hipStream_t s) {
  if (L.r1 <= L.r0 && L.r3 <= L.r2) return;
  if (!L.agg || !xc) throw std::invalid_argument("amg_smooth_prolong: level without a coarse level");
  const unsigned nb = rows2_grid(L.r0, L.r1, L.r2, L.r3);
  auto fn = L.use16 ? (L.full ? k_amg_smooth<true, 1, true> : k_amg_smooth<true, 0, true>)
                    : (L.full ? k_amg_smooth<false, 1, true> : k_amg_smooth<false, 0, true>);
  hipLaunchKernelGGL(fn, dim3(nb), dim3(kBlock), 0, s, CFD_AMG_HEAD(L), x, b, x_out, L, xc);
}
void launch_amg_smooth_zero(const AmgLevelDev& L, const float* b, float* x_out, hipStream_t s) {
  if (L.n) hipLaunchKernelGGL(k_amg_smooth_zero, dim3(grid_for((L.n + 3) / 4)), dim3(kBlock), 0, s, L, b, x_out);
}
void launch_amg_residual(const AmgLevelDev& L, const float* x, const float* b, float* r, hipStream_t s, bool nt) {
  if (L.r1 <= L.r0 && L.r3 <= L.r2) return;
  const unsigned nb = rows2_grid(L.r0, L.r1, L.r2, L.r3);
  auto fn = nt ? CFD_AMG_INSTANCE(k_amg_residual, L, true) : CFD_AMG_INSTANCE(k_amg_residual, L, false);
  hipLaunchKernelGGL(fn, dim3(nb), dim3(kBlock), 0, s, L, x, b, r);
}
void launch_amg_restrict(const AmgLevelDev& L, const float* r, float* cb, float* cx, uint32_t stride_c,
                         uint32_t glo, uint32_t ghi, hipStream_t s, float* sm_out, const float* sm_de, uint32_t I0,
                         uint32_t I1, bool ghosts) {
  if (I1 == 0) I1 = L.nc;
  const size_t n = (size_t)(I1 - I0) + (sm_out || !ghosts ? 0 : (size_t)glo + ghi);
  if (n)
    hipLaunchKernelGGL(k_amg_restrict, dim3(grid_for(n)), dim3(kBlock), 0, s, L, r, cb, cx, stride_c, glo, ghi,
                       sm_out, sm_de, I0, I1);
}
void launch_amg_resrestrict(const AmgLevelDev& L, const float* x, const float* b, float* cb, float* cx,
                            float* sm_out, const float* sm_de, hipStream_t s) {
  if (!L.nc || !L.rr_agg) return;
  const unsigned nb = (unsigned)((L.nc + L.rr_agg - 1) / L.rr_agg);
  if (L.use16)
    hipLaunchKernelGGL(k_amg_resrestrict<true>, dim3(nb), dim3(kBlock), 0, s, L, x, b, cb, cx, sm_out, sm_de);
  else
    hipLaunchKernelGGL(k_amg_resrestrict<false>, dim3(nb), dim3(kBlock), 0, s, L, x, b, cb, cx, sm_out, sm_de);
}
void launch_amg_prolong_smooth_pair(const AmgLevelDev& Lf, const AmgLevelDev& Lc, const AmgUpPairImage& P,
                                    const float* xf, const float* bf, float* xf_out, const float* xc,
                                    const float* bc, const float* xcc, hipStream_t s) {
  if (!P.nblocks) return;
  auto fn = Lf.use16 ? (Lc.use16 ? k_amg_prolong_smooth_pair<true, true> : k_amg_prolong_smooth_pair<true, false>)
                     : (Lc.use16 ? k_amg_prolong_smooth_pair<false, true> : k_amg_prolong_smooth_pair<false, false>);
  hipLaunchKernelGGL(fn, dim3(P.nblocks), dim3(kUpPairRows), 0, s, Lf, Lc, P, xf, bf, xf_out, xc, bc, xcc);
}
void launch_amg_resrestrict_pair(const AmgLevelDev& Lf, const AmgLevelDev& Lm, const AmgPairImage& P,
                                 const float* x, const float* b, float* bm, float* xm, float* cb, float* cx,
                                 float* sm_out, const float* sm_de, hipStream_t s) {
  if (!P.nblocks) return;
  auto fn = P.threads == 256 ? (Lf.use16 ? k_amg_resrestrict_pair<true, 256> : k_amg_resrestrict_pair<false, 256>)
                             : (Lf.use16 ? k_amg_resrestrict_pair<true, kPairThreads>
                                         : k_amg_resrestrict_pair<false, kPairThreads>);
  hipLaunchKernelGGL(fn, dim3(P.nblocks), dim3(P.threads), 0, s, Lf, Lm, P, x, b, bm, xm, cb, cx, sm_out, sm_de);
}
void launch_amg_prolong(const AmgLevelDev& L, float* x, const float* xc, hipStream_t s, uint32_t f0, uint32_t f1, bool nt) {
  if (f1 == 0) f1 = L.n;
  if (f1 > f0)
    hipLaunchKernelGGL(nt ? k_amg_prolong<true> : k_amg_prolong<false>, dim3(grid_for((f1 - f0 + 3) / 4)), dim3(kBlock), 0, s, L, x, xc, f0, f1);
}
void launch_amg_tail(const AmgTailLevel* tail, int first, int nlev, size_t lds_bytes, hipStream_t s) {
  if (lds_bytes == 0) {
    hipLaunchKernelGGL(k_amg_tail, dim3(1), dim3(1024), 0, s, tail, first, nlev);
    return;
  }
  hipLaunchKernelGGL(k_amg_tail_lds, dim3(1), dim3(1024), lds_bytes, s, tail, first, nlev);
}
void launch_amg_tail_blob(const AmgTailLevel* tail, const TailBlobLevel* desc, const uint32_t* blob,
                          uint32_t blob_words, uint32_t vec_floats, int first, int nlev, const float* b_first,
                          uint32_t n_first, hipStream_t s) {
  const size_t lds = 4 * ((size_t)vec_floats + blob_words);
  if (lds > kTailLdsMax || blob_words % 4 || blob_words == 0) throw std::invalid_argument("AMG tail blob larger than the kernel's LDS image");
  if (n_first == 0 || 16 * (size_t)n_first > kTailLdsMax) throw std::invalid_argument("AMG tail: first level size");
  hipLaunchKernelGGL(k_amg_tail_blob, dim3(1), dim3(1024), lds, s, tail, desc, blob, blob_words, vec_floats, first,
                     nlev, b_first, n_first);
}
// Per-device kernel attributes: the LDS-resident tail kernels take more than
// the default 64 KiB of dynamic LDS.  The attribute belongs to the device that
// is current when it is set, so each device gets it once (std::call_once per
// device id; the in-process group runs one host thread per rank and device).
// Returns the dynamic-LDS budget of those kernels on this device: the smaller
// of kTailLdsMax and the device's opt-in per-block limit.
size_t init_kernel_attributes(int device) {
  constexpr int kMaxDevices = 64;
  static std::once_flag once[kMaxDevices];
  static hipError_t status[kMaxDevices];
  static size_t budget[kMaxDevices];
  if (device < 0 || device >= kMaxDevices) throw std::invalid_argument("HIP device id out of range");
  std::call_once(once[device], [device] {
    int optin = 0;
    hipError_t e = hipDeviceGetAttribute(&optin, hipDeviceAttributeSharedMemPerBlockOptin, device);
    size_t lim = kTailLdsMax;
    if (e == hipSuccess && optin > 0) lim = std::min(lim, (size_t)optin);
    if (e == hipSuccess)
      e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_amg_tail_lds),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lim);
    if (e == hipSuccess)
      e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_amg_tail_blob),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lim);
    status[device] = e;
    budget[device] = lim;
  });
  if (status[device] != hipSuccess)
    throw std::runtime_error(std::string("setting the tail kernels' dynamic-LDS limit: ") +
                             hipGetErrorString(status[device]));
  return budget[device];
}
void launch_evolution_partial(StateView cur, StateView prev, int have_prev, uint32_t N, StateView var,
                              uint64_t gbase, uint64_t rec0, uint32_t U, double* partial, uint32_t np,
                              hipStream_t s) {
  if (N)
    hipLaunchKernelGGL(k_evolution_partial, dim3(red_blocks(N)), dim3(kBlock), 0, s, cur, prev, have_prev, N, var,
                       gbase, rec0, U, partial, np);
}
void launch_pack(const PackArgs& a, hipStream_t s) {
  if (a.n) hipLaunchKernelGGL(k_pack, dim3(grid_for(a.n)), dim3(kBlock), 0, s, a);
}
template <class T>
static void seg_reduce(const T* part, uint32_t np, uint32_t nchunks, uint32_t G, int nvec, T* out, uint32_t maxseg,
                       hipStream_t s) {
  if (nvec <= 0 || maxseg == 0) return;
  const unsigned nb = (maxseg + 3) / 4;
  hipLaunchKernelGGL(k_seg_reduce<T>, dim3(nb, (unsigned)nvec), dim3(kBlock), 0, s, part, np, nchunks, G, out,
                     maxseg);
}
void launch_seg_reduce(const float* part, uint32_t np, uint32_t nchunks, uint32_t G, int nvec, float* out,
                       uint32_t maxseg, hipStream_t s) {
  seg_reduce(part, np, nchunks, G, nvec, out, maxseg, s);
}
void launch_seg_reduce_d(const double* part, uint32_t np, uint32_t nchunks, uint32_t G, int nvec, double* out,
                         uint32_t maxseg, hipStream_t s) {
  seg_reduce(part, np, nchunks, G, nvec, out, maxseg, s);
}
void launch_max_combine(const uint32_t* gathered, int R, uint32_t* out, uint32_t* host_out, hipStream_t s) {
  hipLaunchKernelGGL(k_max_combine, dim3(1), dim3(64), 0, s, gathered, R, out, host_out);
}
void launch_evolution_final(const RedSrcD& r, double* out5, hipStream_t s) {
  hipLaunchKernelGGL(k_evolution_final, dim3(1), dim3(kRedFinalThreads), 0, s, r, out5);
}

void build_r_m4(const std::vector<uint32_t>& r_row, const std::vector<uint32_t>& r_col, std::vector<int32_t>& out) {
  const size_t nc = r_row.empty() ? 0 : r_row.size() - 1;
  out.assign(4 * nc, -1);
  for (size_t I = 0; I < nc; ++I) {
    const uint32_t k0 = r_row[I], m = r_row[I + 1] - k0;
    for (uint32_t q = 0; q < m && q < 4; ++q) out[4 * I + q] = (int32_t)r_col[k0 + q];
    if (m > 4) out[4 * I + 3] = -2 - (int32_t)r_col[k0 + 3];  // overflow flag; member 3 = -2 - w
  }
}

}  // namespace cfd2

