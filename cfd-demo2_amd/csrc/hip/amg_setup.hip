// gfx950 kernels of the device-side AMG setup: the
// Galerkin product A_c = (R A) P of linear_solver/amg.rs:187-235 and the
// packing of a level into the layout the V-cycle kernels stream
// (AmgLevelDev).  The greedy index-order aggregation (amg.rs:84-116) stays on
// the host: its sequential first-come semantics are the reference's, it only
// needs the sparsity pattern, and it is O(nnz).
//
// Bit-exactness with the reference's (and the host path's) f32 arithmetic:
// amg.rs multiplies by the unit entries of R and P (1.0f * a == a) and
// accumulates in a HashMap per row in visit order, then sorts the columns.
// For a coarse row I with fine members i_1 < i_2 < ... (R row I):
//   RA[I, j] = ((0 + a[i_1, j]) + a[i_2, j]) + ...   over the members holding column j
//   Ac[I, J] = ((0 + RA[I, j_1]) + RA[I, j_2]) + ... over j ascending with agg[j] = J
// One thread per coarse row walks the members' (column-sorted) rows as a
// k-way merge, so each RA[I, j] is complete, in member order, when column j
// is emitted, and columns are emitted in ascending order -- exactly the
// accumulation order above -- then sorts its few coarse columns.
#include <hip/hip_runtime.h>

#include "amg_setup.hpp"

namespace cfd2 {

namespace {

constexpr int kBlock = 256;

inline unsigned grid_for(size_t n) { return (unsigned)((n + kBlock - 1) / kBlock); }

// entry k of fine row i: ELL slot-major (level 0: the scalar pressure matrix
// as assembled) or CSR (coarse levels produced by k_galerkin)
template <int MODE>  // SetupMatrix::ell
struct Rows {
  SetupMatrix m;
  __device__ __forceinline__ uint32_t len(uint32_t i) const {
    if constexpr (MODE == 1)
      return m.len[i];
    else
      return m.rowptr[i + 1] - m.rowptr[i];
  }
  __device__ __forceinline__ size_t at(uint32_t i, uint32_t k) const {
    if constexpr (MODE == 1)
      return (size_t)k * m.ld + i;
    else
      return (size_t)m.rowptr[i] + k;
  }
  __device__ __forceinline__ int32_t col(uint32_t i, uint32_t k) const { return m.col[at(i, k)]; }
  __device__ __forceinline__ float val(uint32_t i, uint32_t k) const { return m.val[at(i, k)]; }
};

// FILL = false: cnt[I] = number of distinct coarse columns of row I.
// FILL = true: the sorted row written at rowptr_c[I].  `agg` is indexed by
// the fine column (modes 0 / 1); member rows (mode 2) carry the aggregate of
// every entry instead.
template <int MODE, bool FILL>
__global__ void __launch_bounds__(kBlock) k_galerkin(SetupMatrix A, const uint32_t* __restrict__ agg,
                                                     const uint32_t* __restrict__ r_row,
                                                     const uint32_t* __restrict__ r_col, uint32_t nc,
                                                     uint32_t* __restrict__ cnt,
                                                     const uint32_t* __restrict__ rowptr_c,
                                                     uint32_t* __restrict__ col_c, float* __restrict__ val_c,
                                                     uint32_t* overflow) {
  const uint32_t I = blockIdx.x * kBlock + threadIdx.x;
  if (I >= nc) return;
  const Rows<MODE> a{A};
  const uint32_t k0 = r_row[I], m = r_row[I + 1] - k0;
  if (m > (uint32_t)kSetupMaxMembers) {
    atomicOr(overflow, 1u);
    return;
  }
  uint32_t mem[kSetupMaxMembers], cur[kSetupMaxMembers], end[kSetupMaxMembers];
  for (uint32_t t = 0; t < m; ++t) {
    mem[t] = r_col[k0 + t];
    cur[t] = 0;
    end[t] = a.len(mem[t]);
  }
  uint32_t cj[kSetupMaxCoarse];
  float cv[kSetupMaxCoarse];
  uint32_t nl = 0;
  for (;;) {
    // columns are signed local indices (ghosts of lower ranks < 0): local order == global order
    int32_t jmin = INT32_MAX;
    for (uint32_t t = 0; t < m; ++t)
      if (cur[t] < end[t]) jmin = min(jmin, a.col(mem[t], cur[t]));
    if (jmin == INT32_MAX) break;
    float ra = 0.0f;  // RA[I, jmin], members in ascending order (first touch: 0 + ...)
    uint32_t J = 0;
    bool first = true;
    for (uint32_t t = 0; t < m; ++t)
      if (cur[t] < end[t] && a.col(mem[t], cur[t]) == jmin) {
        if constexpr (MODE == 2)
          if (first) J = A.eagg[a.at(mem[t], cur[t])];
        first = false;
        ra += 1.0f * a.val(mem[t], cur[t]);
        ++cur[t];
      }
    if constexpr (MODE != 2) J = agg[jmin];
    uint32_t q = 0;
    while (q < nl && cj[q] != J) ++q;
    if (q == nl) {
      if (nl == (uint32_t)kSetupMaxCoarse) {
        atomicOr(overflow, 2u);
        return;
      }
      cj[nl] = J;
      cv[nl] = 0.0f;
      ++nl;
    }
    cv[q] += ra * 1.0f;
  }
  if constexpr (!FILL) {
    cnt[I] = nl;
  } else {
    for (uint32_t p = 1; p < nl; ++p) {  // insertion sort by coarse column (unique keys)
      const uint32_t kj = cj[p];
      const float kv = cv[p];
      uint32_t q = p;
      while (q > 0 && cj[q - 1] > kj) {
        cj[q] = cj[q - 1];
        cv[q] = cv[q - 1];
        --q;
      }
      cj[q] = kj;
      cv[q] = kv;
    }
    const uint32_t o = rowptr_c[I];
    for (uint32_t p = 0; p < nl; ++p) {
      col_c[o + p] = cj[p];
      val_c[o + p] = cv[p];
    }
  }
}

// Level image (AmgLevelDev) of rows [0, n) with stride st: off-diagonals in
// ELL slot-major order (row order kept), diagonal value and rank, smoother
// diagonal (amg.wgsl:46: 1.0 when |diag| < 1e-14); padding slots / rows hold
// value 0 and the row's own column.  Same bytes as the host level_image.
template <int MODE>
__global__ void __launch_bounds__(kBlock) k_amg_pack(SetupMatrix A, uint32_t n, uint32_t st, int w, int use16,
                                                     float* __restrict__ val, int16_t* __restrict__ col16,
                                                     int32_t* __restrict__ col32, uint8_t* __restrict__ len,
                                                     uint8_t* __restrict__ drank, float* __restrict__ dv,
                                                     float* __restrict__ de) {
  const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= st) return;
  const Rows<MODE> a{A};
  uint32_t off = 0, dr = 0;
  float diag = 1.0f, raw = 0.0f;
  if (i < n) {
    bool has = false;
    const uint32_t l = a.len(i);
    for (uint32_t k = 0; k < l; ++k) {
      const int32_t c = a.col(i, k);
      const float v = a.val(i, k);
      if (c == (int32_t)i) {
        has = true;
        raw = v;
        diag = raw;
        dr = off;
      } else {
        const size_t o = (size_t)off * st + i;
        val[o] = v;
        if (use16)
          col16[o] = (int16_t)(c - (int32_t)i);
        else
          col32[o] = c;
        ++off;
      }
    }
    if (!has) dr = off;
    if (fabsf(diag) < 1e-14f) diag = 1.0f;
  }
  for (uint32_t r = off; r < (uint32_t)max(w, 1); ++r) {
    const size_t o = (size_t)r * st + i;
    val[o] = 0.0f;
    if (use16)
      col16[o] = 0;
    else
      col32[o] = (int32_t)i;
  }
  len[i] = (uint8_t)off;
  drank[i] = (uint8_t)dr;
  dv[i] = raw;
  de[i] = diag;
}

__global__ void __launch_bounds__(kBlock) k_gather_f32(const float* __restrict__ src, const uint32_t* __restrict__ idx,
                                                       uint32_t n, float* __restrict__ dst) {
  const uint32_t k = blockIdx.x * kBlock + threadIdx.x;
  if (k < n) dst[k] = src[idx[k]];
}

template <bool FILL>
void galerkin_mode(const SetupMatrix& A, const uint32_t* agg, const uint32_t* r_row, const uint32_t* r_col,
                   uint32_t nc, uint32_t* cnt, const uint32_t* rowptr_c, uint32_t* col_c, float* val_c,
                   uint32_t* overflow, hipStream_t s) {
  if (A.ell == 1)
    hipLaunchKernelGGL((k_galerkin<1, FILL>), dim3(grid_for(nc)), dim3(kBlock), 0, s, A, agg, r_row, r_col, nc, cnt,
                       rowptr_c, col_c, val_c, overflow);
  else if (A.ell == 2)
    hipLaunchKernelGGL((k_galerkin<2, FILL>), dim3(grid_for(nc)), dim3(kBlock), 0, s, A, agg, r_row, r_col, nc, cnt,
                       rowptr_c, col_c, val_c, overflow);
  else
    hipLaunchKernelGGL((k_galerkin<0, FILL>), dim3(grid_for(nc)), dim3(kBlock), 0, s, A, agg, r_row, r_col, nc, cnt,
                       rowptr_c, col_c, val_c, overflow);
}

}  // namespace

void launch_gather_f32(const float* src, const uint32_t* idx, uint32_t n, float* dst, hipStream_t s) {
  if (n) hipLaunchKernelGGL(k_gather_f32, dim3(grid_for(n)), dim3(kBlock), 0, s, src, idx, n, dst);
}

void launch_galerkin(const SetupMatrix& A, const uint32_t* agg, const uint32_t* r_row, const uint32_t* r_col,
                     uint32_t nc, uint32_t* cnt, const uint32_t* rowptr_c, uint32_t* col_c, float* val_c,
                     uint32_t* overflow, hipStream_t s) {
  if (!nc) return;
  if (rowptr_c != nullptr)
    galerkin_mode<true>(A, agg, r_row, r_col, nc, cnt, rowptr_c, col_c, val_c, overflow, s);
  else
    galerkin_mode<false>(A, agg, r_row, r_col, nc, cnt, rowptr_c, col_c, val_c, overflow, s);
}

void launch_amg_pack(const SetupMatrix& A, uint32_t n, uint32_t st, int w, int use16, float* val, int16_t* col16,
                     int32_t* col32, uint8_t* len, uint8_t* drank, float* dv, float* de, hipStream_t s) {
  if (!st) return;
  if (A.ell == 1)
    hipLaunchKernelGGL(k_amg_pack<1>, dim3(grid_for(st)), dim3(kBlock), 0, s, A, n, st, w, use16, val, col16,
                       col32, len, drank, dv, de);
  else
    hipLaunchKernelGGL(k_amg_pack<0>, dim3(grid_for(st)), dim3(kBlock), 0, s, A, n, st, w, use16, val, col16,
                       col32, len, drank, dv, de);
}

}  // namespace cfd2
