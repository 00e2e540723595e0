// Device-side AMG setup (amg_setup.hip): Galerkin product and level packing.
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>

namespace cfd2 {

// A fine level as the setup kernels read it: ELL slot-major (level 0, the
// assembled scalar matrix: entry k of row i at k*ld + i) or CSR (coarse
// levels).  Columns are signed local indices (global ids on one GPU and on
// replicated levels; owned-relative with ghosts below 0 / above npad on a
// distributed rank), sorted ascending within each row.
// Mode 2 (member rows, the distributed setup): CSR over the rows a rank's
// aggregates sum -- its own and the ones imported from the ranks that own
// them -- with GLOBAL fine column ids as `col` and each entry's coarse
// (aggregate) id in `eagg`, so no rank needs the aggregate of a column it
// does not hold.
struct SetupMatrix {
  int ell;                   // 0 CSR, 1 ELL, 2 member rows
  uint32_t ld;               // ELL slot stride
  const uint32_t* len;       // ELL row lengths
  const uint32_t* rowptr;    // CSR / member rows
  const int32_t* col;
  const float* val;
  const uint32_t* eagg;      // member rows: aggregate id of every entry's column
};

// per-thread capacities of k_galerkin; overflow (flag bit 1: members, bit 2:
// coarse columns) makes the host fall back to its own setup
constexpr int kSetupMaxMembers = 64;
constexpr int kSetupMaxCoarse = 128;

// rowptr_c == nullptr: count pass (cnt[I] = coarse row length); else fill pass.
void launch_galerkin(const SetupMatrix& A, const uint32_t* agg, const uint32_t* r_row, const uint32_t* r_col,
                     uint32_t nc, uint32_t* cnt, const uint32_t* rowptr_c, uint32_t* col_c, float* val_c,
                     uint32_t* overflow, hipStream_t s);
// dst[k] = src[idx[k]], k < n (value gathers of the distributed setup)
void launch_gather_f32(const float* src, const uint32_t* idx, uint32_t n, float* dst, hipStream_t s);
// AmgLevelDev arrays (val, col16 | col32, len, drank, dv, de) of rows [0, n), stride st, ELL width w
void launch_amg_pack(const SetupMatrix& A, uint32_t n, uint32_t st, int w, int use16, float* val, int16_t* col16,
                     int32_t* col32, uint8_t* len, uint8_t* drank, float* dv, float* de, hipStream_t s);

}  // namespace cfd2
