// Device-side AMG setup, one GPU or distributed.
//
// The reference builds its hierarchy on the host after a blocking readback of
// the scalar matrix (linear_solver/amg.rs:246-664).  Here the matrix never
// leaves the GPU: per level
//   host   greedy aggregation on the sparsity pattern (amg.rs:84-116; the
//          sequential first-come order is the reference's semantics), R = P^T
//   device count pass of the Galerkin product (distinct coarse columns per row)
//   host   exclusive scan of the counts -> coarse row pointers
//   device fill pass: sorted coarse rows with the reference's f32
//          accumulation order (amg_setup.hip), packing of the fine level into
//          the V-cycle layout (AmgLevelDev)
//   host   download of the coarse pattern (the next aggregation's input)
// Level 0 is read straight from the assembled ELL scalar matrix.  The result
// is bit-identical to the host path (tests/test_gpu_parity.py compares both);
// should a coarse row exceed the kernel's per-thread capacities, or a level
// need the wide-row layout, the host path runs instead.  A distributed solver
// always takes the host path: its hierarchy is the global one (the same on
// every rank count), built from the all-gathered matrix.
#include <chrono>
#include <cstdio>
#include <cstdlib>

#include "../hip/amg_setup.hpp"
#include "solver_impl.hpp"

namespace cfd2 {

namespace {

// temporary device buffer (setup scratch; the arena holds what the V-cycle keeps)
template <class T>
struct DevTmp {
  T* p = nullptr;
  DevTmp() = default;
  explicit DevTmp(size_t n) { CFD_HIP(hipMalloc(&p, (n ? n : 1) * sizeof(T))); }
  DevTmp(const DevTmp&) = delete;
  DevTmp& operator=(const DevTmp&) = delete;
  DevTmp(DevTmp&& o) noexcept : p(o.p) { o.p = nullptr; }
  DevTmp& operator=(DevTmp&& o) noexcept {
    if (this != &o) {
      if (p) (void)hipFree(p);
      p = o.p;
      o.p = nullptr;
    }
    return *this;
  }
  ~DevTmp() {
    if (p) (void)hipFree(p);
  }
};

// a level as the setup sees it: pattern on the host, values on the device
struct SetupLevel {
  uint32_t n = 0;                  // rows
  const uint32_t* row = nullptr;   // host pattern over rows [0, n) (relative), global columns
  const uint32_t* col = nullptr;
  std::vector<uint32_t> own_row, own_col;  // storage of a downloaded coarse pattern
  SetupMatrix dev{};
  // device CSR of a coarse level: kept (amg_arena) for the numeric re-setup
  uint32_t* d_rowptr = nullptr;
  int32_t* d_col = nullptr;
  float* d_val = nullptr;
};

}  // namespace

// Per level: packing of the level on the device, aggregation + R on the host,
// Galerkin count / fill on the device, download of the coarse pattern.
bool Solver::build_amg_device() {
  if (dist()) return false;  // the global hierarchy of a distributed solver: host path
  const bool timing = std::getenv("CFD_AMG_SETUP_TIMING") != nullptr;
  using clk = std::chrono::steady_clock;
  auto secs = [](clk::time_point a) { return std::chrono::duration<double>(clk::now() - a).count(); };
  levels.clear();
  amg_refresh.clear();
  amg_g = 0;
  auto zeroed = [&](size_t cnt) {
    float* p = arena.alloc<float>(cnt + 64);
    CFD_HIP(hipMemsetAsync(p, 0, (cnt + 64) * sizeof(float), stream));
    return p;
  };
  amg_setup_flag = arena.alloc<uint32_t>(1);
  CFD_HIP(hipMemsetAsync(amg_setup_flag, 0, sizeof(uint32_t), stream));

  SetupLevel cur;
  cur.n = N;
  cur.row = topo.srow.data();
  cur.col = topo.scol.data();
  cur.dev.ell = 1;
  cur.dev.ld = topo.ld;
  cur.dev.len = d_slen;
  cur.dev.col = d_scol;  // global ids on one GPU
  cur.dev.val = sval;

  for (int li = 0; li < kMaxAmgLevels; ++li) {
    const auto t0 = clk::now();
    const uint32_t n = cur.n;
    levels.emplace_back();
    AmgGpuLevel& G = levels.back();
    G.nglob = n;
    G.part = {0, (uint64_t)n};
    G.C0 = 0;
    G.C1 = n;
    // ---- level image (same bytes as the host level_image)
    int wmax = 0;
    bool small_delta = true;
    const uint32_t* crow = cur.row;
    const uint32_t* ccol = cur.col;
#pragma omp parallel for reduction(max : wmax) reduction(&& : small_delta) schedule(static)
    for (long ii = 0; ii < (long)n; ++ii) {
      const uint32_t i = (uint32_t)ii;
      int off = 0;
      for (uint32_t k = crow[i]; k < crow[i + 1]; ++k) {
        const int64_t c = (int64_t)ccol[k];
        if (c == (int64_t)i) continue;
        ++off;
        const int64_t d = c - (int64_t)i;
        if (d < -32768 || d > 32767) small_delta = false;
      }
      wmax = std::max(wmax, off);
    }
    // a row wider than the u8 layout: the host path builds that level with 16-bit lengths
    if (wmax > amg_wide_limit) {
      if (timing) std::fprintf(stderr, "[amg setup] device path: wide rows at level %d, host path\n", li);
      levels.clear();
      amg_refresh.clear();
      return false;
    }
    const uint32_t st = (n + 63) & ~63u;
    const size_t slots = (size_t)std::max(wmax, 1) * st;
    G.nnz = cur.row[n] - cur.row[0];
    G.dev.n = n;
    G.dev.r0 = 0;
    G.dev.r1 = n;
    G.dev.stride = st;
    G.dev.w = wmax;
    G.dev.use16 = small_delta ? 1 : 0;
    float* val = arena.alloc<float>(slots);
    int16_t* col16 = small_delta ? arena.alloc<int16_t>(slots) : nullptr;
    int32_t* col32 = small_delta ? nullptr : arena.alloc<int32_t>(slots);
    uint8_t* len = arena.alloc<uint8_t>(st);
    uint8_t* drank = arena.alloc<uint8_t>(st);
    float* dv = arena.alloc<float>(st);
    float* de = arena.alloc<float>(st);
    launch_amg_pack(cur.dev, n, st, wmax, G.dev.use16, val, col16, col32, len, drank, dv, de, stream);
    CFD_HIP(hipGetLastError());
    G.dev.val = val;
    G.dev.col16 = col16;
    G.dev.col32 = col32;
    G.dev.len = len;
    G.dev.drank = drank;
    G.dev.dv = dv;
    G.dev.de = de;
    amg_refresh.emplace_back();
    amg_refresh.back().fine = cur.dev;
    G.npad = st;
    G.xt = zeroed(st);
    G.r = zeroed(st);
    if (li > 0) {
      G.x = zeroed(st);
      G.b = zeroed(st);
    }
    set_amg_full_policy(G, li);
    // ---- coarsening (amg.rs:374-595: stop at n <= 100, no reduction or the level cap)
    if (!(li < kMaxAmgLevels - 1 && n > 100)) break;
    std::vector<uint32_t> agg, r_row, r_col;
    std::vector<uint64_t> cpart;
    const uint32_t nagg = aggregate_greedy(n, cur.row, cur.col, {0, (uint64_t)n}, agg, cpart);
    if (nagg >= n) break;
    transpose_aggregates(agg, nagg, r_row, r_col);
    const double t_agg = secs(t0);
    std::vector<uint32_t> aggp(st, 0);
    for (uint32_t i = 0; i < n; ++i) aggp[i] = agg[i];
    G.dev.agg = arena.upload(aggp, stream);
    G.dev.r_row = arena.upload(r_row, stream);
    G.dev.r_col = arena.upload(r_col, stream);
    {
      std::vector<int32_t> m4;
      build_r_m4(r_row, r_col, m4);
      G.dev.r_m4 = reinterpret_cast<const int4*>(arena.upload(m4, stream));
    }
    G.dev.nc = nagg;
    const uint32_t* gal_agg = G.dev.agg;  // Galerkin columns: aggregate id of every fine column
    // ---- Galerkin product on the device
    SetupLevel next;
    next.n = nagg;
    DevTmp<uint32_t> d_cnt(nagg);
    launch_galerkin(cur.dev, gal_agg, G.dev.r_row, G.dev.r_col, nagg, d_cnt.p, nullptr, nullptr, nullptr,
                    amg_setup_flag, stream);
    CFD_HIP(hipGetLastError());
    next.own_row.assign((size_t)nagg + 1, 0);
    uint32_t flag = 0;
    CFD_HIP(hipMemcpyAsync(next.own_row.data() + 1, d_cnt.p, (size_t)nagg * sizeof(uint32_t),
                           hipMemcpyDeviceToHost, stream));
    CFD_HIP(hipMemcpyAsync(&flag, amg_setup_flag, sizeof(uint32_t), hipMemcpyDeviceToHost, stream));
    sync();
    if (flag != 0) {
      if (timing) std::fprintf(stderr, "[amg setup] device path: capacity overflow at level %d\n", li);
      levels.clear();
      amg_refresh.clear();
      return false;
    }
    for (uint32_t I = 0; I < nagg; ++I) next.own_row[I + 1] += next.own_row[I];
    const size_t nnz_c = next.own_row[nagg];
    next.d_rowptr = arena.alloc<uint32_t>((size_t)nagg + 1);
    next.d_col = arena.alloc<int32_t>(nnz_c);
    next.d_val = arena.alloc<float>(nnz_c);
    CFD_HIP(hipMemcpyAsync(next.d_rowptr, next.own_row.data(), ((size_t)nagg + 1) * sizeof(uint32_t),
                           hipMemcpyHostToDevice, stream));
    launch_galerkin(cur.dev, gal_agg, G.dev.r_row, G.dev.r_col, nagg, nullptr, next.d_rowptr,
                    reinterpret_cast<uint32_t*>(next.d_col), next.d_val, amg_setup_flag, stream);
    CFD_HIP(hipGetLastError());
    {
      AmgRefreshLevel& F = amg_refresh.back();
      F.has_coarse = true;
      F.gal_agg = gal_agg;
      F.nagg_own = nagg;
      F.rowptr_c = next.d_rowptr;
      F.col_c = reinterpret_cast<uint32_t*>(next.d_col);
      F.val_c = next.d_val;
      F.nnz_own = nnz_c;
    }
    next.own_col.resize(nnz_c);
    CFD_HIP(hipMemcpyAsync(next.own_col.data(), next.d_col, nnz_c * sizeof(uint32_t), hipMemcpyDeviceToHost,
                           stream));
    sync();  // the fine level's buffers may be released after this
    next.row = next.own_row.data();
    next.col = next.own_col.data();
    next.dev.ell = 0;
    next.dev.rowptr = next.d_rowptr;
    next.dev.col = next.d_col;
    next.dev.val = next.d_val;
    if (timing)
      std::fprintf(stderr, "[amg setup] device level %d: n=%u nagg=%u nnz_c=%zu  aggregate+R %.3fs  total %.3fs\n",
                   li, n, nagg, nnz_c, t_agg, secs(t0));
    cur = std::move(next);
  }
  sync();
  return true;
}

// Numeric re-setup from the current matrix (cfg.amg_rebuild_interval): the
// structure built by build_amg_device is value-independent (aggregation and
// R on the pattern, Galerkin patterns structural -- explicit zeros are kept,
// as amg.rs keeps them), so packing every level and re-running the Galerkin
// fill over it in level order gives the bytes a full rebuild gives
// (tests/test_gpu_parity.py::test_amg_refresh_matches_full_rebuild).
void Solver::refresh_amg() {
  const size_t slots_s = (size_t)topo.ws * topo.ld;
  CFD_HIP(hipMemcpyAsync(amg_src, sval, slots_s * sizeof(float), hipMemcpyDeviceToDevice, stream));
  for (size_t li = 0; li < amg_refresh.size(); ++li) {
    const AmgRefreshLevel& F = amg_refresh[li];
    const AmgLevelDev& d = levels[li].dev;
    launch_amg_pack(F.fine, d.n, d.stride, d.w, d.use16, const_cast<float*>(d.val), const_cast<int16_t*>(d.col16),
                    const_cast<int32_t*>(d.col32), const_cast<uint8_t*>(d.len), const_cast<uint8_t*>(d.drank),
                    const_cast<float*>(d.dv), const_cast<float*>(d.de), stream);
    if (!F.has_coarse) continue;
    launch_galerkin(F.fine, F.gal_agg, d.r_row, d.r_col, F.nagg_own, nullptr, F.rowptr_c, F.col_c, F.val_c,
                    amg_setup_flag, stream);
  }
  CFD_HIP(hipGetLastError());
  if (tail_blob_first >= 0) build_tail_blob(tail_blob_first, true);
  sync();
}

}  // namespace cfd2
