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
// is bit-identical to the host path (tests/test_gpu_parity.py and
// tests/test_gpu_dist.py compare both); should a coarse row exceed the
// kernel's per-thread capacities (on any rank) the host path runs instead.
// A distributed rank never sees the whole fine matrix: only the first
// replicated level is all-gathered.
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
  bool dist = false;               // rows partitioned over the ranks (else replicated / one GPU)
  std::vector<uint64_t> part;      // global row partition of the level over the ranks
  uint32_t n = 0;                  // rows this rank holds (own rows if dist)
  const uint32_t* row = nullptr;   // host pattern over rows [0, n) (relative), global columns
  const uint32_t* col = nullptr;
  std::vector<uint32_t> own_row, own_col;  // storage of a downloaded coarse pattern
  SetupMatrix dev{};
  // device CSR of a coarse level: kept (amg_arena) for the numeric re-setup
  uint32_t* d_rowptr = nullptr;
  int32_t* d_col = nullptr;     // global columns
  int32_t* d_relcol = nullptr;  // distributed level: signed local columns
  float* d_val = nullptr;
};

}  // namespace

// Per level (dist: this rank's rows; replicated levels: every rank builds the
// same rows, as the host path does):
//   image    ghosts + halo plan (dist), level packing on the device
//   host     aggregation of the level's own part (aggregates never cross a
//            part), aggregate counts all-gathered -> coarse partition
//   device   Galerkin count / fill for this rank's aggregates; on a
//            distributed level the aggregate ids of the ghost columns arrive
//            by one halo exchange of the (global) agg vector
//   comm     the first replicated level is all-gathered (row lengths,
//            columns, values) so every rank holds it whole
bool Solver::build_amg_device() {
  const bool timing = std::getenv("CFD_AMG_SETUP_TIMING") != nullptr;
  using clk = std::chrono::steady_clock;
  auto secs = [](clk::time_point a) { return std::chrono::duration<double>(clk::now() - a).count(); };
  levels.clear();
  amg_refresh.clear();
  const char* rep_env = std::getenv("CFD_AMG_REPLICATE_ROWS");
  const uint64_t rep = rep_env ? std::strtoull(rep_env, nullptr, 10) : 262144u;
  amg_g = -1;
  auto zeroed = [&](size_t cnt) {
    float* p = arena.alloc<float>(cnt + 64);
    CFD_HIP(hipMemsetAsync(p, 0, (cnt + 64) * sizeof(float), stream));
    return p;
  };
  amg_setup_flag = arena.alloc<uint32_t>(1);
  CFD_HIP(hipMemsetAsync(amg_setup_flag, 0, sizeof(uint32_t), stream));
  auto gather_counts = [&](uint64_t mine) { return allgather_u64(mine); };

  SetupLevel cur;
  cur.dist = dist();
  cur.part = starts;
  cur.n = N;
  cur.row = topo.srow.data();
  cur.col = topo.scol.data();
  cur.dev.ell = 1;
  cur.dev.ld = topo.ld;
  cur.dev.len = d_slen;
  cur.dev.col = d_scol;  // signed local columns (global ids on one GPU)
  cur.dev.val = sval;

  for (int li = 0; li < kMaxAmgLevels; ++li) {
    const auto t0 = clk::now();
    const uint32_t n = cur.n;
    const uint64_t nglob = cur.part.back();
    levels.emplace_back();
    AmgGpuLevel& G = levels.back();
    G.nglob = nglob;
    G.part = cur.part;
    G.C0 = cur.part[rk];
    G.C1 = cur.part[rk + 1];
    // ---- level image (same bytes as the host level_image)
    std::vector<uint32_t> ghost;
    std::vector<int32_t> rcol;  // distributed: signed local column of every entry
    if (cur.dist) {
      G.dist = true;
      G.glo = collect_ghosts(G.C0, G.C1, cur.row, n, cur.col, ghost);
      G.ghi = (uint32_t)ghost.size() - G.glo;
      G.npad = (n + 63) & ~63u;
      const uint64_t C0 = G.C0, C1 = G.C1;
      const uint32_t glo = G.glo, npad = G.npad;
      const size_t nnz = cur.row[n] - cur.row[0];
      rcol.resize(nnz);
#pragma omp parallel for schedule(static)
      for (long k = 0; k < (long)nnz; ++k) {
        const uint32_t c = cur.col[cur.row[0] + k];
        if (c >= C0 && c < C1) {
          rcol[k] = (int32_t)(c - C0);
        } else {
          const uint32_t q = (uint32_t)(std::lower_bound(ghost.begin(), ghost.end(), c) - ghost.begin());
          rcol[k] = q < glo ? (int32_t)q - (int32_t)glo : (int32_t)(npad + (q - glo));
        }
      }
      G.plan = build_halo_plan(cur.part, rk, cur.row, n, cur.col, ghost, G.glo, G.npad);
      make_plan_buffers(G.plan, 1);
      if (li > 0) {  // level 0's device columns (d_scol) are local already
        cur.d_relcol = arena.alloc<int32_t>(nnz);
        CFD_HIP(hipMemcpyAsync(cur.d_relcol, rcol.data(), nnz * sizeof(int32_t), hipMemcpyHostToDevice, stream));
        cur.dev.col = cur.d_relcol;
      }
    }
    int wmax = 0;
    bool small_delta = true;
    const uint32_t* crow = cur.row;
    const uint32_t* ccol = cur.col;
    const int32_t* rc = rcol.data();
    const bool dl = cur.dist;
#pragma omp parallel for reduction(max : wmax) reduction(&& : small_delta) schedule(static)
    for (long ii = 0; ii < (long)n; ++ii) {
      const uint32_t i = (uint32_t)ii;
      int off = 0;
      for (uint32_t k = crow[i]; k < crow[i + 1]; ++k) {
        const int64_t c = dl ? (int64_t)rc[k - crow[0]] : (int64_t)ccol[k];
        if (c == (int64_t)i) continue;
        ++off;
        const int64_t d = c - (int64_t)i;
        if (d < -32768 || d > 32767) small_delta = false;
      }
      wmax = std::max(wmax, off);
    }
    // a row wider than the u8 layout: the host path builds that level with
    // 16-bit lengths (every rank must take the same path: combined over ranks)
    {
      bool wide = wmax > amg_wide_limit;
      if (dist()) {
        const std::vector<uint64_t> fl = gather_counts(wide ? 1u : 0u);
        for (uint64_t f : fl) wide = wide || f != 0;
      }
      if (wide) {
        if (timing) std::fprintf(stderr, "[amg setup] device path: wide rows at level %d, host path\n", li);
        levels.clear();
        amg_refresh.clear();
        return false;
      }
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
    uint32_t sh = 0;  // ghost space below the owned rows of a distributed level's vectors
    if (cur.dist) {
      sh = (G.glo + 63) & ~63u;
      if (li == 0) {
        if (G.glo != topo.glo || G.ghi != topo.ghi || G.npad != topo.npad)
          throw std::logic_error("AMG level 0 ghosts differ from the cell ghosts");
        G.xt = valloc<float>(1);
        G.r = valloc<float>(1);
      } else {
        const size_t cnt = (size_t)sh + G.npad + G.ghi;
        G.x = zeroed(cnt) + sh;
        G.xt = zeroed(cnt) + sh;
        G.b = zeroed(cnt) + sh;
        G.r = zeroed(cnt) + sh;
      }
    } else {
      G.npad = st;
      G.xt = zeroed(st);
      G.r = zeroed(st);
      if (li > 0) {
        G.x = zeroed(st);
        G.b = zeroed(st);
      }
    }
    set_amg_full_policy(G, li);
    // ---- coarsening (amg.rs:374-595: stop at n <= 100, no reduction or the level cap)
    if (!(li < kMaxAmgLevels - 1 && nglob > 100)) break;
    std::vector<uint32_t> agg, r_row, r_col;
    std::vector<uint64_t> cpart;
    uint32_t nagg_own = 0;
    if (cur.dist) {  // own part only: columns outside it never join an aggregate
      const size_t nnz = rcol.size();
      std::vector<uint32_t> lc(nnz);
      for (size_t k = 0; k < nnz; ++k) lc[k] = rcol[k] >= 0 && (uint32_t)rcol[k] < n ? (uint32_t)rcol[k] : 0xFFFFFFFFu;
      std::vector<uint32_t> lrow(cur.row, cur.row + n + 1);
      for (auto& v : lrow) v -= cur.row[0];
      std::vector<uint64_t> lp;
      nagg_own = aggregate_greedy(n, lrow.data(), lc.data(), {0, (uint64_t)n}, agg, lp);
      const std::vector<uint64_t> cnts = gather_counts(nagg_own);
      cpart.assign(R + 1, 0);
      for (int q = 0; q < R; ++q) cpart[q + 1] = cpart[q] + cnts[q];
    } else {
      nagg_own = aggregate_greedy(n, cur.row, cur.col, cur.part, agg, cpart);
    }
    const uint64_t nagg_glob = cpart.back();
    if (nagg_glob >= nglob) break;
    const bool next_dist = cur.dist && nagg_glob > rep;
    if (cur.dist && !next_dist) amg_g = li + 1;
    transpose_aggregates(agg, nagg_own, r_row, r_col);  // local fine rows when distributed
    const double t_agg = secs(t0);
    // V-cycle P: local coarse ids into a distributed next level, global ids into a replicated one
    const uint32_t vbase = (cur.dist && !next_dist) ? (uint32_t)cpart[rk] : 0u;
    std::vector<uint32_t> aggp(st, 0);
    for (uint32_t i = 0; i < n; ++i) aggp[i] = agg[i] + vbase;
    G.dev.agg = arena.upload(aggp, stream);
    G.dev.r_row = arena.upload(r_row, stream);
    G.dev.r_col = arena.upload(r_col, stream);
    {
      std::vector<int32_t> m4;
      build_r_m4(r_row, r_col, m4);
      G.dev.r_m4 = reinterpret_cast<const int4*>(arena.upload(m4, stream));
    }
    G.dev.nc = nagg_own;
    // Galerkin columns: global aggregate ids of every (owned or ghost) fine column
    const uint32_t* gal_agg = G.dev.agg;
    if (cur.dist) {
      uint32_t* gagg = arena.alloc<uint32_t>((size_t)sh + G.npad + G.ghi + 64);
      std::vector<uint32_t> ga(n);
      for (uint32_t i = 0; i < n; ++i) ga[i] = agg[i] + (uint32_t)cpart[rk];
      CFD_HIP(hipMemcpyAsync(gagg + sh, ga.data(), (size_t)n * sizeof(uint32_t), hipMemcpyHostToDevice, stream));
      halo(G.plan, {{reinterpret_cast<float*>(gagg + sh), 1}});  // bit copies
      gal_agg = gagg + sh;
    }
    // ---- Galerkin product on the device (this rank's aggregates)
    SetupLevel next;
    next.n = nagg_own;
    next.part = cpart;
    DevTmp<uint32_t> d_cnt(nagg_own);
    launch_galerkin(cur.dev, gal_agg, G.dev.r_row, G.dev.r_col, nagg_own, d_cnt.p, nullptr, nullptr, nullptr,
                    amg_setup_flag, stream);
    CFD_HIP(hipGetLastError());
    next.own_row.assign((size_t)nagg_own + 1, 0);
    uint32_t flag = 0;
    CFD_HIP(hipMemcpyAsync(next.own_row.data() + 1, d_cnt.p, (size_t)nagg_own * sizeof(uint32_t),
                           hipMemcpyDeviceToHost, stream));
    CFD_HIP(hipMemcpyAsync(&flag, amg_setup_flag, sizeof(uint32_t), hipMemcpyDeviceToHost, stream));
    sync();
    // every rank must take the same path: the overflow flag is combined over ranks
    bool overflow = flag != 0;
    if (dist()) {
      const std::vector<uint64_t> fl = gather_counts(flag);
      for (uint64_t f : fl) overflow = overflow || f != 0;
    }
    if (overflow) {
      if (timing) std::fprintf(stderr, "[amg setup] device path: capacity overflow at level %d\n", li);
      levels.clear();
      amg_refresh.clear();
      return false;
    }
    for (uint32_t I = 0; I < nagg_own; ++I) next.own_row[I + 1] += next.own_row[I];
    size_t nnz_c = next.own_row[nagg_own];
    next.d_rowptr = arena.alloc<uint32_t>((size_t)nagg_own + 1);
    next.d_col = arena.alloc<int32_t>(nnz_c);
    next.d_val = arena.alloc<float>(nnz_c);
    CFD_HIP(hipMemcpyAsync(next.d_rowptr, next.own_row.data(), ((size_t)nagg_own + 1) * sizeof(uint32_t),
                           hipMemcpyHostToDevice, stream));
    launch_galerkin(cur.dev, gal_agg, G.dev.r_row, G.dev.r_col, nagg_own, nullptr, next.d_rowptr,
                    reinterpret_cast<uint32_t*>(next.d_col), next.d_val, amg_setup_flag, stream);
    CFD_HIP(hipGetLastError());
    {
      AmgRefreshLevel& F = amg_refresh.back();
      F.has_coarse = true;
      F.gal_agg = gal_agg;
      F.nagg_own = nagg_own;
      F.rowptr_c = next.d_rowptr;
      F.col_c = reinterpret_cast<uint32_t*>(next.d_col);
      F.val_c = next.d_val;
      F.nnz_own = nnz_c;
    }
    next.dist = next_dist;
    if (cur.dist && !next_dist) {
      // first replicated level: all-gather row lengths, columns and values
      const std::vector<uint64_t> nnzs = gather_counts(nnz_c);
      std::vector<size_t> roff(R + 1), coff(R + 1);
      std::vector<uint64_t> eoff(R + 1, 0);
      for (int q = 0; q < R; ++q) eoff[q + 1] = eoff[q] + nnzs[q];
      for (int q = 0; q <= R; ++q) {
        roff[q] = cpart[q] * sizeof(uint32_t);
        coff[q] = eoff[q] * sizeof(uint32_t);
      }
      const uint64_t ng = cpart[R], nnz_all = eoff[R];
      std::vector<uint32_t> lens(ng, 0);
      for (uint32_t I = 0; I < nagg_own; ++I) lens[cpart[rk] + I] = next.own_row[I + 1] - next.own_row[I];
      DevTmp<uint32_t> d_lens(ng);
      int32_t* d_colall = arena.alloc<int32_t>(nnz_all);
      float* d_valall = arena.alloc<float>(nnz_all);
      CFD_HIP(hipMemcpyAsync(d_lens.p, lens.data(), ng * sizeof(uint32_t), hipMemcpyHostToDevice, stream));
      CFD_HIP(hipMemcpyAsync(d_colall + eoff[rk], next.d_col, nnz_c * sizeof(int32_t), hipMemcpyDeviceToDevice,
                             stream));
      CFD_HIP(hipMemcpyAsync(d_valall + eoff[rk], next.d_val, nnz_c * sizeof(float), hipMemcpyDeviceToDevice,
                             stream));
      comm->allgatherv_inplace(d_lens.p, roff, stream);
      comm->allgatherv_inplace(d_colall, coff, stream);
      comm->allgatherv_inplace(d_valall, coff, stream);
      AmgRefreshLevel& F = amg_refresh.back();
      F.val_all = d_valall;
      F.coff = coff;
      F.e_own = eoff[rk];
      CFD_HIP(hipMemcpyAsync(lens.data(), d_lens.p, ng * sizeof(uint32_t), hipMemcpyDeviceToHost, stream));
      sync();
      next.own_row.assign(ng + 1, 0);
      for (uint64_t I = 0; I < ng; ++I) next.own_row[I + 1] = next.own_row[I] + lens[I];
      next.n = (uint32_t)ng;
      nnz_c = nnz_all;
      next.d_rowptr = arena.alloc<uint32_t>(ng + 1);
      CFD_HIP(hipMemcpyAsync(next.d_rowptr, next.own_row.data(), (ng + 1) * sizeof(uint32_t),
                             hipMemcpyHostToDevice, stream));
      next.d_col = d_colall;
      next.d_val = d_valall;
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
      std::fprintf(stderr, "[amg setup] device level %d%s: n=%u nagg=%llu nnz_c=%zu  aggregate+R %.3fs  total %.3fs\n",
                   li, cur.dist ? " (dist)" : "", n, (unsigned long long)nagg_glob, nnz_c, t_agg, secs(t0));
    cur = std::move(next);
  }
  if (amg_g < 0) amg_g = dist() ? (int)levels.size() : 0;
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
    if (F.val_all) {  // first replicated level: every rank's coarse values (collective)
      if (F.nnz_own)
        CFD_HIP(hipMemcpyAsync(F.val_all + F.e_own, F.val_c, F.nnz_own * sizeof(float), hipMemcpyDeviceToDevice,
                               stream));
      comm->allgatherv_inplace(F.val_all, F.coff, stream);
    }
  }
  CFD_HIP(hipGetLastError());
  if (tail_blob_first >= 0) build_tail_blob(tail_blob_first, true);
  sync();
}

}  // namespace cfd2
