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
// need the wide-row layout, the host path runs instead.
//
// Distributed (build_amg_device_dist): the hierarchy is still the GLOBAL one
// (the one a single GPU builds, so the bits do not depend on the rank count),
// but every rank only touches its own rows:
//   - the greedy index-order aggregation runs as a pipeline over the ranks:
//     rank s aggregates its rows once ranks < s have announced which of its
//     rows (and of its upper ghosts) their aggregates took; all rows below a
//     seed are taken, so that is all the sequential pass needs (an aggregate
//     belongs to its seed's rank and may reach into higher ranks);
//   - the aggregate ids of the ghost columns come by one halo exchange;
//   - the fine rows of an aggregate that straddles ranks are imported from
//     their owners with every entry's global column and aggregate id (member
//     rows, SetupMatrix mode 2): structure once, values by one exchange;
//   - k_galerkin / k_amg_pack run on each rank for its own coarse rows;
//   - the first level with at most CFD_AMG_REPLICATE_ROWS rows is all-gathered
//     and the replicated levels below it are built exactly as on one GPU.
// The numeric re-setup (amg_rebuild_interval) re-runs the same value path over
// the kept structure: packs, value gathers, the member-value exchange, the
// Galerkin fills and the gather of the replicated level.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <unordered_map>

#include "../hip/amg_setup.hpp"
#include "solver_impl.hpp"

namespace cfd2 {

namespace {

constexpr uint32_t kNone = 0xFFFFFFFFu;

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

}  // namespace

// a level as the setup sees it: pattern on the host, values on the device
struct AmgSetupLevel {
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

bool Solver::build_amg_device() {
  if (dist()) return build_amg_device_dist();
  levels.clear();
  amg_refresh.clear();
  amg_g = 0;
  amg_setup_flag = arena.alloc<uint32_t>(1);
  CFD_HIP(hipMemsetAsync(amg_setup_flag, 0, sizeof(uint32_t), stream));
  AmgSetupLevel cur;
  cur.n = N;
  cur.row = topo.srow.data();
  cur.col = topo.scol.data();
  cur.dev.ell = 1;
  cur.dev.ld = topo.ld;
  cur.dev.len = d_slen;
  cur.dev.col = d_scol;  // global ids on one GPU
  cur.dev.val = sval;
  return device_levels(cur, 0, {0, (uint64_t)N});
}

// Per level from li0 on (one GPU: every level; distributed: the replicated
// levels, whose first level carries the coarse row partition part0): packing
// of the level on the device, aggregation + R on the host, Galerkin count /
// fill on the device, download of the coarse pattern.  Every rank of a
// distributed run computes the same replicated levels, so a false return
// (capacity overflow, wide rows) is the same on every rank.
bool Solver::device_levels(AmgSetupLevel& cur_in, int li0, const std::vector<uint64_t>& part0) {
  const bool timing = cfg.log_level >= 2 && rk == 0;
  using clk = std::chrono::steady_clock;
  auto secs = [](clk::time_point a) { return std::chrono::duration<double>(clk::now() - a).count(); };
  auto zeroed = [&](size_t cnt) {
    float* p = arena.alloc<float>(cnt + 64);
    CFD_HIP(hipMemsetAsync(p, 0, (cnt + 64) * sizeof(float), stream));
    return p;
  };
  AmgSetupLevel cur = std::move(cur_in);  // (a moved vector keeps its buffer: row / col stay valid)
  for (int li = li0; li < kMaxAmgLevels; ++li) {
    const auto t0 = clk::now();
    const uint32_t n = cur.n;
    levels.emplace_back();
    AmgGpuLevel& G = levels.back();
    G.nglob = n;
    if (li == li0) {
      G.part = part0;
      G.C0 = part0[rk];
      G.C1 = part0[rk + 1];
    } else {
      G.part = {0, (uint64_t)n};
      G.C0 = 0;
      G.C1 = n;
    }
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
    G.dev.agg = arena.upload(aggp, stream, kAggSlack);
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
    AmgSetupLevel next;
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
      F.r_row = G.dev.r_row;
      F.r_col = G.dev.r_col;
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

// Every rank's u32 vector (collective; sizes may differ, may be empty).
std::vector<std::vector<uint32_t>> Solver::allgatherv_u32(const std::vector<uint32_t>& mine) {
  const std::vector<uint64_t> sz = allgather_u64(mine.size());
  std::vector<size_t> off(R + 1, 0);
  for (int q = 0; q < R; ++q) off[q + 1] = off[q] + sz[q] * sizeof(uint32_t);
  std::vector<std::vector<uint32_t>> all(R);
  if (off[R] == 0) return all;
  DevTmp<uint32_t> buf(off[R] / 4);
  if (!mine.empty())
    CFD_HIP(hipMemcpyAsync(buf.p + off[rk] / 4, mine.data(), mine.size() * 4, hipMemcpyHostToDevice, stream));
  comm->allgatherv_inplace(buf.p, off, stream);
  std::vector<uint32_t> h(off[R] / 4);
  CFD_HIP(hipMemcpyAsync(h.data(), buf.p, off[R], hipMemcpyDeviceToHost, stream));
  sync();
  for (int q = 0; q < R; ++q) all[q].assign(h.begin() + off[q] / 4, h.begin() + off[q + 1] / 4);
  return all;
}

// Distributed device setup (see the file comment).  Returns false on every
// rank together (collective decisions) when the host path must build the
// hierarchy: a Galerkin capacity overflow or rows wider than the u8 layout.
bool Solver::build_amg_device_dist() {
  comm->label = -1;  // setup collectives (watchdog reports)
  const bool timing = cfg.log_level >= 2 && rk == 0;
  using clk = std::chrono::steady_clock;
  auto secs = [](clk::time_point a) { return std::chrono::duration<double>(clk::now() - a).count(); };
  const uint64_t rep = amg_replicate_rows();
  levels.clear();
  amg_refresh.clear();
  amg_g = 0;
  amg_setup_flag = arena.alloc<uint32_t>(1);
  CFD_HIP(hipMemsetAsync(amg_setup_flag, 0, sizeof(uint32_t), stream));
  auto zeroed = [&](size_t cnt) {
    float* p = arena.alloc<float>(cnt + 64);
    CFD_HIP(hipMemsetAsync(p, 0, (cnt + 64) * sizeof(float), stream));
    return p;
  };
  auto any_rank = [&](bool mine) {
    for (uint64_t f : allgather_u64(mine ? 1 : 0))
      if (f) return true;
    return false;
  };

  // the current (row-partitioned) level: own rows' pattern with global
  // columns on the host, values on the device (level 0: the ELL scalar matrix)
  struct DLevel {
    std::vector<uint64_t> part;
    uint64_t C0 = 0, C1 = 0, nglob = 0;
    const uint32_t* row = nullptr;
    const uint32_t* col = nullptr;
    std::vector<uint32_t> own_row, own_col;
    std::vector<uint32_t> ghost;  // ascending global ids
    uint32_t glo = 0;
    bool ell = false;
    const float* val = nullptr;           // device values
    const uint32_t* d_rowptr = nullptr;   // device CSR row pointers (coarse)
  } cur;
  cur.part = starts;
  cur.C0 = starts[rk];
  cur.C1 = starts[rk + 1];
  cur.nglob = NG;
  cur.row = topo.srow.data();
  cur.col = topo.scol.data();
  cur.ghost = topo.ghost;
  cur.glo = topo.glo;
  cur.ell = true;
  cur.val = sval;

  for (int li = 0; li < kMaxAmgLevels; ++li) {
    const auto t0 = clk::now();
    const uint64_t C0 = cur.C0, C1 = cur.C1;
    const uint32_t n = (uint32_t)(C1 - C0);
    const std::vector<uint32_t>& gh = cur.ghost;
    levels.emplace_back();
    AmgGpuLevel& G = levels.back();
    G.dist = true;
    G.nglob = cur.nglob;
    G.part = cur.part;
    G.C0 = C0;
    G.C1 = C1;
    G.glo = cur.glo;
    G.ghi = (uint32_t)gh.size() - cur.glo;
    G.npad = (n + 63) & ~63u;
    if (li == 0 && (G.glo != topo.glo || G.ghi != topo.ghi || G.npad != topo.npad))
      throw std::logic_error("AMG level 0 ghosts differ from the cell ghosts");
    auto rel = [&](uint32_t c) -> int32_t {  // signed local index of an owned row or ghost of this level
      if (c >= C0 && c < C1) return (int32_t)(c - C0);
      const auto it = std::lower_bound(gh.begin(), gh.end(), c);
      if (it == gh.end() || *it != c) throw std::logic_error("AMG: row is neither owned nor a ghost");
      const uint32_t k = (uint32_t)(it - gh.begin());
      return k < G.glo ? (int32_t)k - (int32_t)G.glo : (int32_t)(G.npad + (k - G.glo));
    };
    // ---- halo plan of the level (every rank's ghost list)
    {
      const auto ghosts_all = allgatherv_u32(gh);
      G.plan = build_halo_plan_lists(cur.part, rk, ghosts_all, G.glo, G.npad);
      interior_rows(cur.part, rk, cur.row, n, cur.col, G.plan.lo_end, G.plan.hi_begin);
      make_plan_buffers(G.plan, 1);
    }
    // ---- level image from the local-column view of the level
    const uint32_t* row = cur.row;
    const uint32_t* col = cur.col;
    int wmax = 0;
    bool small_delta = true;
    std::vector<int32_t> lcol;
    if (!cur.ell) lcol.resize(row[n] - row[0]);
    for (uint32_t i = 0; i < n; ++i) {
      int off = 0;
      for (uint32_t k = row[i]; k < row[i + 1]; ++k) {
        const int32_t c = cur.ell ? 0 : rel(col[k]);
        if (!cur.ell) lcol[k - row[0]] = c;
        if (col[k] == C0 + i) continue;
        ++off;
        const int64_t d = (int64_t)(cur.ell ? rel(col[k]) : c) - (int64_t)i;
        if (d < -32768 || d > 32767) small_delta = false;
      }
      wmax = std::max(wmax, off);
    }
    if (any_rank(wmax > amg_wide_limit)) {  // the host path handles (or rejects) wide rows
      if (timing) std::fprintf(stderr, "[amg setup] device path: wide rows at level %d, host path\n", li);
      return false;
    }
    SetupMatrix src{};
    if (cur.ell) {
      src.ell = 1;
      src.ld = topo.ld;
      src.len = d_slen;
      src.col = d_scol;  // signed local columns
      src.val = cur.val;
    } else {
      src.ell = 0;
      src.rowptr = cur.d_rowptr;
      src.col = arena.upload(lcol, stream);
      src.val = cur.val;
    }
    {
      const uint32_t st = G.npad;
      const size_t slots = (size_t)std::max(wmax, 1) * st;
      G.nnz = row[n] - row[0];
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
      launch_amg_pack(src, n, st, wmax, G.dev.use16, val, col16, col32, len, drank, dv, de, stream);
      CFD_HIP(hipGetLastError());
      G.dev.val = val;
      G.dev.col16 = col16;
      G.dev.col32 = col32;
      G.dev.len = len;
      G.dev.drank = drank;
      G.dev.dv = dv;
      G.dev.de = de;
    }
    if (li == 0) {
      G.xt = valloc<float>(1);
      G.r = valloc<float>(1);
    } else {
      const uint32_t sh = (G.glo + 63) & ~63u;
      const size_t cnt = (size_t)sh + G.npad + G.ghi;
      G.x = zeroed(cnt) + sh;
      G.xt = zeroed(cnt) + sh;
      G.b = zeroed(cnt) + sh;
      G.r = zeroed(cnt) + sh;
    }
    set_amg_full_policy(G, li);
    amg_refresh.emplace_back();
    amg_refresh.back().fine = src;
    amg_refresh.back().dist = true;

    // ---- coarsening (amg.rs:374-595)
    if (!(li < kMaxAmgLevels - 1 && cur.nglob > 100)) break;
    // greedy index-order aggregation as a pipeline over the ranks
    std::vector<uint32_t> agg(n, kNone);
    std::unordered_map<uint32_t, uint32_t> upmark;  // upper ghost rows already taken -> aggregate
    std::vector<std::vector<uint32_t>> exp_rows(R);  // own rows (local) that rank s < rk aggregates
    std::vector<uint32_t> imp;                       // upper rows this rank's aggregates took (global)
    std::vector<uint64_t> cpart(R + 1, 0);
    if (amg_local) {
      // partition-aware mode: the greedy pass over the own rows only (a seed
      // takes no ghost row), local ids first, then every rank's count gives
      // the global ids (seed order = rank order, as amg_setup.cpp)
      uint32_t cnt = 0;
      for (uint32_t i = 0; i < n; ++i) {
        if (agg[i] != kNone) continue;
        agg[i] = cnt;
        for (uint32_t k = row[i]; k < row[i + 1]; ++k) {
          const uint32_t c = col[k];
          if (c >= C0 && c < C1 && agg[c - C0] == kNone) agg[c - C0] = cnt;
        }
        ++cnt;
      }
      const std::vector<uint64_t> counts = allgather_u64(cnt);
      for (int q = 0; q < R; ++q) cpart[q + 1] = cpart[q] + counts[q];
      for (uint32_t& a : agg) a += (uint32_t)cpart[rk];
    }
    for (int s = 0; s < R && !amg_local; ++s) {
      std::vector<uint32_t> msg;
      if (s == rk) {
        const uint32_t base = (uint32_t)cpart[s];
        uint32_t cnt = 0;
        msg.push_back(0);
        for (uint32_t i = 0; i < n; ++i) {
          if (agg[i] != kNone) continue;
          const uint32_t id = base + cnt++;
          agg[i] = id;
          for (uint32_t k = row[i]; k < row[i + 1]; ++k) {
            const uint32_t c = col[k];
            if (c >= C0 && c < C1) {
              if (agg[c - C0] == kNone) agg[c - C0] = id;
            } else if (c >= C1) {  // rows below a seed are all taken already
              if (upmark.emplace(c, id).second) {
                msg.push_back(c);
                msg.push_back(id);
                imp.push_back(c);
              }
            }
          }
        }
        msg[0] = cnt;
      }
      const auto all = allgatherv_u32(msg);
      const auto& m = all[s];
      if (m.empty()) throw std::logic_error("AMG setup: empty aggregation message");
      cpart[s + 1] = cpart[s] + m[0];
      if (s == rk) continue;
      for (size_t t = 1; t + 1 < m.size(); t += 2) {
        const uint32_t c = m[t], id = m[t + 1];
        if (c >= C0 && c < C1) {
          if (s > rk) throw std::logic_error("AMG setup: a higher rank aggregated a lower rank's row");
          agg[c - C0] = id;
          exp_rows[s].push_back((uint32_t)(c - C0));
        } else if (c >= C1) {
          upmark.emplace(c, id);
        }
      }
    }
    const uint64_t nagg_total = cpart[R];
    if (nagg_total >= cur.nglob) break;  // no reduction: this level is the coarsest
    const uint64_t I0 = cpart[rk], I1 = cpart[rk + 1];
    const uint32_t nown_c = (uint32_t)(I1 - I0);
    const bool next_dist = nagg_total > rep;

    // aggregates of the ghost columns: one halo of agg over the level's plan
    std::vector<uint32_t> gagg(gh.size(), kNone);
    {
      const uint32_t sh = (G.glo + 63) & ~63u;
      const size_t cnt = (size_t)sh + G.npad + G.ghi;
      DevTmp<float> tmp(cnt + 1);
      if (n) CFD_HIP(hipMemcpyAsync(tmp.p + sh, agg.data(), (size_t)n * 4, hipMemcpyHostToDevice, stream));
      halo(G.plan, {{tmp.p + sh, 1}});
      if (G.glo)
        CFD_HIP(hipMemcpyAsync(gagg.data(), tmp.p + sh - G.glo, (size_t)G.glo * 4, hipMemcpyDeviceToHost, stream));
      if (G.ghi)
        CFD_HIP(hipMemcpyAsync(gagg.data() + G.glo, tmp.p + sh + G.npad, (size_t)G.ghi * 4, hipMemcpyDeviceToHost,
                               stream));
      sync();
    }
    auto agg_of = [&](uint32_t c) -> uint32_t {
      if (c >= C0 && c < C1) return agg[c - C0];
      const auto it = std::lower_bound(gh.begin(), gh.end(), c);
      if (it == gh.end() || *it != c) throw std::logic_error("AMG setup: column is neither owned nor a ghost");
      return gagg[it - gh.begin()];
    };
    auto vsrc = [&](uint32_t i, uint32_t k) -> uint32_t {  // value index of entry k of own row i
      return cur.ell ? (k - row[i]) * topo.ld + i : k - row[0];
    };
    // ---- member rows: own rows, then the imported upper rows (ascending ids)
    std::sort(imp.begin(), imp.end());
    std::vector<uint32_t> mrow(1, 0), magg, msrc;
    std::vector<int32_t> mkey;
    mkey.reserve(row[n] - row[0]);
    magg.reserve(row[n] - row[0]);
    msrc.reserve(row[n] - row[0]);
    for (uint32_t i = 0; i < n; ++i) {
      for (uint32_t k = row[i]; k < row[i + 1]; ++k) {
        mkey.push_back((int32_t)col[k]);
        magg.push_back(agg_of(col[k]));
        msrc.push_back(vsrc(i, k));
      }
      mrow.push_back((uint32_t)mkey.size());
    }
    const uint32_t n_own_e = (uint32_t)mkey.size();
    // exports (rows of mine in lower ranks' aggregates) and imports, per peer
    std::vector<uint32_t> imp_cnt(R, 0);
    for (uint32_t c : imp) imp_cnt[owner_of(cur.part, c)]++;
    std::vector<uint32_t> esrc;          // value index of every exported entry, peer by peer
    std::vector<uint32_t> elen, eent;    // exported row lengths / (key, agg) pairs, peer by peer
    std::vector<size_t> eoff_r(R + 1, 0), eoff_e(R + 1, 0);  // per peer: rows, entries
    for (int s = 0; s < R; ++s) {
      auto& v = exp_rows[s];
      std::sort(v.begin(), v.end());
      for (uint32_t i : v) {
        elen.push_back(row[i + 1] - row[i]);
        for (uint32_t k = row[i]; k < row[i + 1]; ++k) {
          eent.push_back(col[k]);
          eent.push_back(agg_of(col[k]));
          esrc.push_back(vsrc(i, k));
        }
      }
      eoff_r[s + 1] = elen.size();
      eoff_e[s + 1] = esrc.size();
    }
    std::vector<size_t> ioff_r(R + 1, 0);
    for (int q = 0; q < R; ++q) ioff_r[q + 1] = ioff_r[q] + imp_cnt[q];
    // structure exchange: lengths, then (key, agg) pairs
    std::vector<uint32_t> ilen(imp.size());
    std::vector<size_t> ioff_e(R + 1, 0);
    {
      DevTmp<uint32_t> sb(elen.size() + 1), rb(imp.size() + 1);
      if (!elen.empty())
        CFD_HIP(hipMemcpyAsync(sb.p, elen.data(), elen.size() * 4, hipMemcpyHostToDevice, stream));
      std::vector<Msg> msgs;
      for (int q = 0; q < R; ++q) {
        if (q == rk) continue;
        const size_t sbytes = (eoff_r[q + 1] - eoff_r[q]) * 4, rbytes = (size_t)imp_cnt[q] * 4;
        if (sbytes || rbytes) msgs.push_back({q, sb.p + eoff_r[q], sbytes, rb.p + ioff_r[q], rbytes});
      }
      comm->exchange(msgs, stream);
      if (!imp.empty()) CFD_HIP(hipMemcpyAsync(ilen.data(), rb.p, imp.size() * 4, hipMemcpyDeviceToHost, stream));
      sync();
    }
    for (int q = 0; q < R; ++q) {
      size_t e = 0;
      for (size_t t = ioff_r[q]; t < ioff_r[q + 1]; ++t) e += ilen[t];
      ioff_e[q + 1] = ioff_e[q] + e;
    }
    std::vector<uint32_t> ient(2 * ioff_e[R]);
    {
      DevTmp<uint32_t> sb(eent.size() + 1), rb(ient.size() + 1);
      if (!eent.empty())
        CFD_HIP(hipMemcpyAsync(sb.p, eent.data(), eent.size() * 4, hipMemcpyHostToDevice, stream));
      std::vector<Msg> msgs;
      for (int q = 0; q < R; ++q) {
        if (q == rk) continue;
        const size_t sbytes = 2 * (eoff_e[q + 1] - eoff_e[q]) * 4, rbytes = 2 * (ioff_e[q + 1] - ioff_e[q]) * 4;
        if (sbytes || rbytes) msgs.push_back({q, sb.p + 2 * eoff_e[q], sbytes, rb.p + 2 * ioff_e[q], rbytes});
      }
      comm->exchange(msgs, stream);
      if (!ient.empty()) CFD_HIP(hipMemcpyAsync(ient.data(), rb.p, ient.size() * 4, hipMemcpyDeviceToHost, stream));
      sync();
    }
    for (size_t t = 0, e = 0; t < imp.size(); ++t) {
      for (uint32_t k = 0; k < ilen[t]; ++k, ++e) {
        mkey.push_back((int32_t)ient[2 * e]);
        magg.push_back(ient[2 * e + 1]);
      }
      mrow.push_back((uint32_t)mkey.size());
    }
    const uint32_t n_imp_e = (uint32_t)(mkey.size() - n_own_e);
    // R over member rows (own i -> i, imported t -> n + t), ascending global order
    std::vector<uint32_t> m_rrow(nown_c + 1, 0), m_rcol;
    std::vector<uint32_t> m_of;  // aggregate (local) of every member row in my aggregates, or kNone
    m_of.reserve(n + imp.size());
    for (uint32_t i = 0; i < n; ++i) m_of.push_back(agg[i] >= I0 && agg[i] < I1 ? agg[i] - (uint32_t)I0 : kNone);
    for (uint32_t c : imp) m_of.push_back(upmark.at(c) - (uint32_t)I0);
    for (uint32_t a : m_of)
      if (a != kNone) m_rrow[a + 1]++;
    for (uint32_t I = 0; I < nown_c; ++I) m_rrow[I + 1] += m_rrow[I];
    m_rcol.resize(m_rrow[nown_c]);
    {
      std::vector<uint32_t> pos(m_rrow.begin(), m_rrow.end() - 1);
      for (uint32_t t = 0; t < (uint32_t)m_of.size(); ++t)
        if (m_of[t] != kNone) m_rcol[pos[m_of[t]]++] = t;
    }
    // device member matrix; values: own entries gathered, imported ones exchanged
    AmgRefreshLevel& F = amg_refresh.back();
    F.has_coarse = true;
    F.src_val = cur.val;
    F.n_own_e = n_own_e;
    F.n_exp_e = (uint32_t)esrc.size();
    F.msrc = arena.upload(msrc, stream);
    F.esrc = arena.upload(esrc, stream);
    F.ebuf = arena.alloc<float>(esrc.size() + 1);
    float* mval = arena.alloc<float>((size_t)n_own_e + n_imp_e + 1);
    for (int q = 0; q < R; ++q) {
      if (q == rk) continue;
      const size_t sbytes = (eoff_e[q + 1] - eoff_e[q]) * 4, rbytes = (ioff_e[q + 1] - ioff_e[q]) * 4;
      if (sbytes || rbytes)
        F.val_msgs.push_back({q, F.ebuf + eoff_e[q], sbytes, mval + n_own_e + ioff_e[q], rbytes});
    }
    F.mem.ell = 2;
    F.mem.rowptr = arena.upload(mrow, stream);
    F.mem.col = arena.upload(mkey, stream);
    F.mem.eagg = arena.upload(magg, stream);
    F.mem.val = mval;
    F.r_row = arena.upload(m_rrow, stream);
    F.r_col = arena.upload(m_rcol, stream);
    F.nagg_own = nown_c;
    member_values(F);
    // Galerkin count pass
    std::vector<uint32_t> crow(nown_c + 1, 0);
    uint32_t flag = 0;
    {
      DevTmp<uint32_t> d_cnt(nown_c);
      launch_galerkin(F.mem, nullptr, F.r_row, F.r_col, nown_c, d_cnt.p, nullptr, nullptr, nullptr, amg_setup_flag,
                      stream);
      CFD_HIP(hipGetLastError());
      if (nown_c)
        CFD_HIP(hipMemcpyAsync(crow.data() + 1, d_cnt.p, (size_t)nown_c * 4, hipMemcpyDeviceToHost, stream));
      CFD_HIP(hipMemcpyAsync(&flag, amg_setup_flag, sizeof(uint32_t), hipMemcpyDeviceToHost, stream));
      sync();
    }
    if (any_rank(flag != 0)) {
      if (timing) std::fprintf(stderr, "[amg setup] device path: capacity overflow at level %d\n", li);
      return false;
    }
    for (uint32_t I = 0; I < nown_c; ++I) crow[I + 1] += crow[I];
    const size_t nnz_c = crow[nown_c];
    uint32_t* d_crow = arena.upload(crow, stream);
    // fill: into this rank's coarse rows, or straight into the all-gathered
    // arrays of the first replicated level
    std::vector<uint64_t> cnz;  // every rank's coarse nnz (replicated next level)
    std::vector<size_t> goff(R + 1, 0);
    int32_t* g_col = nullptr;
    float* g_val = nullptr;
    if (next_dist) {
      F.col_c = reinterpret_cast<uint32_t*>(arena.alloc<int32_t>(nnz_c + 1));
      F.val_c = arena.alloc<float>(nnz_c + 1);
    } else {
      cnz = allgather_u64(nnz_c);
      for (int q = 0; q < R; ++q) goff[q + 1] = goff[q] + cnz[q];
      g_col = arena.alloc<int32_t>(goff[R] + 1);
      g_val = arena.alloc<float>(goff[R] + 1);
      F.col_c = reinterpret_cast<uint32_t*>(g_col + goff[rk]);
      F.val_c = g_val + goff[rk];
    }
    F.rowptr_c = d_crow;
    F.nnz_own = nnz_c;
    launch_galerkin(F.mem, nullptr, F.r_row, F.r_col, nown_c, nullptr, d_crow, F.col_c, F.val_c, amg_setup_flag,
                    stream);
    CFD_HIP(hipGetLastError());
    std::vector<uint32_t> ccol(nnz_c);
    if (nnz_c)
      CFD_HIP(hipMemcpyAsync(ccol.data(), F.col_c, nnz_c * 4, hipMemcpyDeviceToHost, stream));
    sync();

    // ---- next level's ghosts (distributed next level)
    std::vector<uint32_t> ngh;
    uint32_t nglo = 0;
    const uint32_t nnpad = (nown_c + 63) & ~63u;
    if (next_dist) {
      for (uint32_t c : ccol)
        if (c < I0 || c >= I1) ngh.push_back(c);
      for (uint32_t a : agg)
        if (a < I0 || a >= I1) ngh.push_back(a);
      std::sort(ngh.begin(), ngh.end());
      ngh.erase(std::unique(ngh.begin(), ngh.end()), ngh.end());
      nglo = (uint32_t)(std::lower_bound(ngh.begin(), ngh.end(), (uint32_t)I0) - ngh.begin());
    }
    auto rel_next = [&](uint32_t c) -> int32_t {
      if (c >= I0 && c < I1) return (int32_t)(c - I0);
      const auto it = std::lower_bound(ngh.begin(), ngh.end(), c);
      if (it == ngh.end() || *it != c) throw std::logic_error("AMG: coarse row is neither owned nor a ghost");
      const uint32_t k = (uint32_t)(it - ngh.begin());
      return k < nglo ? (int32_t)k - (int32_t)nglo : (int32_t)(nnpad + (k - nglo));
    };
    // ---- P and R of this level in the V-cycle layout (as build_amg_host)
    {
      std::vector<uint32_t> aggp(G.dev.stride, 0), r_row(nown_c + 1), r_col(m_rcol.size());
      for (uint32_t i = 0; i < n; ++i) aggp[i] = next_dist ? (uint32_t)rel_next(agg[i]) : agg[i];
      for (uint32_t I = 0; I <= nown_c; ++I) r_row[I] = m_rrow[I];
      for (size_t k = 0; k < m_rcol.size(); ++k) {
        const uint32_t t = m_rcol[k];
        const int32_t lf = t < n ? (int32_t)t : rel(imp[t - n]);
        if (lf < 0) throw std::logic_error("AMG: aggregate member below its seed's rank");
        r_col[k] = (uint32_t)lf;
      }
      G.dev.nc = nown_c;
      const uint32_t nown = n;
      G.rc_hi = nown_c;
      for (uint32_t I = 0; I < nown_c; ++I) {
        bool ghost = false;
        for (uint32_t k = r_row[I]; k < r_row[I + 1]; ++k) ghost |= r_col[k] >= nown;
        if (ghost) {
          G.rc_hi = I;
          break;
        }
      }
      G.pf_lo = 0;
      if (next_dist) {
        for (uint32_t i = 0; i < nown; ++i)
          if ((int32_t)aggp[i] < 0 || aggp[i] >= nown_c) G.pf_lo = i + 1;
        G.pf_lo = std::min((G.pf_lo + 3) & ~3u, nown);
      }
      G.dev.agg = arena.upload(aggp, stream, kAggSlack);
      G.dev.r_row = arena.upload(r_row, stream);
      G.dev.r_col = arena.upload(r_col, stream);
      std::vector<int32_t> m4;
      build_r_m4(r_row, r_col, m4);
      G.dev.r_m4 = reinterpret_cast<const int4*>(arena.upload(m4, stream));
    }
    if (timing)
      std::fprintf(stderr,
                   "[amg setup] rank %d distributed level %d: n=%u (of %llu) nagg=%u (of %llu) imported rows %zu "
                   "nnz_c=%zu  %.3fs\n",
                   rk, li, n, (unsigned long long)cur.nglob, nown_c, (unsigned long long)nagg_total, imp.size(),
                   nnz_c, secs(t0));

    if (!next_dist) {
      // ---- first replicated level: all-gather the coarse rows, then one-GPU setup
      amg_g = li + 1;
      std::vector<size_t> boff(R + 1);
      for (int q = 0; q <= R; ++q) boff[q] = goff[q] * 4;
      comm->allgatherv_inplace(g_col, boff, stream);
      comm->allgatherv_inplace(g_val, boff, stream);
      F.rep_val = g_val;
      F.rep_off = boff;
      std::vector<uint32_t> lens(nown_c);
      for (uint32_t I = 0; I < nown_c; ++I) lens[I] = crow[I + 1] - crow[I];
      const auto all_lens = allgatherv_u32(lens);
      AmgSetupLevel rl;
      rl.n = (uint32_t)nagg_total;
      rl.own_row.assign((size_t)rl.n + 1, 0);
      {
        size_t I = 0;
        for (int q = 0; q < R; ++q)
          for (uint32_t l : all_lens[q]) {
            rl.own_row[I + 1] = rl.own_row[I] + l;
            ++I;
          }
        if (I != rl.n || rl.own_row[rl.n] != goff[R]) throw std::logic_error("AMG: replicated level gather");
      }
      rl.own_col.resize(goff[R]);
      if (goff[R])
        CFD_HIP(hipMemcpyAsync(rl.own_col.data(), g_col, goff[R] * 4, hipMemcpyDeviceToHost, stream));
      rl.d_rowptr = arena.upload(rl.own_row, stream);
      rl.d_col = g_col;
      rl.d_val = g_val;
      sync();
      rl.row = rl.own_row.data();
      rl.col = rl.own_col.data();
      rl.dev.ell = 0;
      rl.dev.rowptr = rl.d_rowptr;
      rl.dev.col = rl.d_col;
      rl.dev.val = rl.d_val;
      return device_levels(rl, li + 1, cpart);
    }
    // ---- next distributed level
    DLevel nx;
    nx.part = cpart;
    nx.C0 = I0;
    nx.C1 = I1;
    nx.nglob = nagg_total;
    nx.own_row = std::move(crow);
    nx.own_col = std::move(ccol);
    nx.ghost = std::move(ngh);
    nx.glo = nglo;
    nx.ell = false;
    nx.val = F.val_c;
    nx.d_rowptr = d_crow;
    cur = std::move(nx);
    cur.row = cur.own_row.data();
    cur.col = cur.own_col.data();
  }
  amg_g = (int)levels.size();
  sync();
  return true;
}

// member values of a distributed level: own entries gathered from the level's
// values, exported entries gathered and sent to the ranks that aggregate them
void Solver::member_values(const AmgRefreshLevel& F) {
  launch_gather_f32(F.src_val, F.msrc, F.n_own_e, const_cast<float*>(F.mem.val), stream);
  launch_gather_f32(F.src_val, F.esrc, F.n_exp_e, F.ebuf, stream);
  CFD_HIP(hipGetLastError());
  comm->exchange(F.val_msgs, stream);
}

// Numeric re-setup from the current matrix (cfg.amg_rebuild_interval): the
// structure built by build_amg_device is value-independent (aggregation and
// R on the pattern, Galerkin patterns structural -- explicit zeros are kept,
// as amg.rs keeps them), so packing every level and re-running the Galerkin
// fill over it in level order gives the bytes a full rebuild gives
// (tests/test_gpu_parity.py::test_amg_refresh_matches_full_rebuild).  A
// distributed level re-runs its member-value gathers and exchange first, and
// the last one re-gathers the replicated level's values.
void Solver::refresh_amg() {
  if (comm) comm->label = -1;
  const size_t slots_s = (size_t)topo.ws * topo.ld;
  CFD_HIP(hipMemcpyAsync(amg_src, sval, slots_s * sizeof(float), hipMemcpyDeviceToDevice, stream));
  for (size_t li = 0; li < amg_refresh.size(); ++li) {
    const AmgRefreshLevel& F = amg_refresh[li];
    const AmgLevelDev& d = levels[li].dev;
    launch_amg_pack(F.fine, d.n, d.stride, d.w, d.use16, const_cast<float*>(d.val), const_cast<int16_t*>(d.col16),
                    const_cast<int32_t*>(d.col32), const_cast<uint8_t*>(d.len), const_cast<uint8_t*>(d.drank),
                    const_cast<float*>(d.dv), const_cast<float*>(d.de), stream);
    if (!F.has_coarse) continue;
    if (F.dist) {
      member_values(F);
      launch_galerkin(F.mem, nullptr, F.r_row, F.r_col, F.nagg_own, nullptr, F.rowptr_c, F.col_c, F.val_c,
                      amg_setup_flag, stream);
      if (F.rep_val) comm->allgatherv_inplace(F.rep_val, F.rep_off, stream);
    } else {
      launch_galerkin(F.fine, F.gal_agg, F.r_row, F.r_col, F.nagg_own, nullptr, F.rowptr_c, F.col_c, F.val_c,
                      amg_setup_flag, stream);
    }
  }
  CFD_HIP(hipGetLastError());
  if (tail_blob_first >= 0) build_tail_blob(tail_blob_first, true);
  sync();
}

}  // namespace cfd2
