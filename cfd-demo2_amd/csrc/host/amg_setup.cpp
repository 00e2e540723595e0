// Host AMG setup: restatement of src/solver/gpu/linear_solver/amg.rs.
//   aggregate            amg.rs:84-116   greedy, index order, no strength test
//   build_prolongation   amg.rs:118-139  piecewise-constant P (one 1.0 per fine row)
//   transpose            amg.rs:141-185  R = P^T, fine indices ascending per row
//   galerkin_product     amg.rs:187-235  (R*A)*P, f32 accumulation in visit order
//   level loop           amg.rs:374-595  stop at n <= 100, no reduction, or 20 levels
// Distributed solver: the same global aggregation (so the hierarchy, and every
// result, does not depend on the rank count); a coarse row belongs to the rank
// that owns its seed, the aggregate's first (smallest) fine row, so coarse rows
// stay contiguous per rank and an aggregate may reach into the next ranks.
// The hierarchy is built once (first AMG solve) and frozen.
// P and R hold only 1.0 values, so they are stored as index arrays.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <limits>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "solver_impl.hpp"

namespace cfd2 {

namespace {

// C = A * B for general CSR.  Per row, products are accumulated per output
// column in visit order (the reference's HashMap accumulation: first touch
// starts at 0, then += a*b), then the row's columns are sorted.  Rows are
// independent, so they are built in parallel (OpenMP, contiguous row chunks
// concatenated in order) with a small per-row accumulator instead of a dense
// one: identical arithmetic, O(nnz) memory.
HostCsr spgemm(const HostCsr& a, const HostCsr& b) {
  HostCsr c;
  c.rows = a.rows;
  c.cols = b.cols;
  c.row.assign(a.rows + 1, 0);
  // visit-order accumulation of row i into acc (first touch = 0, then += a*b)
  auto row_product = [&](size_t i, std::vector<std::pair<uint32_t, float>>& acc) {
    acc.clear();
    for (uint32_t ka = a.row[i]; ka < a.row[i + 1]; ++ka) {
      const uint32_t j = a.col[ka];
      const float va = a.val[ka];
      for (uint32_t kb = b.row[j]; kb < b.row[j + 1]; ++kb) {
        const uint32_t k = b.col[kb];
        size_t q = 0;
        while (q < acc.size() && acc[q].first != k) ++q;
        if (q == acc.size()) acc.push_back({k, 0.0f});
        acc[q].second += va * b.val[kb];
      }
    }
  };
  // pass 1: row lengths (parallel, no allocation), pass 2: fill in place
#pragma omp parallel
  {
    std::vector<std::pair<uint32_t, float>> acc;
#pragma omp for schedule(static)
    for (long i = 0; i < (long)a.rows; ++i) {
      row_product(i, acc);
      c.row[i + 1] = (uint32_t)acc.size();
    }
  }
  for (size_t i = 0; i < a.rows; ++i) c.row[i + 1] += c.row[i];
  c.col.resize(c.row[a.rows]);
  c.val.resize(c.row[a.rows]);
#pragma omp parallel
  {
    std::vector<std::pair<uint32_t, float>> acc;
#pragma omp for schedule(static)
    for (long i = 0; i < (long)a.rows; ++i) {
      row_product(i, acc);
      std::sort(acc.begin(), acc.end(),
                [](const std::pair<uint32_t, float>& x, const std::pair<uint32_t, float>& y) {
                  return x.first < y.first;
                });
      uint32_t o = c.row[i];
      for (const auto& e : acc) {
        c.col[o] = e.first;
        c.val[o] = e.second;
        ++o;
      }
    }
  }
  return c;
}

}  // namespace

uint32_t aggregate_greedy(size_t n, const uint32_t* row, const uint32_t* col, const std::vector<uint64_t>& part,
                          std::vector<uint32_t>& agg, std::vector<uint64_t>& cpart, bool local) {
  const uint32_t NONE = std::numeric_limits<uint32_t>::max();
  agg.assign(n, NONE);
  cpart.assign(part.size(), 0);
  // greedy index-order pass (amg.rs:84-116): a row still free becomes a seed
  // and takes every free neighbour.  Rows before a seed are all taken, so the
  // seed is its aggregate's smallest row and aggregates are numbered in seed
  // order: cpart[q] = first aggregate seeded at or after part[q].
  // local (partition-aware mode, cfd_config.amg_local_aggregation): a seed
  // takes only free neighbours of its own part, so no aggregate straddles two
  // parts -- the same pass over the pattern without its cross-part entries.
  uint32_t nagg = 0;
  size_t q = 0;
  for (size_t i = 0; i < n; ++i) {
    while (q + 1 < part.size() && part[q] <= i) cpart[q++] = nagg;
    if (agg[i] != NONE) continue;
    agg[i] = nagg;
    // part of row i: [part[q - 1], part[q])
    const uint64_t lo = q > 0 ? part[q - 1] : 0, hi = q < part.size() ? part[q] : n;
    for (uint32_t k = row[i]; k < row[i + 1]; ++k) {
      const uint32_t j = col[k];
      if (local && (j < lo || j >= hi)) continue;
      if (agg[j] == NONE) agg[j] = nagg;
    }
    ++nagg;
  }
  while (q < part.size()) cpart[q++] = nagg;
  return nagg;
}

void transpose_aggregates(const std::vector<uint32_t>& agg, uint32_t nagg, std::vector<uint32_t>& r_row,
                          std::vector<uint32_t>& r_col) {
  const size_t n = agg.size();
  r_row.assign(nagg + 1, 0);
  for (size_t i = 0; i < n; ++i) r_row[agg[i] + 1]++;
  for (uint32_t I = 0; I < nagg; ++I) r_row[I + 1] += r_row[I];
  r_col.resize(n);
  std::vector<uint32_t> pos(r_row.begin(), r_row.end() - 1);
  for (size_t i = 0; i < n; ++i) r_col[pos[agg[i]]++] = (uint32_t)i;  // ascending i
}

std::vector<AmgHostLevel> build_amg_hierarchy(const HostCsr& fine, size_t max_levels,
                                               const std::vector<uint64_t>& part0, bool local, uint64_t rep_rows,
                                               bool timing) {
  std::vector<AmgHostLevel> levels;
  HostCsr cur = fine;
  // row partition of the current level (distributed solver): coarse rows
  // follow their seeds (seed order = rank order)
  std::vector<uint64_t> part = part0.empty() ? std::vector<uint64_t>{0, (uint64_t)fine.rows} : part0;
  // partition-aware mode: the row-partitioned levels (level 0 and every next
  // level of more than rep_rows rows) aggregate per part; from the first
  // replicated level on, the global pass
  bool local_level = local && part.size() > 2;
  for (size_t li = 0; li < max_levels; ++li) {
    AmgHostLevel L;
    L.part = part;
    const size_t n = cur.rows;
    bool coarsened = false;
    if (li < max_levels - 1 && n > 100) {
      std::vector<uint32_t> agg;
      std::vector<uint64_t> cpart;
      const uint32_t nagg = aggregate_greedy(n, cur.row.data(), cur.col.data(), part, agg, cpart, local_level);
      if (nagg < n) {
        // P (n x nagg) and R = P^T as CSR with unit values
        HostCsr P, R;
        P.rows = n;
        P.cols = nagg;
        P.row.resize(n + 1);
        P.col.resize(n);
        P.val.assign(n, 1.0f);
        for (size_t i = 0; i < n; ++i) {
          P.row[i] = (uint32_t)i;
          P.col[i] = agg[i];
        }
        P.row[n] = (uint32_t)n;
        R.rows = nagg;
        R.cols = n;
        transpose_aggregates(agg, nagg, R.row, R.col);
        R.val.assign(n, 1.0f);
        const auto t0 = std::chrono::steady_clock::now();
        HostCsr RA = spgemm(R, cur);
        const auto t1 = std::chrono::steady_clock::now();
        HostCsr next = spgemm(RA, P);
        const auto t2 = std::chrono::steady_clock::now();
        if (timing)
          std::fprintf(stderr, "[amg setup] level %zu: n=%zu nagg=%u  R*A %.3fs  (RA)*P %.3fs\n", li, n, nagg,
                       std::chrono::duration<double>(t1 - t0).count(), std::chrono::duration<double>(t2 - t1).count());
        L.agg = std::move(agg);
        L.r_row = R.row;
        L.r_col = R.col;
        L.nc = nagg;
        L.has_op = true;
        L.A = std::move(cur);
        cur = std::move(next);
        part = std::move(cpart);
        local_level = local_level && nagg > rep_rows;
        coarsened = true;
      }
    }
    if (!coarsened) L.A = cur;
    levels.push_back(std::move(L));
    if (!coarsened) break;
  }
  return levels;
}

}  // namespace cfd2

namespace cfd2 {

bool build_pair_partition(const std::vector<uint32_t>& fr_row, const std::vector<uint32_t>& fr_col,
                          const std::vector<uint32_t>& mr_row, const std::vector<uint32_t>& mr_col,
                          const std::vector<uint32_t>& mrow, const std::vector<uint32_t>& mcol, uint32_t cap,
                          PairPartition& out) {
  const uint32_t nm = (uint32_t)mrow.size() - 1, nc = (uint32_t)mr_row.size() - 1;
  if (fr_row.size() != (size_t)nm + 1 || mr_col.size() != nm) return false;
  auto nfine = [&](uint32_t g) { return fr_row[g + 1] - fr_row[g]; };
  out = PairPartition{};
  out.jb.push_back(0);
  // greedy: stamp[g] = block whose S holds row g
  std::vector<int32_t> stamp(nm, -1);
  std::vector<uint32_t> added;
  uint32_t nS = 0, nF = 0, nJ = 0;
  int32_t blk = 0;
  for (uint32_t J = 0; J < nc;) {
    added.clear();
    uint32_t dS = 0, dF = 0;
    auto take = [&](uint32_t g) {
      if (stamp[g] == blk) return;
      stamp[g] = blk;
      added.push_back(g);
      ++dS;
      dF += nfine(g);
    };
    for (uint32_t k = mr_row[J]; k < mr_row[J + 1]; ++k) {
      const uint32_t g = mr_col[k];
      take(g);
      for (uint32_t e = mrow[g]; e < mrow[g + 1]; ++e) take(mcol[e]);
    }
    if (nS + dS <= cap && nF + dF <= cap && nJ + 1 <= cap) {
      nS += dS;
      nF += dF;
      ++nJ;
      ++J;
      continue;
    }
    for (uint32_t g : added) stamp[g] = -1;  // J opens the next block
    if (nJ == 0) return false;               // one aggregate alone does not fit
    out.jb.push_back(J);
    ++blk;
    nS = nF = nJ = 0;
  }
  if (nJ) out.jb.push_back(nc);
  const uint32_t nb = (uint32_t)out.jb.size() - 1;
  out.sb.assign(1, 0);
  out.fo.assign(1, 0);
  out.s.clear();
  out.f.clear();
  out.lc.assign(mcol.size(), 0);
  std::vector<int32_t> loc(nm, -1);
  std::vector<uint32_t> ring;
  for (uint32_t k = 0; k < nb; ++k) {
    const size_t base = out.s.size();
    for (uint32_t q = mr_row[out.jb[k]]; q < mr_row[out.jb[k + 1]]; ++q) {
      loc[mr_col[q]] = (int32_t)(out.s.size() - base);
      out.s.push_back(mr_col[q]);
    }
    const size_t own_end = out.s.size();
    ring.clear();
    for (size_t q = base; q < own_end; ++q)
      for (uint32_t e = mrow[out.s[q]]; e < mrow[out.s[q] + 1]; ++e)
        if (loc[mcol[e]] == -1) {
          loc[mcol[e]] = -2;  // queued
          ring.push_back(mcol[e]);
        }
    std::sort(ring.begin(), ring.end());
    for (uint32_t c : ring) {
      loc[c] = (int32_t)(out.s.size() - base);
      out.s.push_back(c);
    }
    for (size_t q = base; q < own_end; ++q)
      for (uint32_t e = mrow[out.s[q]]; e < mrow[out.s[q] + 1]; ++e) out.lc[e] = (uint16_t)loc[mcol[e]];
    for (size_t q = base; q < out.s.size(); ++q) {
      for (uint32_t e = fr_row[out.s[q]]; e < fr_row[out.s[q] + 1]; ++e) out.f.push_back(fr_col[e]);
      out.fo.push_back((uint32_t)out.f.size());
    }
    for (size_t q = base; q < out.s.size(); ++q) loc[out.s[q]] = -1;
    if (out.s.size() - base > cap || out.fo.back() - out.fo[base] > cap)
      throw std::logic_error("AMG pair partition: block " + std::to_string(k) + " over capacity (S " +
                             std::to_string(out.s.size() - base) + ", f " +
                             std::to_string(out.fo.back() - out.fo[base]) + ", cap " + std::to_string(cap) + ")");
    out.sb.push_back((uint32_t)out.s.size());
  }
  return true;
}

bool build_up_pair_partition(const std::vector<uint32_t>& frow, const std::vector<uint32_t>& fcol,
                             const std::vector<uint32_t>& agg, uint32_t nc, uint32_t rows, uint32_t cap,
                             UpPairPartition& out) {
  const uint32_t nf = (uint32_t)frow.size() - 1;
  if (agg.size() < nf || rows == 0) return false;
  out = UpPairPartition{};
  out.tb.assign(1, 0);
  out.lt.assign(fcol.size(), 0);
  out.lto.assign(nf, 0);
  std::vector<int32_t> loc(nc, -1);
  std::vector<uint32_t> tl;
  for (uint32_t r0 = 0; r0 < nf; r0 += rows) {
    const uint32_t r1 = std::min(nf, r0 + rows);
    tl.clear();
    auto add = [&](uint32_t c) {
      if (c >= nc) throw std::logic_error("AMG up pair: aggregate out of range");
      if (loc[c] == -1) {
        loc[c] = -2;
        tl.push_back(c);
      }
    };
    for (uint32_t f = r0; f < r1; ++f) {
      add(agg[f]);
      for (uint32_t e = frow[f]; e < frow[f + 1]; ++e) add(agg[fcol[e]]);
    }
    std::sort(tl.begin(), tl.end());
    if (tl.size() > cap) return false;
    for (size_t q = 0; q < tl.size(); ++q) loc[tl[q]] = (int32_t)q;
    for (uint32_t f = r0; f < r1; ++f) {
      out.lto[f] = (uint16_t)loc[agg[f]];
      for (uint32_t e = frow[f]; e < frow[f + 1]; ++e) out.lt[e] = (uint16_t)loc[agg[fcol[e]]];
    }
    for (uint32_t c : tl) loc[c] = -1;
    out.t.insert(out.t.end(), tl.begin(), tl.end());
    out.tb.push_back((uint32_t)out.t.size());
  }
  return true;
}

}  // namespace cfd2
