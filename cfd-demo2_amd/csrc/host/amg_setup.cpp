// Host AMG setup: restatement of src/solver/gpu/linear_solver/amg.rs.
//   aggregate            amg.rs:84-116   greedy, index order, no strength test
//   build_prolongation   amg.rs:118-139  piecewise-constant P (one 1.0 per fine row)
//   transpose            amg.rs:141-185  R = P^T, fine indices ascending per row
//   galerkin_product     amg.rs:187-235  (R*A)*P, f32 accumulation in visit order
//   level loop           amg.rs:374-595  stop at n <= 100, no reduction, or 20 levels
// Distributed solver: the aggregation runs part by part (rank ranges of the
// level's rows) and never lets an aggregate cross a part; with
// one part this is exactly the reference's greedy index-order aggregation.
// The hierarchy is built once (first AMG solve) and frozen.
// P and R hold only 1.0 values, so they are stored as index arrays.
#include <algorithm>
#include <limits>

#include "solver_impl.hpp"

namespace cfd2 {

namespace {

// C = A * B for general CSR, per-row dense accumulator visited in the same
// order as the reference's HashMap accumulation, then columns sorted.
HostCsr spgemm(const HostCsr& a, const HostCsr& b) {
  HostCsr c;
  c.rows = a.rows;
  c.cols = b.cols;
  c.row.assign(a.rows + 1, 0);
  std::vector<float> acc(b.cols, 0.0f);
  std::vector<uint8_t> seen(b.cols, 0);
  std::vector<uint32_t> touched;
  for (size_t i = 0; i < a.rows; ++i) {
    c.row[i] = (uint32_t)c.col.size();
    touched.clear();
    for (uint32_t ka = a.row[i]; ka < a.row[i + 1]; ++ka) {
      const uint32_t j = a.col[ka];
      const float va = a.val[ka];
      for (uint32_t kb = b.row[j]; kb < b.row[j + 1]; ++kb) {
        const uint32_t k = b.col[kb];
        if (!seen[k]) {
          seen[k] = 1;
          acc[k] = 0.0f;
          touched.push_back(k);
        }
        acc[k] += va * b.val[kb];
      }
    }
    std::sort(touched.begin(), touched.end());
    for (uint32_t k : touched) {
      c.col.push_back(k);
      c.val.push_back(acc[k]);
      seen[k] = 0;
    }
  }
  c.row[a.rows] = (uint32_t)c.col.size();
  return c;
}

}  // namespace

std::vector<AmgHostLevel> build_amg_hierarchy(const HostCsr& fine, size_t max_levels,
                                               const std::vector<uint64_t>& part0) {
  std::vector<AmgHostLevel> levels;
  HostCsr cur = fine;
  // row partition of the current level (distributed solver): aggregates never
  // cross a part, so coarse rows stay contiguous per rank (seed order = rank order)
  std::vector<uint64_t> part = part0.empty() ? std::vector<uint64_t>{0, (uint64_t)fine.rows} : part0;
  for (size_t li = 0; li < max_levels; ++li) {
    AmgHostLevel L;
    L.part = part;
    const size_t n = cur.rows;
    bool coarsened = false;
    if (li < max_levels - 1 && n > 100) {
      const uint32_t NONE = std::numeric_limits<uint32_t>::max();
      std::vector<uint32_t> agg(n, NONE);
      std::vector<uint64_t> cpart(part.size(), 0);
      uint32_t nagg = 0;
      for (size_t p = 0; p + 1 < part.size(); ++p) {
        cpart[p] = nagg;
        const uint64_t lo = part[p], hi = part[p + 1];
        for (size_t i = lo; i < hi; ++i) {
          if (agg[i] != NONE) continue;
          agg[i] = nagg;
          for (uint32_t k = cur.row[i]; k < cur.row[i + 1]; ++k) {
            const uint32_t j = cur.col[k];
            if (j != i && j >= lo && j < hi && agg[j] == NONE) agg[j] = nagg;
          }
          ++nagg;
        }
      }
      cpart.back() = nagg;
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
        R.row.assign(nagg + 1, 0);
        for (size_t i = 0; i < n; ++i) R.row[agg[i] + 1]++;
        for (uint32_t I = 0; I < nagg; ++I) R.row[I + 1] += R.row[I];
        R.col.resize(n);
        R.val.assign(n, 1.0f);
        {
          std::vector<uint32_t> pos(R.row.begin(), R.row.end() - 1);
          for (size_t i = 0; i < n; ++i) R.col[pos[agg[i]]++] = (uint32_t)i;  // ascending i
        }
        HostCsr next = spgemm(spgemm(R, cur), P);
        L.agg = std::move(agg);
        L.r_row = R.row;
        L.r_col = R.col;
        L.nc = nagg;
        L.has_op = true;
        L.A = std::move(cur);
        cur = std::move(next);
        part = std::move(cpart);
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
