#include "dist.hpp"

#include <algorithm>
#include <cstdlib>
#include <stdexcept>
#include <string>

#include "../hip/kernels.hpp"

namespace cfd2 {

// Rank r owns the segments [floor(nseg r / R), floor(nseg (r+1) / R)) of the
// canonical reduction tree (kernels.hpp red_geom): whole segments, so every
// reduction gives the same bits on any rank count.
std::vector<uint64_t> partition_starts(uint64_t n, int R) {
  if (R < 1) throw std::invalid_argument("nranks must be >= 1");
  if ((uint64_t)R > n) throw std::invalid_argument("more ranks than cells");
  const RedGeom g = red_geom(n);
  if ((uint64_t)R > g.nseg)
    throw std::invalid_argument("more ranks than reduction segments (" + std::to_string(g.nseg) + " of " +
                                std::to_string(g.seg_cells) + " cells)");
  std::vector<uint64_t> s(R + 1);
  for (int r = 0; r <= R; ++r) s[r] = std::min<uint64_t>(n, g.seg_cells * ((uint64_t)g.nseg * (uint64_t)r / (uint64_t)R));
  s[R] = n;
  return s;
}

int owner_of(const std::vector<uint64_t>& starts, uint64_t g) {
  return (int)(std::upper_bound(starts.begin(), starts.end(), g) - starts.begin()) - 1;
}

uint32_t collect_ghosts(uint64_t c0, uint64_t c1, const uint32_t* row, uint32_t n, const uint32_t* col,
                        std::vector<uint32_t>& ghost) {
  ghost.clear();
  for (uint64_t k = row[0]; k < row[n]; ++k)
    if (col[k] < c0 || col[k] >= c1) ghost.push_back(col[k]);
  std::sort(ghost.begin(), ghost.end());
  ghost.erase(std::unique(ghost.begin(), ghost.end()), ghost.end());
  return (uint32_t)(std::lower_bound(ghost.begin(), ghost.end(), (uint32_t)c0) - ghost.begin());
}

void interior_rows(const std::vector<uint64_t>& starts, int rank, const uint32_t* row, uint32_t n,
                   const uint32_t* col, uint32_t& lo_end, uint32_t& hi_begin) {
  const uint64_t c0 = starts[rank];
  int64_t last_lo = -1, first_hi = n;
  for (uint32_t li = 0; li < n; ++li) {
    if (row[li + 1] == row[li]) continue;
    if (col[row[li]] < c0) last_lo = li;
    if (col[row[li + 1] - 1] >= starts[rank + 1] && first_hi == (int64_t)n) first_hi = li;
  }
  lo_end = (uint32_t)((last_lo + 1 + 3) & ~(int64_t)3);
  hi_begin = (uint32_t)(first_hi & ~(int64_t)3);
  if (lo_end > n) lo_end = n;
  if (hi_begin < lo_end) hi_begin = lo_end;
}

HaloPlan build_halo_plan_lists(const std::vector<uint64_t>& starts, int rank,
                               const std::vector<std::vector<uint32_t>>& ghosts, uint32_t glo, uint32_t npad) {
  const int R = (int)starts.size() - 1;
  const uint64_t c0 = starts[rank], c1 = starts[rank + 1];
  const std::vector<uint32_t>& mine = ghosts[rank];
  HaloPlan P;
  for (int q = 0; q < R; ++q) {
    if (q == rank) continue;
    const auto lo = std::lower_bound(mine.begin(), mine.end(), (uint32_t)starts[q]);
    const auto hi = std::lower_bound(mine.begin(), mine.end(), (uint32_t)starts[q + 1]);
    const auto& theirs = ghosts[q];
    const auto slo = std::lower_bound(theirs.begin(), theirs.end(), (uint32_t)c0);
    const auto shi = std::lower_bound(theirs.begin(), theirs.end(), (uint32_t)c1);
    const uint32_t rc = (uint32_t)(hi - lo), sc = (uint32_t)(shi - slo);
    if (rc == 0 && sc == 0) continue;
    HaloPeer h;
    h.rank = q;
    const uint32_t k0 = (uint32_t)(lo - mine.begin());
    h.recv_rel = k0 < glo ? (int32_t)k0 - (int32_t)glo : (int32_t)(npad + (k0 - glo));
    h.recv_cnt = rc;
    h.send_off = (uint32_t)P.send_idx.size();
    h.send_cnt = sc;
    bool run = true;
    for (auto it = slo; it != shi; ++it) {
      const int32_t li = (int32_t)(*it - c0);
      if (it != slo && li != P.send_idx.back() + 1) run = false;
      P.send_idx.push_back(li);
    }
    h.direct = sc == 0 ? 0 : (run ? P.send_idx[h.send_off] : -1);
    P.peers.push_back(h);
  }
  P.all_direct = true;
  for (const HaloPeer& h : P.peers) P.all_direct = P.all_direct && h.direct >= 0;
  return P;
}

HaloPlan build_halo_plan(const std::vector<uint64_t>& starts, int rank, const uint32_t* row, uint32_t n,
                         const uint32_t* col, const std::vector<uint32_t>& ghost, uint32_t glo, uint32_t npad) {
  const int R = (int)starts.size() - 1;
  const uint64_t c0 = starts[rank];
  std::vector<std::vector<int32_t>> send(R);
  for (uint32_t li = 0; li < n; ++li) {
    int last = -1;
    for (uint64_t k = row[li]; k < row[li + 1]; ++k) {
      const uint32_t g = col[k];
      if (g >= c0 && g < starts[rank + 1]) continue;
      const int q = owner_of(starts, g);
      if (q == last) continue;  // columns ascend: same-peer runs are contiguous
      auto& v = send[q];
      if (v.empty() || v.back() != (int32_t)li) v.push_back((int32_t)li);
      last = q;
    }
  }
  HaloPlan P;
  {  // boundary row ranges (columns ascend: a row's first / last column decide)
    int64_t last_lo = -1, first_hi = n;
    for (uint32_t li = 0; li < n; ++li) {
      if (row[li + 1] == row[li]) continue;
      if (col[row[li]] < c0) last_lo = li;
      if (col[row[li + 1] - 1] >= starts[rank + 1] && first_hi == (int64_t)n) first_hi = li;
    }
    P.lo_end = (uint32_t)((last_lo + 1 + 3) & ~(int64_t)3);
    P.hi_begin = (uint32_t)(first_hi & ~(int64_t)3);
    if (P.lo_end > n) P.lo_end = n;
    if (P.hi_begin < P.lo_end) P.hi_begin = P.lo_end;
  }
  for (int q = 0; q < R; ++q) {
    if (q == rank) continue;
    const auto lo = std::lower_bound(ghost.begin(), ghost.end(), (uint32_t)starts[q]);
    const auto hi = std::lower_bound(ghost.begin(), ghost.end(), (uint32_t)starts[q + 1]);
    const uint32_t rc = (uint32_t)(hi - lo);
    if (rc == 0 && send[q].empty()) continue;
    HaloPeer h;
    h.rank = q;
    const uint32_t k0 = (uint32_t)(lo - ghost.begin());
    h.recv_rel = k0 < glo ? (int32_t)k0 - (int32_t)glo : (int32_t)(npad + (k0 - glo));
    h.recv_cnt = rc;
    h.send_off = (uint32_t)P.send_idx.size();
    h.send_cnt = (uint32_t)send[q].size();
    const auto& v = send[q];
    bool run = true;
    for (size_t t = 1; t < v.size() && run; ++t) run = v[t] == v[0] + (int32_t)t;
    h.direct = v.empty() ? 0 : (run ? v[0] : -1);
    P.send_idx.insert(P.send_idx.end(), send[q].begin(), send[q].end());
    P.peers.push_back(h);
  }
  P.all_direct = true;
  for (const HaloPeer& h : P.peers) P.all_direct = P.all_direct && h.direct >= 0;
  return P;
}

}  // namespace cfd2
