// Slab partition and halo plans of the distributed solver.
//
// Rank r owns the contiguous global rows [start(r), start(r+1)), whole
// segments of the canonical reduction tree (partition_starts).  The cut-cell mesher numbers cells x-major, so these are
// vertical slabs and a rank's ghosts come from its slab neighbours.  A rank
// stores ghosts of lower ranks at local indices [-glo, 0) and of higher ranks
// at [npad, npad + ghi) (npad = owned rows rounded up to 64), so local order
// is global order and every row keeps the reference's column order.
#pragma once
#include <cstdint>
#include <vector>

namespace cfd2 {

std::vector<uint64_t> partition_starts(uint64_t n, int R);
int owner_of(const std::vector<uint64_t>& starts, uint64_t g);

struct HaloPeer {
  int rank = 0;
  int32_t recv_rel = 0;   // local index of the first ghost this peer sends
  uint32_t recv_cnt = 0;
  uint32_t send_off = 0;  // into HaloPlan::send_idx
  uint32_t send_cnt = 0;
  int32_t direct = -1;    // the rows sent are the contiguous run [direct, direct + send_cnt) (else -1)
};

struct HaloPlan {
  std::vector<HaloPeer> peers;
  std::vector<int32_t> send_idx;  // owned local rows, grouped per peer, ascending
  int32_t* d_send_idx = nullptr;
  float* d_stage = nullptr;       // pack buffer (send_idx.size() x max comps)
  int max_comps = 0;
  // every peer's send rows are one contiguous run (x-major slabs: the first /
  // last columns of cells): fields are sent straight from their rows, no pack
  bool all_direct = false;
  // rows reading ghosts: [0, lo_end) (lower ghosts) and [hi_begin, n) (upper);
  // the rows between are interior and overlap the exchange (multiples of 4)
  uint32_t lo_end = 0, hi_begin = 0;
};

// Ghost list (ascending) of owned rows [c0, c1) whose global CSR pattern is
// (row[0..n], col); returns glo (ghosts below c0).
uint32_t collect_ghosts(uint64_t c0, uint64_t c1, const uint32_t* row, uint32_t n, const uint32_t* col,
                        std::vector<uint32_t>& ghost);

// Rows of [0, n) that read lower ghosts end before lo_end, rows reading upper
// ghosts start at hi_begin (multiples of 4; the rows between are interior).
void interior_rows(const std::vector<uint64_t>& starts, int rank, const uint32_t* row, uint32_t n,
                   const uint32_t* col, uint32_t& lo_end, uint32_t& hi_begin);

// Halo plan from every rank's ghost list (ascending global ids): this rank
// receives its ghosts owned by q from q and sends q the rows of q's list it
// owns (general patterns: the AMG levels, whose ghosts include the coarse
// rows their prolongation reads).  lo_end / hi_begin are left at 0.
HaloPlan build_halo_plan_lists(const std::vector<uint64_t>& starts, int rank,
                               const std::vector<std::vector<uint32_t>>& ghosts, uint32_t glo, uint32_t npad);

// Halo plan for a symmetric pattern: the rows this rank sends to peer q are its
// owned rows with a column owned by q (= q's ghosts from this rank).
HaloPlan build_halo_plan(const std::vector<uint64_t>& starts, int rank, const uint32_t* row, uint32_t n,
                         const uint32_t* col, const std::vector<uint32_t>& ghost, uint32_t glo, uint32_t npad);

}  // namespace cfd2
