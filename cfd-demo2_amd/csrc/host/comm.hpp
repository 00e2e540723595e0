// Communication layer of the distributed solver.
//
// A rank exchanges halos with its slab neighbours and all-gathers small
// vectors of per-rank partial sums.  Every operation is stream-ordered on the
// caller's HIP stream.  Two transports:
//   RcclComm  -- one process per GPU, RCCL point-to-point + all-gather over
//                xGMI (the production path; torch.distributed's "nccl" is RCCL).
//   LocalComm -- several ranks in ONE process (one host thread per rank, any
//                devices, including all on one GPU): peer copies ordered by HIP
//                events.  Used by cfd_group_* and by the single-GPU parity
//                tests of the distributed algorithm (RCCL refuses two ranks on
//                one device).
#pragma once
#include <hip/hip_runtime_api.h>

#include <condition_variable>
#include <cstdint>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <vector>

namespace cfd2 {

struct RcclError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

// One point-to-point transfer with `peer`: send sbytes from sbuf (if > 0),
// receive rbytes into rbuf (if > 0).  Transfers with the same peer are matched
// in list order, send k of one side with receive k of the other.
struct Msg {
  int peer;
  const void* sbuf;
  size_t sbytes;
  void* rbuf;
  size_t rbytes;
};

// Traffic counters of one rank's transport (cfd_comm_stats).
struct CommStats {
  uint64_t exchanges = 0, allgathers = 0, bytes_sent = 0, bytes_gathered = 0;
};

class Comm {
 public:
  virtual ~Comm() = default;
  int rank = 0, size = 1;
  int kind = 0;  // cfd_comm_stats.transport
  CommStats stats;
  // the transport's own view of the communicator (RCCL: ncclCommCount /
  // ncclCommUserRank; the others: size / rank)
  virtual int comm_count() const { return size; }
  virtual int comm_rank() const { return rank; }
  void count_exchange(const std::vector<Msg>& msgs) {
    ++stats.exchanges;
    for (const Msg& m : msgs) stats.bytes_sent += m.sbytes;
  }
  void count_allgather(size_t bytes) {
    ++stats.allgathers;
    stats.bytes_gathered += bytes;
  }
  virtual void exchange(const std::vector<Msg>& msgs, hipStream_t s) = 0;
  // recv[r * bytes ...] = rank r's send (bytes each), all ranks
  virtual void allgather(const void* send, void* recv, size_t bytes, hipStream_t s) = 0;
  // Variable-size in-place all-gather: every rank's piece [off[r], off[r+1]) of
  // buf (bytes) is distributed to all ranks.
  void allgatherv_inplace(void* buf, const std::vector<size_t>& off, hipStream_t s);
  // A rank failed: wake every rank blocked in this transport (in-process
  // group) so they fail too instead of waiting forever.  RCCL / host
  // transports: no-op (the launcher tears the processes down).
  virtual void abort() {}
  // After every rank has returned from a failed collective call: clear the
  // abort so the group can be used again (the caller restores a consistent
  // state, e.g. by cfd_state_load; a symmetric failure such as divergence
  // leaves every rank at the same point anyway).
  virtual void reset() {}
};

// ---- RCCL ----
constexpr int kUniqueIdBytes = 128;
void rccl_unique_id(uint8_t out[kUniqueIdBytes]);
std::unique_ptr<Comm> make_rccl_comm(int nranks, int rank, const uint8_t uid[kUniqueIdBytes]);

// ---- host-staged callbacks (test transport, cfd_solver_create_dist_host) ----
using HostExchangeFn = int32_t (*)(void* user, int32_t n, const int32_t* peer, void* const* send,
                                   const uint64_t* send_bytes, void* const* recv, const uint64_t* recv_bytes);
using HostAllgatherFn = int32_t (*)(void* user, void* send, void* recv, uint64_t bytes);
std::unique_ptr<Comm> make_host_comm(int nranks, int rank, HostExchangeFn ex, HostAllgatherFn ag, void* user);

// ---- in-process group ----
class LocalGroup {
 public:
  explicit LocalGroup(int n);
  ~LocalGroup();
  int size() const { return n_; }
  // throws std::runtime_error once the group is aborted (sticky)
  void barrier();
  void abort();
  void reset();  // only while no rank is inside barrier()
  struct Slot {
    std::vector<Msg> posted;
    const void* gather_src = nullptr;
    hipEvent_t ready = nullptr, done = nullptr;
    int device = 0;
  };
  std::vector<Slot> slots;

 private:
  int n_;
  std::mutex mu_;
  std::condition_variable cv_;
  int arrived_ = 0;
  uint64_t gen_ = 0;
  bool aborted_ = false;
};

std::unique_ptr<Comm> make_local_comm(std::shared_ptr<LocalGroup> g, int rank, int device);

}  // namespace cfd2
