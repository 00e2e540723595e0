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

#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
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

// Progress watchdog of a transport (cfd_config.comm_timeout_s).  A stalled
// collective otherwise hangs the process in its next stream synchronisation
// with no diagnostic.  Every operation the transport enqueues is followed by
// a completion event on its stream (note_stream); operations that block the
// host (the host-staged callbacks, ncclCommInitRank) are bracketed by
// host_begin / host_end.  A background thread polls them (and the
// transport's asynchronous error, RCCL: ncclCommGetAsyncError) every 200 ms.
// When an operation is older than the timeout, or an asynchronous error or
// a failed event query appears, it prints the rank, device, operation,
// category and age on stderr, aborts the transport (RCCL: ncclCommAbort)
// and ends the process with status kCommWatchdogExit.  It never re-execs.
constexpr int kCommWatchdogExit = 70;
class Watchdog {
 public:
  using AsyncErr = std::function<std::string()>;  // "" while healthy
  using Abort = std::function<void()>;
  // timeout_s <= 0: disabled (no thread, every call a no-op)
  Watchdog(int rank, int device, double timeout_s, AsyncErr err, Abort abort);
  ~Watchdog();
  Watchdog(const Watchdog&) = delete;
  Watchdog& operator=(const Watchdog&) = delete;
  bool enabled() const { return timeout_s_ > 0.0; }
  void note_stream(hipStream_t s, const char* op, int label, size_t bytes);
  void host_begin(const char* op, int label);
  void host_end();
  void stop();  // joins the polling thread (idempotent)

 private:
  struct Pending {
    hipEvent_t ev;
    const char* op;
    int label;
    size_t bytes;
    uint64_t seq;
    std::chrono::steady_clock::time_point t;
  };
  void loop();
  [[noreturn]] void fire(const std::string& why, const char* op, int label, size_t bytes, uint64_t seq, double age);
  int rank_, device_;
  double timeout_s_;
  AsyncErr err_;
  Abort abort_;
  std::mutex mu_;
  std::condition_variable cv_;
  bool stop_ = false;
  std::deque<Pending> pend_;
  std::vector<hipEvent_t> free_;
  uint64_t seq_ = 0;
  bool host_active_ = false;
  const char* host_op_ = "";
  int host_label_ = -1;
  uint64_t host_seq_ = 0;
  std::chrono::steady_clock::time_point host_t_;
  std::thread th_;
};
// name of a Comm::label (the solver's communication categories, cfd_comm_timing)
const char* comm_label_name(int label);

class Comm {
 public:
  virtual ~Comm() = default;
  int rank = 0, size = 1;
  int kind = 0;  // cfd_comm_stats.transport
  // category of the operations the solver issues next (Solver::CommCat; -1
  // setup): names the stalled operation in a watchdog report
  int label = -1;
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
// timeout_s: the progress watchdog's limit (<= 0 off); device: the rank's GPU
std::unique_ptr<Comm> make_rccl_comm(int nranks, int rank, const uint8_t uid[kUniqueIdBytes], int device = 0,
                                     double timeout_s = 0.0);

// ---- host-staged callbacks (test transport, cfd_solver_create_dist_host) ----
using HostExchangeFn = int32_t (*)(void* user, int32_t n, const int32_t* peer, void* const* send,
                                   const uint64_t* send_bytes, void* const* recv, const uint64_t* recv_bytes);
using HostAllgatherFn = int32_t (*)(void* user, void* send, void* recv, uint64_t bytes);
std::unique_ptr<Comm> make_host_comm(int nranks, int rank, HostExchangeFn ex, HostAllgatherFn ag, void* user,
                                     int device = 0, double timeout_s = 0.0);

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
