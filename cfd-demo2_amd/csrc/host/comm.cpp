// Transports of the distributed solver: RCCL (one process per GPU) and an
// in-process group (one host thread per rank).  See comm.hpp.
#include "comm.hpp"

#include <rccl/rccl.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>

#include "solver_impl.hpp"

namespace cfd2 {

#define CFD_NCCL(expr)                                                                   \
  do {                                                                                   \
    ncclResult_t _r = (expr);                                                            \
    if (_r != ncclSuccess) throw RcclError(std::string(#expr) + ": " + ncclGetErrorString(_r)); \
  } while (0)

// ------------------------------------------------------------- watchdog
const char* comm_label_name(int label) {
  switch (label) {  // Solver::CommCat
    case -1: return "setup";
    case 0: return "Krylov halo";
    case 1: return "state halo";
    case 2: return "reduction all-gather";
    case 3: return "replicated AMG level all-gather";
    default: return "AMG level halo";
  }
}

Watchdog::Watchdog(int rank, int device, double timeout_s, AsyncErr err, Abort abort)
    : rank_(rank), device_(device), timeout_s_(timeout_s), err_(std::move(err)), abort_(std::move(abort)) {
  if (enabled()) th_ = std::thread([this] { loop(); });
}

Watchdog::~Watchdog() {
  stop();
  for (const Pending& p : pend_) (void)hipEventDestroy(p.ev);
  for (hipEvent_t e : free_) (void)hipEventDestroy(e);
}

void Watchdog::stop() {
  if (th_.joinable()) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    th_.join();
  }
}

void Watchdog::note_stream(hipStream_t s, const char* op, int label, size_t bytes) {
  if (!enabled()) return;
  hipEvent_t ev = nullptr;
  {
    std::lock_guard<std::mutex> lk(mu_);
    if (!free_.empty()) {
      ev = free_.back();
      free_.pop_back();
    }
  }
  if (!ev) CFD_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  CFD_HIP(hipEventRecord(ev, s));
  std::lock_guard<std::mutex> lk(mu_);
  pend_.push_back({ev, op, label, bytes, ++seq_, std::chrono::steady_clock::now()});
}

void Watchdog::host_begin(const char* op, int label) {
  if (!enabled()) return;
  std::lock_guard<std::mutex> lk(mu_);
  host_active_ = true;
  host_op_ = op;
  host_label_ = label;
  host_seq_ = ++seq_;
  host_t_ = std::chrono::steady_clock::now();
}

void Watchdog::host_end() {
  if (!enabled()) return;
  std::lock_guard<std::mutex> lk(mu_);
  host_active_ = false;
}

void Watchdog::loop() {
  bool device_set = false;
  std::unique_lock<std::mutex> lk(mu_);
  while (!stop_) {
    cv_.wait_for(lk, std::chrono::milliseconds(200), [&] { return stop_; });
    if (stop_) break;
    const auto now = std::chrono::steady_clock::now();
    const std::string e = err_ ? err_() : std::string();
    if (!e.empty()) {
      if (!pend_.empty()) {
        const Pending& p = pend_.front();
        fire("asynchronous transport error: " + e, p.op, p.label, p.bytes, p.seq,
             std::chrono::duration<double>(now - p.t).count());
      }
      fire("asynchronous transport error: " + e, host_active_ ? host_op_ : "(none in flight)", host_label_, 0,
           host_seq_, host_active_ ? std::chrono::duration<double>(now - host_t_).count() : 0.0);
    }
    if (host_active_) {
      const double age = std::chrono::duration<double>(now - host_t_).count();
      if (age > timeout_s_) fire("host-blocking operation timed out", host_op_, host_label_, 0, host_seq_, age);
    }
    if (!pend_.empty() && !device_set) {
      (void)hipSetDevice(device_);
      device_set = true;
    }
    while (!pend_.empty()) {
      const Pending p = pend_.front();
      const hipError_t q = hipEventQuery(p.ev);
      if (q == hipSuccess) {
        pend_.pop_front();
        free_.push_back(p.ev);
        continue;
      }
      const double age = std::chrono::duration<double>(now - p.t).count();
      if (q != hipErrorNotReady)
        fire(std::string("completion query failed: ") + hipGetErrorString(q), p.op, p.label, p.bytes, p.seq, age);
      if (age > timeout_s_) fire("stream operation not complete", p.op, p.label, p.bytes, p.seq, age);
      break;
    }
  }
}

void Watchdog::fire(const std::string& why, const char* op, int label, size_t bytes, uint64_t seq, double age) {
  std::fprintf(stderr,
               "cfd2 comm watchdog: rank %d (HIP device %d): %s -- operation #%llu '%s' (category: %s, %zu bytes) "
               "in flight for %.1f s (limit %.1f s, cfd_config.comm_timeout_s); aborting the transport and exiting "
               "with status %d\n",
               rank_, device_, why.c_str(), (unsigned long long)seq, op, comm_label_name(label), bytes, age,
               timeout_s_, kCommWatchdogExit);
  std::fflush(stderr);
  std::fflush(stdout);
  if (abort_) abort_();
  std::_Exit(kCommWatchdogExit);
}

void Comm::allgatherv_inplace(void* buf, const std::vector<size_t>& off, hipStream_t s) {
  std::vector<Msg> msgs;
  char* b = static_cast<char*>(buf);
  for (int q = 0; q < size; ++q) {
    if (q == rank) continue;
    msgs.push_back({q, b + off[rank], off[rank + 1] - off[rank], b + off[q], off[q + 1] - off[q]});
  }
  exchange(msgs, s);
}

// ------------------------------------------------------------------- RCCL
void rccl_unique_id(uint8_t out[kUniqueIdBytes]) {
  static_assert(sizeof(ncclUniqueId) == kUniqueIdBytes, "ncclUniqueId size");
  ncclUniqueId id;
  CFD_NCCL(ncclGetUniqueId(&id));
  std::memcpy(out, &id, sizeof(id));
}

namespace {

class RcclComm final : public Comm {
 public:
  RcclComm(int nranks, int r, const uint8_t uid[kUniqueIdBytes], int device, double timeout_s)
      : wd_(r, device, timeout_s,
            [this]() -> std::string {
              ncclComm_t c = comm_;
              if (!c) return {};
              ncclResult_t a = ncclSuccess;
              if (ncclCommGetAsyncError(c, &a) != ncclSuccess) return "ncclCommGetAsyncError failed";
              return (a == ncclSuccess || a == ncclInProgress) ? std::string() : std::string(ncclGetErrorString(a));
            },
            [this] {
              ncclComm_t c = comm_;
              if (c) (void)ncclCommAbort(c);
            }) {
    ncclUniqueId id;
    std::memcpy(&id, uid, sizeof(id));
    wd_.host_begin("ncclCommInitRank", -1);  // blocks until every rank has joined
    ncclComm_t c = nullptr;
    CFD_NCCL(ncclCommInitRank(&c, nranks, id, r));
    comm_ = c;
    wd_.host_end();
    rank = r;
    size = nranks;
    kind = 1;
  }
  int comm_count() const override {
    int n = -1;
    return ncclCommCount(comm_, &n) == ncclSuccess ? n : -1;
  }
  int comm_rank() const override {
    int r = -1;
    return ncclCommUserRank(comm_, &r) == ncclSuccess ? r : -1;
  }
  ~RcclComm() override {
    wd_.stop();  // no poll of the communicator while it goes
    ncclComm_t c = comm_;
    comm_ = nullptr;
    if (c) (void)ncclCommDestroy(c);
  }
  void exchange(const std::vector<Msg>& msgs, hipStream_t s) override {
    if (msgs.empty()) return;
    count_exchange(msgs);
    size_t bytes = 0;
    CFD_NCCL(ncclGroupStart());
    for (const Msg& m : msgs) {
      if (m.sbytes) CFD_NCCL(ncclSend(m.sbuf, m.sbytes, ncclChar, m.peer, comm_, s));
      if (m.rbytes) CFD_NCCL(ncclRecv(m.rbuf, m.rbytes, ncclChar, m.peer, comm_, s));
      bytes += m.sbytes + m.rbytes;
    }
    CFD_NCCL(ncclGroupEnd());
    wd_.note_stream(s, "grouped ncclSend/ncclRecv", label, bytes);
  }
  void allgather(const void* send, void* recv, size_t bytes, hipStream_t s) override {
    count_allgather(bytes);
    CFD_NCCL(ncclAllGather(send, recv, bytes, ncclChar, comm_, s));
    wd_.note_stream(s, "ncclAllGather", label, bytes);
  }

 private:
  std::atomic<ncclComm_t> comm_{nullptr};
  Watchdog wd_;
};

}  // namespace

std::unique_ptr<Comm> make_rccl_comm(int nranks, int rank, const uint8_t uid[kUniqueIdBytes], int device,
                                     double timeout_s) {
  return std::make_unique<RcclComm>(nranks, rank, uid, device, timeout_s);
}

// ------------------------------------------------------ host-staged callbacks
namespace {

// Every transfer goes device -> host staging -> caller callback -> host
// staging -> device, after the stream has drained (test transport only).
class HostComm final : public Comm {
 public:
  HostComm(int nranks, int r, HostExchangeFn ex, HostAllgatherFn ag, void* user, int device, double timeout_s)
      : ex_(ex), ag_(ag), user_(user), wd_(r, device, timeout_s, nullptr, nullptr) {
    rank = r;
    size = nranks;
    kind = 3;
  }
  void exchange(const std::vector<Msg>& msgs, hipStream_t s) override {
    if (msgs.empty()) return;
    count_exchange(msgs);
    CFD_HIP(hipStreamSynchronize(s));
    const size_t n = msgs.size();
    std::vector<std::vector<char>> sb(n), rb(n);
    std::vector<int32_t> peer(n);
    std::vector<void*> sp(n), rp(n);
    std::vector<uint64_t> sn(n), rn(n);
    for (size_t i = 0; i < n; ++i) {
      const Msg& m = msgs[i];
      peer[i] = m.peer;
      sb[i].resize(m.sbytes + 1);
      rb[i].resize(m.rbytes + 1);
      if (m.sbytes) CFD_HIP(hipMemcpy(sb[i].data(), m.sbuf, m.sbytes, hipMemcpyDeviceToHost));
      sp[i] = sb[i].data();
      rp[i] = rb[i].data();
      sn[i] = m.sbytes;
      rn[i] = m.rbytes;
    }
    wd_.host_begin("host-staged exchange callback", label);
    const int32_t rc = ex_(user_, (int32_t)n, peer.data(), sp.data(), sn.data(), rp.data(), rn.data());
    wd_.host_end();
    if (rc != 0) throw std::runtime_error("host transport: exchange callback failed");
    for (size_t i = 0; i < n; ++i)
      if (msgs[i].rbytes) CFD_HIP(hipMemcpy(msgs[i].rbuf, rb[i].data(), msgs[i].rbytes, hipMemcpyHostToDevice));
  }
  void allgather(const void* send, void* recv, size_t bytes, hipStream_t s) override {
    count_allgather(bytes);
    CFD_HIP(hipStreamSynchronize(s));
    std::vector<char> sb(bytes + 1), rb((size_t)size * bytes + 1);
    if (bytes) CFD_HIP(hipMemcpy(sb.data(), send, bytes, hipMemcpyDeviceToHost));
    wd_.host_begin("host-staged all-gather callback", label);
    const int32_t rc = ag_(user_, sb.data(), rb.data(), bytes);
    wd_.host_end();
    if (rc != 0) throw std::runtime_error("host transport: allgather callback failed");
    if (bytes) CFD_HIP(hipMemcpy(recv, rb.data(), (size_t)size * bytes, hipMemcpyHostToDevice));
  }

 private:
  HostExchangeFn ex_;
  HostAllgatherFn ag_;
  void* user_;
  Watchdog wd_;
};

}  // namespace

std::unique_ptr<Comm> make_host_comm(int nranks, int rank, HostExchangeFn ex, HostAllgatherFn ag, void* user,
                                     int device, double timeout_s) {
  return std::make_unique<HostComm>(nranks, rank, ex, ag, user, device, timeout_s);
}

// ----------------------------------------------------------- local group
LocalGroup::LocalGroup(int n) : slots(n), n_(n) {}

LocalGroup::~LocalGroup() {
  for (auto& sl : slots) {
    if (sl.ready) (void)hipEventDestroy(sl.ready);
    if (sl.done) (void)hipEventDestroy(sl.done);
  }
}

void LocalGroup::barrier() {
  std::unique_lock<std::mutex> lk(mu_);
  if (aborted_) throw std::runtime_error("in-process group aborted: another rank failed");
  const uint64_t g = gen_;
  if (++arrived_ == n_) {
    arrived_ = 0;
    ++gen_;
    cv_.notify_all();
  } else {
    cv_.wait(lk, [&] { return gen_ != g || aborted_; });
    if (gen_ == g) throw std::runtime_error("in-process group aborted: another rank failed");
  }
}

void LocalGroup::abort() {
  std::lock_guard<std::mutex> lk(mu_);
  aborted_ = true;
  cv_.notify_all();
}

void LocalGroup::reset() {
  std::lock_guard<std::mutex> lk(mu_);
  aborted_ = false;
  arrived_ = 0;
  ++gen_;
  for (auto& sl : slots) {
    sl.posted.clear();
    sl.gather_src = nullptr;
  }
}

namespace {

// Pull model: after barrier 1 every rank copies what it receives out of the
// senders' buffers (ordered after the senders' `ready` events), records `done`;
// after barrier 2 each sender's stream waits on its receivers' `done`, so
// later writes to a send buffer cannot overtake a pending pull.
class LocalComm final : public Comm {
 public:
  LocalComm(std::shared_ptr<LocalGroup> g, int r, int device) : g_(std::move(g)) {
    rank = r;
    size = g_->size();
    kind = 2;
    auto& sl = g_->slots[r];
    sl.device = device;
    CFD_HIP(hipSetDevice(device));
    CFD_HIP(hipEventCreateWithFlags(&sl.ready, hipEventDisableTiming));
    CFD_HIP(hipEventCreateWithFlags(&sl.done, hipEventDisableTiming));
  }

  void exchange(const std::vector<Msg>& msgs, hipStream_t s) override {
    count_exchange(msgs);
    auto& me = g_->slots[rank];
    me.posted = msgs;
    CFD_HIP(hipEventRecord(me.ready, s));
    g_->barrier();
    std::vector<int> used(size, 0);
    std::vector<char> senders(size, 0);
    for (const Msg& m : msgs) {
      if (!m.rbytes) continue;
      const auto& src = g_->slots[m.peer];
      // k-th receive from peer q <-> k-th send of q to this rank
      int k = used[m.peer]++;
      const Msg* match = nullptr;
      for (const Msg& sm : src.posted) {
        if (sm.peer != rank || !sm.sbytes) continue;
        if (k-- == 0) {
          match = &sm;
          break;
        }
      }
      if (!match || match->sbytes != m.rbytes)
        throw std::logic_error("LocalComm: unmatched transfer " + std::to_string(m.peer) + " -> " +
                               std::to_string(rank));
      if (!senders[m.peer]) {
        CFD_HIP(hipStreamWaitEvent(s, src.ready, 0));
        senders[m.peer] = 1;
      }
      if (src.device == me.device)
        CFD_HIP(hipMemcpyAsync(m.rbuf, match->sbuf, m.rbytes, hipMemcpyDeviceToDevice, s));
      else
        CFD_HIP(hipMemcpyPeerAsync(m.rbuf, me.device, match->sbuf, src.device, m.rbytes, s));
    }
    CFD_HIP(hipEventRecord(me.done, s));
    g_->barrier();
    std::vector<char> waited(size, 0);
    for (const Msg& m : msgs)
      if (m.sbytes && !waited[m.peer]) {
        CFD_HIP(hipStreamWaitEvent(s, g_->slots[m.peer].done, 0));
        waited[m.peer] = 1;
      }
  }

  void abort() override { g_->abort(); }
  void reset() override { g_->reset(); }

  void allgather(const void* send, void* recv, size_t bytes, hipStream_t s) override {
    count_allgather(bytes);
    auto& me = g_->slots[rank];
    me.gather_src = send;
    CFD_HIP(hipEventRecord(me.ready, s));
    g_->barrier();
    for (int q = 0; q < size; ++q) {
      const auto& src = g_->slots[q];
      if (q != rank) CFD_HIP(hipStreamWaitEvent(s, src.ready, 0));
      char* dst = static_cast<char*>(recv) + (size_t)q * bytes;
      if (src.device == me.device)
        CFD_HIP(hipMemcpyAsync(dst, src.gather_src, bytes, hipMemcpyDeviceToDevice, s));
      else
        CFD_HIP(hipMemcpyPeerAsync(dst, me.device, src.gather_src, src.device, bytes, s));
    }
    CFD_HIP(hipEventRecord(me.done, s));
    g_->barrier();
    for (int q = 0; q < size; ++q)
      if (q != rank) CFD_HIP(hipStreamWaitEvent(s, g_->slots[q].done, 0));
  }

 private:
  std::shared_ptr<LocalGroup> g_;
};

}  // namespace

std::unique_ptr<Comm> make_local_comm(std::shared_ptr<LocalGroup> g, int rank, int device) {
  return std::make_unique<LocalComm>(std::move(g), rank, device);
}

}  // namespace cfd2
