// Transports of the distributed solver: RCCL (one process per GPU) and an
// in-process group (one host thread per rank).  See comm.hpp.
#include "comm.hpp"

#include <rccl/rccl.h>

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
  RcclComm(int nranks, int r, const uint8_t uid[kUniqueIdBytes]) {
    ncclUniqueId id;
    std::memcpy(&id, uid, sizeof(id));
    CFD_NCCL(ncclCommInitRank(&comm_, nranks, id, r));
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
    if (comm_) (void)ncclCommDestroy(comm_);
  }
  void exchange(const std::vector<Msg>& msgs, hipStream_t s) override {
    if (msgs.empty()) return;
    count_exchange(msgs);
    CFD_NCCL(ncclGroupStart());
    for (const Msg& m : msgs) {
      if (m.sbytes) CFD_NCCL(ncclSend(m.sbuf, m.sbytes, ncclChar, m.peer, comm_, s));
      if (m.rbytes) CFD_NCCL(ncclRecv(m.rbuf, m.rbytes, ncclChar, m.peer, comm_, s));
    }
    CFD_NCCL(ncclGroupEnd());
  }
  void allgather(const void* send, void* recv, size_t bytes, hipStream_t s) override {
    count_allgather(bytes);
    CFD_NCCL(ncclAllGather(send, recv, bytes, ncclChar, comm_, s));
  }

 private:
  ncclComm_t comm_ = nullptr;
};

}  // namespace

std::unique_ptr<Comm> make_rccl_comm(int nranks, int rank, const uint8_t uid[kUniqueIdBytes]) {
  return std::make_unique<RcclComm>(nranks, rank, uid);
}

// ------------------------------------------------------ host-staged callbacks
namespace {

// Every transfer goes device -> host staging -> caller callback -> host
// staging -> device, after the stream has drained (test transport only).
class HostComm final : public Comm {
 public:
  HostComm(int nranks, int r, HostExchangeFn ex, HostAllgatherFn ag, void* user)
      : ex_(ex), ag_(ag), user_(user) {
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
    if (ex_(user_, (int32_t)n, peer.data(), sp.data(), sn.data(), rp.data(), rn.data()) != 0)
      throw std::runtime_error("host transport: exchange callback failed");
    for (size_t i = 0; i < n; ++i)
      if (msgs[i].rbytes) CFD_HIP(hipMemcpy(msgs[i].rbuf, rb[i].data(), msgs[i].rbytes, hipMemcpyHostToDevice));
  }
  void allgather(const void* send, void* recv, size_t bytes, hipStream_t s) override {
    count_allgather(bytes);
    CFD_HIP(hipStreamSynchronize(s));
    std::vector<char> sb(bytes + 1), rb((size_t)size * bytes + 1);
    if (bytes) CFD_HIP(hipMemcpy(sb.data(), send, bytes, hipMemcpyDeviceToHost));
    if (ag_(user_, sb.data(), rb.data(), bytes) != 0) throw std::runtime_error("host transport: allgather callback failed");
    if (bytes) CFD_HIP(hipMemcpy(recv, rb.data(), (size_t)size * bytes, hipMemcpyHostToDevice));
  }

 private:
  HostExchangeFn ex_;
  HostAllgatherFn ag_;
  void* user_;
};

}  // namespace

std::unique_ptr<Comm> make_host_comm(int nranks, int rank, HostExchangeFn ex, HostAllgatherFn ag, void* user) {
  return std::make_unique<HostComm>(nranks, rank, ex, ag, user);
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
