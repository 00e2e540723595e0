// C ABI of the solver (include/cfd2_amd.h).  Each entry replaces one method of
// the reference's `impl GpuSolver` (src/solver/gpu/solver.rs, init/mod.rs);
// exceptions become status codes (the reference panics).
#include <algorithm>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <exception>
#include <memory>
#include <new>
#include <thread>
#include <vector>

#include "error.hpp"
#include "solver_impl.hpp"

struct cfd_solver {
  cfd2::Solver* s;
};

using cfd2::set_error;

namespace {

template <class F>
cfd_status guard(F&& f) {
  try {
    f();
    return CFD_OK;
  } catch (const cfd2::HipError& e) {
    return set_error(CFD_ERR_HIP, e.what());
  } catch (const cfd2::RcclError& e) {
    return set_error(CFD_ERR_RCCL, e.what());
  } catch (const std::domain_error& e) {
    return set_error(CFD_ERR_DIVERGED, e.what());
  } catch (const std::invalid_argument& e) {
    const std::string m = e.what();
    return set_error(m.find("Diagonal not found") != std::string::npos ? CFD_ERR_DIAGONAL : CFD_ERR_INVALID, m);
  } catch (const std::bad_alloc&) {
    return set_error(CFD_ERR_HIP, "out of host memory");
  } catch (const std::exception& e) {
    return set_error(CFD_ERR_INTERNAL, e.what());
  }
}

#define CHECK_S(h)                                       \
  if (!(h) || !(h)->s) return set_error(CFD_ERR_INVALID, "null solver handle")

template <class F>
cfd_status set_const(cfd_solver* s, F&& f) {  // setters write + update_constants
  CHECK_S(s);
  f(s->s->constants);
  return CFD_OK;
}

}  // namespace

extern "C" {

void cfd_config_default(cfd_config* c) {
  if (!c) return;
  c->n_outer_correctors = 20;
  c->convergence_lag = 1;
  c->fixed_outer = 0;
  c->fixed_inner = 0;
  c->max_restart = 50;
  c->max_outer_restarts = 20;
  c->fgmres_rtol = 1e-5f;
  c->fgmres_atol = 1e-7f;
  c->log_level = 0;
  c->amg_rebuild_interval = 0;
  c->amg_local_aggregation = 0;
  c->comm_timeout_s = 180.0f;
}

cfd_status cfd_solver_create(const cfd_mesh_view* mesh, const cfd_config* cfg, int32_t hip_device,
                             cfd_solver** out) {
  if (!mesh || !out) return set_error(CFD_ERR_INVALID, "null argument");
  cfd_config c;
  if (cfg)
    c = *cfg;
  else
    cfd_config_default(&c);
  cfd2::Solver* sp = nullptr;
  const cfd_status st = guard([&] { sp = new cfd2::Solver(*mesh, c, hip_device); });
  if (st != CFD_OK) return st;
  *out = new cfd_solver{sp};
  return CFD_OK;
}

void cfd_solver_destroy(cfd_solver* s) {
  if (!s) return;
  delete s->s;
  delete s;
}

cfd_status cfd_set_u(cfd_solver* s, const double* uv) {
  CHECK_S(s);
  if (!uv) return set_error(CFD_ERR_INVALID, "null u");
  return guard([&] { s->s->set_u(uv); });
}
cfd_status cfd_set_p(cfd_solver* s, const double* p) {
  CHECK_S(s);
  if (!p) return set_error(CFD_ERR_INVALID, "null p");
  return guard([&] { s->s->set_p(p); });
}
cfd_status cfd_get_constants(const cfd_solver* s, cfd_constants* out) {
  CHECK_S(s);
  if (!out) return set_error(CFD_ERR_INVALID, "null out");
  *out = s->s->constants;
  return CFD_OK;
}
cfd_status cfd_set_constants(cfd_solver* s, const cfd_constants* c) {
  CHECK_S(s);
  if (!c) return set_error(CFD_ERR_INVALID, "null constants");
  s->s->constants = *c;
  return CFD_OK;
}
cfd_status cfd_set_dt(cfd_solver* s, float dt) {  // solver.rs:36-44
  return set_const(s, [&](cfd_constants& c) {
    c.dt_old = (c.dt > 0.0f) ? c.dt : dt;
    c.dt = dt;
  });
}
cfd_status cfd_set_viscosity(cfd_solver* s, float v) { return set_const(s, [&](cfd_constants& c) { c.viscosity = v; }); }
cfd_status cfd_set_alpha_p(cfd_solver* s, float v) { return set_const(s, [&](cfd_constants& c) { c.alpha_p = v; }); }
cfd_status cfd_set_alpha_u(cfd_solver* s, float v) { return set_const(s, [&](cfd_constants& c) { c.alpha_u = v; }); }
cfd_status cfd_set_density(cfd_solver* s, float v) { return set_const(s, [&](cfd_constants& c) { c.density = v; }); }
cfd_status cfd_set_scheme(cfd_solver* s, uint32_t v) { return set_const(s, [&](cfd_constants& c) { c.scheme = v; }); }
cfd_status cfd_set_time_scheme(cfd_solver* s, uint32_t v) {
  return set_const(s, [&](cfd_constants& c) { c.time_scheme = v; });
}
cfd_status cfd_set_inlet_velocity(cfd_solver* s, float v) {
  return set_const(s, [&](cfd_constants& c) { c.inlet_velocity = v; });
}
cfd_status cfd_set_ramp_time(cfd_solver* s, float v) { return set_const(s, [&](cfd_constants& c) { c.ramp_time = v; }); }
cfd_status cfd_set_precond_type(cfd_solver* s, uint32_t v) {
  return set_const(s, [&](cfd_constants& c) { c.precond_type = v; });
}
// Kernels take the constants by value at launch, so the host copy *is* the
// uploaded uniform: update_constants (solver.rs:91-95) has nothing left to do.
cfd_status cfd_update_constants(cfd_solver* s) {
  CHECK_S(s);
  return CFD_OK;
}
cfd_status cfd_initialize_history(cfd_solver* s) {
  CHECK_S(s);
  return guard([&] { s->s->initialize_history(); });
}
cfd_status cfd_step(cfd_solver* s) {
  CHECK_S(s);
  return guard([&] { s->s->step(); });
}
cfd_status cfd_synchronize(cfd_solver* s) {
  CHECK_S(s);
  return guard([&] {
    CFD_HIP(hipSetDevice(s->s->device));
    CFD_HIP(hipDeviceSynchronize());
  });
}
cfd_status cfd_get_u(cfd_solver* s, double* uv) {
  CHECK_S(s);
  if (!uv) return set_error(CFD_ERR_INVALID, "null out");
  return guard([&] { s->s->get_u(uv); });
}
cfd_status cfd_get_p(cfd_solver* s, double* p) {
  CHECK_S(s);
  if (!p) return set_error(CFD_ERR_INVALID, "null out");
  return guard([&] { s->s->get_p(p); });
}
cfd_status cfd_get_d_p(cfd_solver* s, double* dp) {
  CHECK_S(s);
  if (!dp) return set_error(CFD_ERR_INVALID, "null out");
  return guard([&] { s->s->get_d_p(dp); });
}
cfd_status cfd_get_step_info(const cfd_solver* s, cfd_step_info* out) {
  CHECK_S(s);
  if (!out) return set_error(CFD_ERR_INVALID, "null out");
  *out = s->s->info;
  return CFD_OK;
}
// The reference's stop state is three plain public fields (structs.rs:244-247)
// that callers write between steps (the GUI clears should_stop before it
// resumes, src/ui/app.rs:852-857); check_evolution reads and updates them.
cfd_status cfd_set_stop_state(cfd_solver* s, int32_t should_stop, uint32_t degenerate_count,
                              uint32_t steady_state_count) {
  CHECK_S(s);
  s->s->info.should_stop = should_stop ? 1 : 0;
  s->s->info.degenerate_count = degenerate_count;
  s->s->info.steady_state_count = steady_state_count;
  return CFD_OK;
}
cfd_status cfd_set_n_outer_correctors(cfd_solver* s, int32_t n) {
  CHECK_S(s);
  if (n < 0) return set_error(CFD_ERR_INVALID, "n_outer_correctors < 0");
  s->s->cfg.n_outer_correctors = n;  // read by every step (Solver::step)
  return CFD_OK;
}
cfd_status cfd_state_save(cfd_solver* s, const char* path) {
  CHECK_S(s);
  if (!path) return set_error(CFD_ERR_INVALID, "null path");
  // a rank of a group whose step failed holds a state from the middle of that
  // step: a checkpoint of it would later load as a consistent one
  if (s->s->needs_restore)
    return set_error(CFD_ERR_INVALID, "state save refused: the group needs restore after a failed step");
  return guard([&] { s->s->save_state(path); });
}
cfd_status cfd_state_load(cfd_solver* s, const char* path) {
  CHECK_S(s);
  if (!path) return set_error(CFD_ERR_INVALID, "null path");
  return guard([&] {
    s->s->load_state(path);
    s->s->needs_restore = false;  // a consistent state on this rank again
  });
}
uint32_t cfd_num_cells(const cfd_solver* s) { return (s && s->s) ? s->s->N : 0; }
uint32_t cfd_num_faces(const cfd_solver* s) { return (s && s->s) ? s->s->F : 0; }

cfd_status cfd_profile_enable(cfd_solver* s, int32_t enable) {
  CHECK_S(s);
  s->s->prof = enable != 0;
  return CFD_OK;
}
cfd_status cfd_profile_reset(cfd_solver* s) {
  CHECK_S(s);
  return guard([&] {
    CFD_HIP(hipStreamSynchronize(s->s->stream));
    s->s->graph_harvest_all(true);  // replays before the reset do not count
    s->s->prof_used = 0;
    s->s->prof_ms = 0.0;
    s->s->prof_launches = 0;
    s->s->prof_seq = 0;
    s->s->prof_grow(8192);  // 4096 timed launches without growing inside the timed steps
  });
}
cfd_status cfd_graph_enable(cfd_solver* s, int32_t enable) {
  CHECK_S(s);
  return guard([&] {
    CFD_HIP(hipSetDevice(s->s->device));
    s->s->drop_graphs();
    s->s->graph_on = enable != 0;
  });
}
cfd_status cfd_graph_stats(const cfd_solver* s, int32_t* enabled, uint64_t* captures, uint64_t* replays) {
  CHECK_S(s);
  if (enabled) *enabled = s->s->graph_on && s->s->R == 1 ? 1 : 0;
  if (captures) *captures = s->s->graph_captures;
  if (replays) *replays = s->s->graph_replays;
  return CFD_OK;
}
cfd_status cfd_profile_smoother(const cfd_solver* cs, double* total_ms, uint64_t* launches,
                                double* bytes_per_launch) {
  CHECK_S(cs);
  cfd2::Solver* s = cs->s;
  return guard([&] {
    CFD_HIP(hipStreamSynchronize(s->stream));
    s->graph_harvest_all(false);
    for (size_t k = 0; k + 1 < s->prof_used; k += 2) {
      float ms = 0.0f;
      CFD_HIP(hipEventElapsedTime(&ms, s->prof_ev[k], s->prof_ev[k + 1]));
      s->prof_ms += ms;
    }
    s->prof_used = 0;
    if (total_ms) *total_ms = s->prof_ms;
    if (launches) *launches = s->prof_launches;
    if (bytes_per_launch) *bytes_per_launch = s->smoother_bytes();
  });
}
cfd_status cfd_amg_levels(const cfd_solver* s, int32_t* num_levels, uint32_t* rows, uint64_t* nnz) {
  CHECK_S(s);
  const auto& L = s->s->levels;
  if (num_levels) *num_levels = (int32_t)L.size();
  for (size_t i = 0; i < L.size() && i < 20; ++i) {
    if (rows) rows[i] = L[i].dev.n;
    if (nnz) nnz[i] = L[i].nnz;
  }
  return CFD_OK;
}
cfd_status cfd_debug_amg_info(cfd_solver* s, int32_t level, int32_t* setup_path, uint64_t* digest) {
  CHECK_S(s);
  return guard([&] {
    if (setup_path) *setup_path = s->s->amg_setup_path;
    if (digest) *digest = s->s->amg_level_digest(level);
  });
}
double cfd_smoother_layout_bytes(const cfd_solver* s) { return (s && s->s) ? s->s->smoother_layout_bytes() : 0.0; }
double cfd_step_layout_bytes(const cfd_solver* s) { return (s && s->s) ? s->s->layout_step_bytes() : 0.0; }
double cfd_step_algorithmic_bytes(const cfd_solver* s) {
  return (s && s->s) ? s->s->algorithmic_step_bytes() : 0.0;
}
size_t cfd_debug_buffer_len(const cfd_solver* s, int32_t id) { return (s && s->s) ? s->s->debug_len(id) : 0; }
cfd_status cfd_debug_buffer(cfd_solver* s, int32_t id, float* out, size_t count) {
  CHECK_S(s);
  const size_t len = s->s->debug_len(id);
  if (!out || len == 0 || count < len) return set_error(CFD_ERR_INVALID, "bad debug buffer request");
  return guard([&] { s->s->debug_buffer(id, out); });
}
cfd_status cfd_debug_prepare_assemble(cfd_solver* s, int32_t assemble) {
  CHECK_S(s);
  return guard([&] { s->s->debug_prepare_assemble(assemble != 0); });
}

cfd_status cfd_debug_reference_semantics(cfd_solver* s, int32_t flags) {
  CHECK_S(s);
  return guard([&] { s->s->set_reference_semantics(flags); });
}

// ---------------------------------------------------------------- multi-GPU
cfd_status cfd_dist_unique_id(uint8_t out[128]) {
  if (!out) return set_error(CFD_ERR_INVALID, "null out");
  return guard([&] { cfd2::rccl_unique_id(out); });
}

cfd_status cfd_solver_create_dist(const cfd_mesh_view* mesh, const cfd_config* cfg, int32_t hip_device,
                                  int32_t nranks, int32_t rank, const uint8_t unique_id[128], cfd_solver** out) {
  if (!mesh || !out || !unique_id) return set_error(CFD_ERR_INVALID, "null argument");
  if (nranks < 1 || rank < 0 || rank >= nranks) return set_error(CFD_ERR_INVALID, "bad rank / nranks");
  cfd_config c;
  if (cfg)
    c = *cfg;
  else
    cfd_config_default(&c);
  cfd2::Solver* sp = nullptr;
  const cfd_status st = guard([&] {
    CFD_HIP(hipSetDevice(hip_device));
    auto comm = cfd2::make_rccl_comm(nranks, rank, unique_id, hip_device, c.comm_timeout_s);
    sp = new cfd2::Solver(*mesh, c, hip_device, std::move(comm));
  });
  if (st != CFD_OK) return st;
  *out = new cfd_solver{sp};
  return CFD_OK;
}

cfd_status cfd_solver_create_dist_host(const cfd_mesh_view* mesh, const cfd_config* cfg, int32_t hip_device,
                                       int32_t nranks, int32_t rank, cfd_exchange_fn exchange,
                                       cfd_allgather_fn allgather, void* user, cfd_solver** out) {
  if (!mesh || !out || !exchange || !allgather) return set_error(CFD_ERR_INVALID, "null argument");
  if (nranks < 1 || rank < 0 || rank >= nranks) return set_error(CFD_ERR_INVALID, "bad rank / nranks");
  cfd_config c;
  if (cfg)
    c = *cfg;
  else
    cfd_config_default(&c);
  cfd2::Solver* sp = nullptr;
  const cfd_status st = guard([&] {
    CFD_HIP(hipSetDevice(hip_device));
    auto comm = cfd2::make_host_comm(nranks, rank, exchange, allgather, user, hip_device, c.comm_timeout_s);
    sp = new cfd2::Solver(*mesh, c, hip_device, std::move(comm));
  });
  if (st != CFD_OK) return st;
  *out = new cfd_solver{sp};
  return CFD_OK;
}

cfd_status cfd_group_create(const cfd_mesh_view* mesh, const cfd_config* cfg, int32_t nranks,
                            const int32_t* devices, cfd_solver** out) {
  if (!mesh || !out || !devices || nranks < 1) return set_error(CFD_ERR_INVALID, "bad argument");
  cfd_config c;
  if (cfg)
    c = *cfg;
  else
    cfd_config_default(&c);
  auto group = std::make_shared<cfd2::LocalGroup>(nranks);
  std::vector<cfd2::Solver*> made;
  const cfd_status st = guard([&] {
    // ranks on distinct devices copy from each other's memory (LocalComm,
    // hipMemcpyPeerAsync): enable peer access both ways once per device pair
    // where the devices support it; elsewhere the runtime stages the copies
    // through host memory (slower, still correct)
    for (int a = 0; a < nranks; ++a)
      for (int b = 0; b < nranks; ++b) {
        if (devices[a] == devices[b]) continue;
        int can = 0;
        CFD_HIP(hipDeviceCanAccessPeer(&can, devices[a], devices[b]));
        if (!can) {
          std::fprintf(stderr, "cfd_group_create: device %d cannot access device %d; peer copies are staged\n",
                       devices[a], devices[b]);
          continue;
        }
        CFD_HIP(hipSetDevice(devices[a]));
        const hipError_t e = hipDeviceEnablePeerAccess(devices[b], 0);
        if (e == hipErrorPeerAccessAlreadyEnabled)
          (void)hipGetLastError();
        else
          CFD_HIP(e);
      }
    for (int r = 0; r < nranks; ++r) {
      auto comm = cfd2::make_local_comm(group, r, devices[r]);
      made.push_back(new cfd2::Solver(*mesh, c, devices[r], nranks > 1 ? std::move(comm) : nullptr));
    }
  });
  if (st != CFD_OK) {
    for (auto* p : made) delete p;
    return st;
  }
  for (int r = 0; r < nranks; ++r) out[r] = new cfd_solver{made[r]};
  return CFD_OK;
}

}  // extern "C"

namespace {
// a collective call on every rank of an in-process group, one host thread each.
// mutates: the call advances the solver state (a step).  If it fails on any
// rank, the ranks may have stopped at different points of it, so every rank is
// marked needs_restore and later mutating calls are refused until each rank is
// restored (cfd_state_load) or the group is explicitly reset (cfd_group_reset).
template <class F>
cfd_status group_run(cfd_solver* const* h, int32_t n, F&& f, bool mutates = false) {
  if (!h || n < 1) return set_error(CFD_ERR_INVALID, "bad argument");
  for (int r = 0; r < n; ++r) CHECK_S(h[r]);
  if (mutates)
    for (int r = 0; r < n; ++r)
      if (h[r]->s->needs_restore)
        return set_error(CFD_ERR_INVALID, "rank " + std::to_string(r) +
                                              ": group needs restore after a failed step (cfd_state_load on "
                                              "every rank, or cfd_group_reset)");
  std::vector<cfd_status> st(n, CFD_OK);
  std::vector<std::string> msg(n);
  std::vector<std::thread> th;
  for (int r = 0; r < n; ++r)
    th.emplace_back([&, r] {
      st[r] = guard([&] { f(*h[r]->s); });
      if (st[r] != CFD_OK) {
        msg[r] = cfd_last_error();
        // wake the ranks waiting for this one in a collective (they fail too);
        // a rank that was itself woken by an abort has nothing to add
        if (h[r]->s->comm && msg[r].find("group aborted") == std::string::npos) h[r]->s->comm->abort();
      }
    });
  for (auto& t : th) t.join();
  // every rank has returned: the group is usable again (LocalGroup::reset)
  if (h[0]->s->comm) h[0]->s->comm->reset();
  // report the first rank that failed on its own (the others fail with "aborted")
  int first = -1;
  for (int r = 0; r < n; ++r)
    if (st[r] != CFD_OK && (first < 0 || msg[first].find("group aborted") != std::string::npos)) first = r;
  if (first >= 0) {
    if (mutates)
      for (int r = 0; r < n; ++r) h[r]->s->needs_restore = true;
    return set_error(st[first], "rank " + std::to_string(first) + ": " + msg[first]);
  }
  return CFD_OK;
}
}  // namespace

extern "C" {

cfd_status cfd_group_step(cfd_solver* const* h, int32_t n) {
  return group_run(h, n, [](cfd2::Solver& s) { s.step(); }, true);
}

cfd_status cfd_group_reset(cfd_solver* const* h, int32_t n) {
  if (!h || n < 1) return set_error(CFD_ERR_INVALID, "bad argument");
  for (int r = 0; r < n; ++r) CHECK_S(h[r]);
  for (int r = 0; r < n; ++r) h[r]->s->needs_restore = false;
  return CFD_OK;
}

int32_t cfd_group_needs_restore(cfd_solver* const* h, int32_t n) {
  if (!h || n < 1) return 0;
  for (int r = 0; r < n; ++r)
    if (h[r] && h[r]->s && h[r]->s->needs_restore) return 1;
  return 0;
}

cfd_status cfd_group_state_save(cfd_solver* const* h, int32_t n, const char* path) {
  if (!path) return set_error(CFD_ERR_INVALID, "null path");
  // the ranks of a failed group step stopped at different points of it: a file
  // of that state would clear needs_restore on load (cfd_state_load) and the
  // group would continue from an inconsistent state
  if (cfd_group_needs_restore(h, n))
    return set_error(CFD_ERR_INVALID, "group state save refused: the group needs restore after a failed step "
                                      "(cfd_state_load on every rank, or cfd_group_reset)");
  return group_run(h, n, [path](cfd2::Solver& s) { s.save_state(path); });
}

cfd_status cfd_debug_comm_watchdog(float timeout_s, int32_t hang_ms) {
  return guard([&] {
    cfd2::Watchdog wd(0, -1, timeout_s, nullptr, nullptr);
    wd.host_begin("cfd_debug_comm_watchdog host wait", -1);
    std::this_thread::sleep_for(std::chrono::milliseconds(hang_ms > 0 ? hang_ms : 0));
    wd.host_end();
  });
}

// RCCL plumbing self-test on ONE GPU (RCCL refuses two ranks per device, so
// the multi-rank path cannot run on a one-GPU box): a 1-rank communicator,
// a grouped send/recv to self through Comm::exchange and an all-gather.
cfd_status cfd_debug_rccl_selftest(int32_t device) {
  return guard([&] {
    CFD_HIP(hipSetDevice(device));
    uint8_t uid[128];
    cfd2::rccl_unique_id(uid);
    auto comm = cfd2::make_rccl_comm(1, 0, uid);
    hipStream_t s;
    CFD_HIP(hipStreamCreate(&s));
    const size_t n = 4096;
    std::vector<float> h(n), back(2 * n, 0.0f);
    for (size_t i = 0; i < n; ++i) h[i] = (float)i * 0.5f;
    float *a, *b;
    CFD_HIP(hipMalloc(&a, n * sizeof(float)));
    CFD_HIP(hipMalloc(&b, 2 * n * sizeof(float)));
    CFD_HIP(hipMemcpyAsync(a, h.data(), n * sizeof(float), hipMemcpyHostToDevice, s));
    CFD_HIP(hipMemsetAsync(b, 0, 2 * n * sizeof(float), s));
    // two matched transfers to self: [0, n/2) -> b[n..], [n/2, n) -> b[n + n/2..]
    std::vector<cfd2::Msg> msgs = {{0, a, n / 2 * sizeof(float), b + n, n / 2 * sizeof(float)},
                                   {0, a + n / 2, n / 2 * sizeof(float), b + n + n / 2, n / 2 * sizeof(float)}};
    comm->exchange(msgs, s);
    comm->allgather(a, b, n * sizeof(float), s);
    CFD_HIP(hipMemcpyAsync(back.data(), b, 2 * n * sizeof(float), hipMemcpyDeviceToHost, s));
    CFD_HIP(hipStreamSynchronize(s));
    (void)hipFree(a);
    (void)hipFree(b);
    (void)hipStreamDestroy(s);
    for (size_t i = 0; i < n; ++i)
      if (back[i] != h[i] || back[n + i] != h[i]) throw std::runtime_error("RCCL self-test: wrong data");
  });
}

cfd_status cfd_dist_comm_stats(cfd_solver* s, cfd_comm_stats* out, int32_t reset) {
  CHECK_S(s);
  if (!out) return set_error(CFD_ERR_INVALID, "null out");
  std::memset(out, 0, sizeof(*out));
  out->device = s->s->device;
  out->comm_count = 1;
  auto& c = s->s->comm;
  if (c) {
    out->transport = c->kind;
    out->comm_count = c->comm_count();
    out->comm_rank = c->comm_rank();
    out->exchanges = c->stats.exchanges;
    out->allgathers = c->stats.allgathers;
    out->bytes_sent = c->stats.bytes_sent;
    out->bytes_gathered = c->stats.bytes_gathered;
    if (reset) c->stats = cfd2::CommStats{};
  }
  return CFD_OK;
}

cfd_status cfd_comm_timing_enable(cfd_solver* s, int32_t enable) {
  CHECK_S(s);
  return guard([&] {
    s->s->comm_prof_reset();
    s->s->comm_prof = enable != 0;
  });
}

cfd_status cfd_comm_timing(cfd_solver* s, cfd_comm_timing_entry* out, int32_t cap, int32_t* count) {
  CHECK_S(s);
  if (!count || (cap > 0 && !out)) return set_error(CFD_ERR_INVALID, "null argument");
  return guard([&] {
    cfd2::Solver& S = *s->s;
    S.comm_drain();
    int32_t k = 0;
    for (int c = 0; c < cfd2::Solver::kCommCats && k < cap; ++c) {
      const auto& t = S.comm_times[c];
      if (!t.calls) continue;
      cfd_comm_timing_entry& e = out[k++];
      e.category = std::min(c, (int)cfd2::Solver::kCommAmgHalo);
      e.level = c >= cfd2::Solver::kCommAmgHalo ? c - cfd2::Solver::kCommAmgHalo : -1;
      e.calls = t.calls;
      e.bytes = t.bytes;
      e.wait_us = 1e3 * t.wait_ms;
      e.comm_us = 1e3 * t.comm_ms;
    }
    *count = k;
  });
}

cfd_status cfd_debug_group_fault_midstep(cfd_solver* const* h, int32_t n, int32_t fail_rank) {
  return group_run(
      h, n,
      [fail_rank](cfd2::Solver& s) {
        s.debug_fault_after_prepare = fail_rank;
        s.step();
      },
      true);
}

cfd_status cfd_debug_group_fault(cfd_solver* const* h, int32_t n, int32_t fail_rank) {
  return group_run(h, n, [fail_rank](cfd2::Solver& s) {
    if (s.rk == fail_rank) throw std::runtime_error("injected fault");
    (void)s.allgather_u64(1);  // waits for the failed rank until the abort wakes it
  });
}

cfd_status cfd_dist_info(const cfd_solver* s, int32_t* rank, int32_t* nranks, uint32_t* c0, uint32_t* c1,
                         uint32_t* ng) {
  CHECK_S(s);
  if (rank) *rank = s->s->rk;
  if (nranks) *nranks = s->s->R;
  if (c0) *c0 = s->s->topo.c0;
  if (c1) *c1 = s->s->topo.c1;
  if (ng) *ng = s->s->NG;
  return CFD_OK;
}

cfd_status cfd_dist_plan(const cfd_mesh_view* mesh, int32_t nranks, int32_t rank, uint32_t* c0, uint32_t* c1,
                         uint32_t* num_ghosts, uint32_t* num_peers, uint32_t* num_send, uint32_t* ghost_global,
                         int32_t* peer_rank, uint32_t* peer_recv, uint32_t* peer_send, uint32_t* send_global) {
  if (!mesh) return set_error(CFD_ERR_INVALID, "null mesh");
  if (nranks < 1 || rank < 0 || rank >= nranks) return set_error(CFD_ERR_INVALID, "bad rank / nranks");
  return guard([&] {
    const auto starts = cfd2::partition_starts(mesh->num_cells, nranks);
    cfd2::Topology t;
    cfd2::build_topology(*mesh, t, (uint32_t)starts[rank], (uint32_t)starts[rank + 1]);
    const cfd2::HaloPlan P =
        cfd2::build_halo_plan(starts, rank, t.srow.data(), t.N, t.scol.data(), t.ghost, t.glo, t.npad);
    if (c0) *c0 = t.c0;
    if (c1) *c1 = t.c1;
    if (num_ghosts) *num_ghosts = (uint32_t)t.ghost.size();
    if (num_peers) *num_peers = (uint32_t)P.peers.size();
    if (num_send) *num_send = (uint32_t)P.send_idx.size();
    if (ghost_global) std::copy(t.ghost.begin(), t.ghost.end(), ghost_global);
    for (size_t k = 0; k < P.peers.size(); ++k) {
      if (peer_rank) peer_rank[k] = P.peers[k].rank;
      if (peer_recv) peer_recv[k] = P.peers[k].recv_cnt;
      if (peer_send) peer_send[k] = P.peers[k].send_cnt;
    }
    if (send_global)
      for (size_t k = 0; k < P.send_idx.size(); ++k) send_global[k] = t.c0 + (uint32_t)P.send_idx[k];
  });
}

}  // extern "C"
