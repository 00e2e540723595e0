// Host driver of the HIP coupled step: restates the control flow of
//   coupled_solver.rs:33-580            step_coupled / check_evolution
//   coupled_solver_fgmres.rs:1728-2448  solve_coupled_fgmres (FGMRES(50) + Schur)
//   linear_solver/amg.rs:666-770        v_cycle
//   solver.rs:9-44, 97-128, 276-294     set_u / set_p / set_dt / getters / history
// over the kernels of ../hip/kernels.hip, on one HIP stream.  All vectors stay
// in HBM; host round trips are the ones the reference control flow needs
// (blocking norms at solve start / restart, lagged residual reads), and none
// under the fixed benchmark schedule except the two early-exit norms.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <string>
#include <cstring>
#include <limits>

#include "solver_impl.hpp"

namespace cfd2 {

namespace {
// Rust's `{:.2e}` (the reference's log format): 1.23e-5, 3.40e38, NaN, inf
std::string e2(double v) {
  if (std::isnan(v)) return "NaN";
  if (std::isinf(v)) return v > 0 ? "inf" : "-inf";
  char buf[48];
  std::snprintf(buf, sizeof(buf), "%.2e", v);
  const std::string s(buf);
  const size_t e = s.find('e');
  size_t i = e + 1;
  const bool neg = s[i] == '-';
  if (s[i] == '-' || s[i] == '+') ++i;
  while (i + 1 < s.size() && s[i] == '0') ++i;
  return s.substr(0, e) + "e" + (neg ? "-" : "") + s.substr(i);
}
const char* tf(bool b) { return b ? "true" : "false"; }
// device scalars dsc[0..15]: rhs_norm, resid, inv_resid, wnorm, inv_w, resid_est
constexpr int kHOff = 16;
}  // namespace

template <class T>
T* Solver::valloc(int comps) {
  T* base = arena.alloc<T>(vlen * comps + 64);
  CFD_HIP(hipMemsetAsync(base, 0, (vlen * comps + 64) * sizeof(T), stream));
  return base + (size_t)shift * comps;
}

void Solver::make_plan_buffers(HaloPlan& p, int max_comps) {
  p.d_send_idx = arena.upload(p.send_idx, stream);
  p.max_comps = max_comps;
  p.d_stage = arena.alloc<float>(p.send_idx.size() * (size_t)max_comps + 1);
}

Solver::Solver(const cfd_mesh_view& mesh, const cfd_config& c, int dev, std::unique_ptr<Comm> cm)
    : cfg(c), device(dev) {
  if (cfg.max_restart < 1 || cfg.max_restart > 63) throw std::invalid_argument("max_restart must be 1..63");
  m = cfg.max_restart;
  m1 = m + 1;
  NG = mesh.num_cells;
  if (cm && cm->size > 1) {
    comm = std::move(cm);
    R = comm->size;
    rk = comm->rank;
  }
  starts = partition_starts(NG, R);
  build_topology(mesh, topo, (uint32_t)starts[rk], (uint32_t)starts[rk + 1]);
  N = topo.N;
  F = topo.F;
  red = red_geom(NG);
  if (red.nseg > kRedMaxSegments)
    throw std::invalid_argument("mesh too large for the reduction tree (at most 268 M cells)");
  nchunks = (N + kRedChunkCells - 1) / kRedChunkCells;
  nunits = (nchunks + red.U - 1) / red.U;
  pstride = (nunits + 3) & ~3u;
  shift = (topo.glo + 63) & ~63u;
  vlen = (size_t)shift + topo.npad + topo.ghi;
  CFD_HIP(hipSetDevice(device));
  lds_budget = init_kernel_attributes(device);
  amg_wide_limit = (int)std::max<uint64_t>(1, std::min<uint64_t>(255, knob_u64(Knob::AmgWideLimit, 255)));
  check_sync = cfg.log_level >= 3;  // debug: synchronise and check after every launch
  small_forms = knob_on(Knob::SmallMeshForms);
  nt_mask = (unsigned)knob_u64(Knob::Nt, nt_mask);
  // C1-size meshes: 64 MB of the dots pass kept in the Infinity Cache for a
  // top-down update (profiles/r04/ab_cgskeep2_c1.txt: update 36.5-36.9 ->
  // 32.3 us, dots +0.3 us per iteration); from 2^22 cells on the kept lines
  // cost more than they return (ab_cgskeep_c2.txt: dots 284 -> 293 us)
  cgs_keep_bytes = N < (1u << 22) ? (size_t)64 << 20 : 0;  // (kernels.hip CFD_CGS_SER_MIN_CELLS)
  CFD_HIP(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
  amg_local = dist() && cfg.amg_local_aggregation != 0;
  // hipGraph replay: opt-in through cfd_graph_enable (replay measured no faster
  // than eager launches on this pool, profiles/r05/ab_graph_c0_c1.txt: C0
  // 13.36-13.47 vs 13.30-13.51 ms/step, C1 39.6-39.9 vs 38.8-39.1); halo
  // exchanges and collectives stay eager
  graph_on = false;
  if (dist()) {
    overlap_min_rows = (uint32_t)knob_u64(Knob::OverlapMinRows, overlap_min_rows);
    CFD_HIP(hipStreamCreateWithFlags(&cstream, hipStreamNonBlocking));
    CFD_HIP(hipEventCreateWithFlags(&hev_pack, hipEventDisableTiming));
    CFD_HIP(hipEventCreateWithFlags(&hev_done, hipEventDisableTiming));
    cell_plan = build_halo_plan(starts, rk, topo.srow.data(), N, topo.scol.data(), topo.ghost, topo.glo,
                                topo.npad);
    make_plan_buffers(cell_plan, 8);
    // segments of every rank (ranks own whole segments: partition_starts)
    std::vector<uint32_t> src(red.nseg);
    for (int q = 0; q < R; ++q) {
      const uint64_t s0 = starts[q] / red.seg_cells;
      const uint64_t s1 = (starts[q + 1] + red.seg_cells - 1) / red.seg_cells;
      maxseg = std::max(maxseg, (uint32_t)(s1 - s0));
      for (uint64_t sg = s0; sg < s1; ++sg) src[sg] = ((uint32_t)q << 20) | (uint32_t)(sg - s0);
    }
    if (maxseg >= (1u << 20) || R >= (1 << 12)) throw std::invalid_argument("too many segments / ranks");
    d_seg_src = arena.upload(src, stream);
    red_local = arena.alloc<float>((size_t)m1 * maxseg);
    red_gather = arena.alloc<float>((size_t)R * m1 * maxseg);
    red_local_d = arena.alloc<double>((size_t)5 * maxseg);
    red_gather_d = arena.alloc<double>((size_t)R * 5 * maxseg);
    mx_gather = arena.alloc<uint32_t>(2 * (size_t)R);
    d_u64 = arena.alloc<uint64_t>((size_t)R + 1);  // not lazily: the AMG build runs on amg_arena
    // check_evolution's stride bug reads records (i >> 2) of the global state
    ev_a = (uint64_t)topo.c0 >> 2;
    ev_b = (((uint64_t)topo.c1 - 1) >> 2) + 1;
    const size_t ne = ev_b - ev_a;
    evrec.u = arena.alloc<float2>(ne);
    evrec.p = arena.alloc<float>(ne);
    evrec.dp = arena.alloc<float>(ne);
    evrec.gp = arena.alloc<float2>(ne);
  }
  // static mesh data
  d_vol = arena.upload(topo.vol, stream);
  fs.other = arena.upload(topo.fs_other, stream);
  fs.meta = arena.upload(topo.fs_meta, stream);
  fs.area = arena.upload(topo.fs_area, stream);
  fs.nx = arena.upload(topo.fs_nx, stream);
  fs.ny = arena.upload(topo.fs_ny, stream);
  fs.lam_s = arena.upload(topo.fs_lam_s, stream);
  fs.lam_f = arena.upload(topo.fs_lam_f, stream);
  fs.dist_a = arena.upload(topo.fs_dist_a, stream);
  fs.dist_e = arena.upload(topo.fs_dist_e, stream);
  fs.dvx = arena.upload(topo.fs_dvx, stream);
  fs.dvy = arena.upload(topo.fs_dvy, stream);
  fs.rx = arena.upload(topo.fs_rx, stream);
  fs.ry = arena.upload(topo.fs_ry, stream);
  fs.rox = arena.upload(topo.fs_rox, stream);
  fs.roy = arena.upload(topo.fs_roy, stream);
  fs.nface = arena.upload(topo.nface, stream);
  fs.wf = topo.wf;
  d_scol = arena.upload(topo.ell_col, stream);
  d_slen = arena.upload(topo.ell_len, stream);
  d_sdrank = arena.upload(topo.ell_drank, stream);
  if (topo.use16) d_scol16 = arena.upload(topo.ell_col16, stream);
  d_slen8 = arena.upload(topo.ell_len8, stream);
  d_sdrank8 = arena.upload(topo.ell_drank8, stream);
  if (topo.use16)
    d_tcol16 = arena.upload(topo.tcol16, stream);
  else
    d_tcol = arena.upload(topo.tcol, stream);
  d_tlg = arena.upload(topo.tlg, stream);
  d_tdrank8 = arena.upload(topo.tdrank8, stream);
  // fields (init/fields.rs:62-139): zero-initialised, with ghost space
  auto zeros_state = [&](StateView& v) {
    v.u = valloc<float2>(1);
    v.p = valloc<float>(1);
    v.dp = valloc<float>(1);
    v.gp = valloc<float2>(1);
  };
  for (auto& r : ring) zeros_state(r);
  zeros_state(prev);
  dp_scratch = valloc<float>(1);
  gp_scratch = valloc<float2>(1);
  const size_t slots_f = (size_t)topo.wf * N, slots_s = (size_t)topo.ws * topo.ld;
  flux_s = arena.alloc<float>(slots_f);
  CFD_HIP(hipMemsetAsync(flux_s, 0, slots_f * sizeof(float), stream));
  grad_u = valloc<float2>(1);
  grad_v = valloc<float2>(1);
  cval_a = arena.alloc<float2>(slots_s);
  cval_g = arena.alloc<float2>(slots_s);
  CFD_HIP(hipMemsetAsync(cval_a, 0, slots_s * sizeof(float2), stream));
  CFD_HIP(hipMemsetAsync(cval_g, 0, slots_s * sizeof(float2), stream));
  cdiag2 = arena.alloc<float2>(topo.ld);
  CFD_HIP(hipMemsetAsync(cdiag2, 0, topo.ld * sizeof(float2), stream));
  sval = arena.alloc<float>(slots_s);
  CFD_HIP(hipMemsetAsync(sval, 0, slots_s * sizeof(float), stream));
  rhs = valloc<float>(3);
  x = valloc<float>(3);
  dinv_uv = valloc<float>(1);
  dinv_p = valloc<float>(1);
  partial_d = arena.alloc<double>(5 * (size_t)pstride + 5);
  maxbits = arena.alloc<uint32_t>(4);
  blockmax = arena.alloc<uint32_t>(2 * (((size_t)N + 255) / 256) + 2);
  // pinned, mapped (for every device: portable) and coherent: kernels may store
  // the per-iteration residual into it directly (d_pin, the device view),
  // visible to the host after the event
  CFD_HIP(hipHostMalloc((void**)&h_pin, 4096 * sizeof(float),
                        hipHostMallocMapped | hipHostMallocCoherent | hipHostMallocPortable));
  CFD_HIP(hipHostGetDevicePointer((void**)&d_pin, h_pin, 0));
  for (auto& e : ev_outer) CFD_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  // constants (init/fields.rs:100-115)
  constants.dt = 0.0001f;
  constants.dt_old = 0.0001f;
  constants.time = 0.0f;
  constants.viscosity = 0.01f;
  constants.density = 1.0f;
  constants.component = 0;
  constants.alpha_p = 1.0f;
  constants.scheme = 0;
  constants.alpha_u = 0.7f;
  constants.stride_x = 65535u * 64u;
  constants.time_scheme = 0;
  constants.inlet_velocity = 1.0f;
  constants.ramp_time = 0.1f;
  constants.precond_type = 0;
  std::memset(&info, 0, sizeof(info));
  sync();
}

Solver::~Solver() {
  if (stream) (void)hipStreamSynchronize(stream);
  for (IterGraph& G : graphs) {
    if (G.exec) (void)hipGraphExecDestroy(G.exec);
    for (auto e : G.ev) (void)hipEventDestroy(e);
  }
  for (auto e : ev_iter) (void)hipEventDestroy(e);
  for (auto e : ev_outer)
    if (e) (void)hipEventDestroy(e);
  for (auto e : prof_ev) (void)hipEventDestroy(e);
  if (cstream) (void)hipStreamSynchronize(cstream);
  for (auto e : comm_ev_pool) (void)hipEventDestroy(e);
  if (h_pin) (void)hipHostFree(h_pin);
  if (cstream) (void)hipStreamSynchronize(cstream);
  if (hev_pack) (void)hipEventDestroy(hev_pack);
  if (hev_done) (void)hipEventDestroy(hev_done);
  comm.reset();
  arena.release();
  amg_arena.release();
  if (cstream) (void)hipStreamDestroy(cstream);
  if (stream) (void)hipStreamDestroy(stream);
}

CoupledMatrix Solver::cmat() const {
  CoupledMatrix A;
  A.N = N;
  A.r0 = 0;
  A.r1 = N;
  A.r2 = A.r3 = 0;
  A.ld = topo.ld;
  A.ws = topo.ws;
  A.use16 = topo.use16 ? 1 : 0;
  A.col = d_tcol;
  A.col16 = d_tcol16;
  A.lg = d_tlg;
  A.drank = d_tdrank8;
  A.cval_a = cval_a;
  A.cval_g = cval_g;
  A.cdiag2 = cdiag2;
  A.reg = !topo.tmode.empty() && topo.ws <= kCoupledRegMaxWs ? 1 : 0;
  for (int r = 0; r < 8; ++r) A.tmode[r] = r < (int)topo.tmode.size() ? topo.tmode[r] : 0;
  return A;
}

void Solver::log(const char* fmt, ...) const {
  if (cfg.log_level < 1 || rk != 0) return;
  va_list ap;
  va_start(ap, fmt);
  std::vfprintf(stderr, fmt, ap);
  va_end(ap);
}

// ---------------------------------------------------------------- state API
// set_u / set_p take the GLOBAL per-cell arrays; a distributed rank keeps its
// owned cells and ghosts.  Getters return the owned cells.
void Solver::set_u(const double* uv) {  // solver.rs:9-21 (clobbers the whole state)
  CFD_HIP(hipSetDevice(device));
  std::vector<float> img;
  local_image(uv, 2, img);
  StateView& s = S();
  CFD_HIP(hipMemcpyAsync(vbase(s.u, 1), img.data(), vlen * sizeof(float2), hipMemcpyHostToDevice, stream));
  CFD_HIP(hipMemsetAsync(vbase(s.p, 1), 0, vlen * sizeof(float), stream));
  CFD_HIP(hipMemsetAsync(vbase(s.dp, 1), 0, vlen * sizeof(float), stream));
  CFD_HIP(hipMemsetAsync(vbase(s.gp, 1), 0, vlen * sizeof(float2), stream));
  sync();
}

void Solver::set_p(const double* pv) {  // solver.rs:23-34
  CFD_HIP(hipSetDevice(device));
  std::vector<float> img;
  local_image(pv, 1, img);
  StateView& s = S();
  CFD_HIP(hipMemsetAsync(vbase(s.u, 1), 0, vlen * sizeof(float2), stream));
  CFD_HIP(hipMemcpyAsync(vbase(s.p, 1), img.data(), vlen * sizeof(float), hipMemcpyHostToDevice, stream));
  CFD_HIP(hipMemsetAsync(vbase(s.dp, 1), 0, vlen * sizeof(float), stream));
  CFD_HIP(hipMemsetAsync(vbase(s.gp, 1), 0, vlen * sizeof(float2), stream));
  sync();
}

namespace {
void copy_state(const StateView& src, StateView& dst, size_t off, size_t n, hipStream_t s) {
  CFD_HIP(hipMemcpyAsync(dst.u - off, src.u - off, n * sizeof(float2), hipMemcpyDeviceToDevice, s));
  CFD_HIP(hipMemcpyAsync(dst.p - off, src.p - off, n * sizeof(float), hipMemcpyDeviceToDevice, s));
  CFD_HIP(hipMemcpyAsync(dst.dp - off, src.dp - off, n * sizeof(float), hipMemcpyDeviceToDevice, s));
  CFD_HIP(hipMemcpyAsync(dst.gp - off, src.gp - off, n * sizeof(float2), hipMemcpyDeviceToDevice, s));
}
}  // namespace

void Solver::initialize_history() {  // solver.rs:276-294
  CFD_HIP(hipSetDevice(device));
  copy_state(ring[i_state], ring[i_old], shift, vlen, stream);
  copy_state(ring[i_state], ring[i_old_old], shift, vlen, stream);
  sync();
}

void Solver::get_u(double* uv) {
  CFD_HIP(hipSetDevice(device));
  std::vector<float2> u(N);
  CFD_HIP(hipMemcpyAsync(u.data(), S().u, N * sizeof(float2), hipMemcpyDeviceToHost, stream));
  sync();
  for (uint32_t i = 0; i < N; ++i) {
    uv[2 * i] = u[i].x;
    uv[2 * i + 1] = u[i].y;
  }
}

void Solver::get_p(double* out) {
  CFD_HIP(hipSetDevice(device));
  std::vector<float> p(N);
  CFD_HIP(hipMemcpyAsync(p.data(), S().p, N * sizeof(float), hipMemcpyDeviceToHost, stream));
  sync();
  for (uint32_t i = 0; i < N; ++i) out[i] = p[i];
}

void Solver::get_d_p(double* out) {
  CFD_HIP(hipSetDevice(device));
  std::vector<float> p(N);
  CFD_HIP(hipMemcpyAsync(p.data(), S().dp, N * sizeof(float), hipMemcpyDeviceToHost, stream));
  sync();
  for (uint32_t i = 0; i < N; ++i) out[i] = p[i];
}

// ------------------------------------------------------------ distribution
// Halo exchange of per-cell fields over `plan`: pack the rows the peers need,
// then one grouped transfer per (peer, field) straight into the ghost slots.
void Solver::halo(HaloPlan& plan, std::initializer_list<HField> fields) {
  if (!dist()) return;
  halo_begin(plan, fields);
  halo_end();
}

void Solver::halo_end() {
  if (!comm_prof) {
    CFD_HIP(hipStreamWaitEvent(stream, hev_done, 0));
    return;
  }
  // the compute stream's stall on the exchange: from reaching the wait to its release
  hipEvent_t a = comm_event(), b = comm_event();
  CFD_HIP(hipEventRecord(a, stream));
  CFD_HIP(hipStreamWaitEvent(stream, hev_done, 0));
  CFD_HIP(hipEventRecord(b, stream));
  comm_recs.push_back({halo_cat, 0, a, b});
}

// The pool grows for as long as comm_prof is on: a drain (both streams
// synchronised) inside the timed step would stall it and shift the waits
// measured after it (a C4 step records ~18 k events).  The pool
// is folded and reused only by comm_drain() (cfd_comm_timing, enable/disable).
hipEvent_t Solver::comm_event() {
  if (comm_ev_used == comm_ev_pool.size()) {
    for (int k = 0; k < 1024; ++k) {
      hipEvent_t e;
      CFD_HIP(hipEventCreate(&e));
      comm_ev_pool.push_back(e);
    }
  }
  return comm_ev_pool[comm_ev_used++];
}

void Solver::comm_drain() {
  if (comm_recs.empty()) return;
  CFD_HIP(hipStreamSynchronize(stream));
  if (cstream) CFD_HIP(hipStreamSynchronize(cstream));
  for (const CommRec& r : comm_recs) {
    float ms = 0.0f;
    CFD_HIP(hipEventElapsedTime(&ms, r.a, r.b));
    CommTimes& t = comm_times[r.cat];
    if (r.kind == 0 || r.kind == 2) t.wait_ms += ms;
    if (r.kind == 1 || r.kind == 2) t.comm_ms += ms;
  }
  comm_recs.clear();
  comm_ev_used = 0;
}

void Solver::comm_prof_reset() {
  comm_drain();
  for (CommTimes& t : comm_times) t = CommTimes{};
}

void Solver::halo_begin(HaloPlan& plan, std::initializer_list<HField> fields) {
  const uint32_t ns = (uint32_t)plan.send_idx.size();
  PackArgs pa{};
  int tot = 0;
  for (const HField& f : fields) {
    if (pa.nf == 8) throw std::logic_error("halo: too many fields");
    pa.f[pa.nf++] = PackField{f.ptr, f.comps, (uint32_t)((size_t)ns * tot)};
    tot += f.comps;
  }
  if (tot > plan.max_comps) throw std::logic_error("halo: stage buffer too small");
  pa.idx = plan.d_send_idx;
  pa.n = ns;
  pa.stage = plan.d_stage;
  if (!plan.all_direct) launch_pack(pa, stream);
  std::vector<Msg> msgs;
  for (const HaloPeer& h : plan.peers) {
    for (int f = 0; f < pa.nf; ++f) {
      const PackField& F = pa.f[f];
      Msg mm;
      mm.peer = h.rank;
      mm.sbuf = plan.all_direct ? F.src + (ptrdiff_t)h.direct * F.comps
                                : plan.d_stage + F.stage_off + (size_t)h.send_off * F.comps;
      mm.sbytes = (size_t)h.send_cnt * F.comps * sizeof(float);
      mm.rbuf = const_cast<float*>(F.src) + (ptrdiff_t)h.recv_rel * F.comps;
      mm.rbytes = (size_t)h.recv_cnt * F.comps * sizeof(float);
      msgs.push_back(mm);
    }
  }
  CFD_HIP(hipEventRecord(hev_pack, stream));
  CFD_HIP(hipStreamWaitEvent(cstream, hev_pack, 0));
  halo_cat = comm_cat;
  comm->label = halo_cat;
  if (comm_prof) {
    hipEvent_t a = comm_event(), b = comm_event();
    CFD_HIP(hipEventRecord(a, cstream));
    comm->exchange(msgs, cstream);
    CFD_HIP(hipEventRecord(b, cstream));
    comm_recs.push_back({halo_cat, 1, a, b});
    CommTimes& t = comm_times[halo_cat];
    t.calls++;
    for (const Msg& mm : msgs) t.bytes += mm.sbytes;
  } else {
    comm->exchange(msgs, cstream);
  }
  CFD_HIP(hipEventRecord(hev_done, cstream));
}

// ghosts of the current FluidState slot: u, p (all = also d_p, grad_p)
void Solver::halo_state(bool all) {
  StateView& s = S();
  if (all)
    halo(cell_plan, {{(float*)s.u, 2}, {s.p, 1}, {s.dp, 1}, {(float*)s.gp, 2}});
  else
    halo(cell_plan, {{(float*)s.u, 2}, {s.p, 1}});
}

// Canonical reductions (kernels.hpp): one GPU hands the chunk partials to the
// finishing kernel; a distributed rank reduces its own segments, all-gathers
// the segment values, and every rank finishes the same global tree.
RedSrc Solver::combine(const float* part, int nvec) {
  RedSrc r;
  r.G = red.G / red.U;  // units per segment
  r.nseg = red.nseg;
  r.nvec = (uint32_t)nvec;
  if (!dist()) {
    r.p = part;
    r.stride = pstride;
    r.nchunks = nunits;
    return r;
  }
  launch_seg_reduce(part, pstride, nunits, r.G, nvec, red_local, maxseg, stream);
  const size_t bytes = (size_t)nvec * maxseg * sizeof(float);
  timed_gather(kCommReduceGather, bytes, [&] { comm->allgather(red_local, red_gather, bytes, stream); });
  r.p = red_gather;
  r.stride = maxseg;
  r.seg_src = d_seg_src;
  return r;
}

RedSrcD Solver::combine_d(const double* part, int nvec) {
  RedSrcD r;
  r.G = red.G / red.U;  // units per segment
  r.nseg = red.nseg;
  r.nvec = (uint32_t)nvec;
  if (!dist()) {
    r.p = part;
    r.stride = pstride;
    r.nchunks = nunits;
    return r;
  }
  launch_seg_reduce_d(part, pstride, nunits, r.G, nvec, red_local_d, maxseg, stream);
  const size_t bytes = (size_t)nvec * maxseg * sizeof(double);
  timed_gather(kCommReduceGather, bytes, [&] { comm->allgather(red_local_d, red_gather_d, bytes, stream); });
  r.p = red_gather_d;
  r.stride = maxseg;
  r.seg_src = d_seg_src;
  return r;
}

// ------------------------------------------------------------------ kernels
void Solver::rotate() {  // coupled_solver.rs:43-71
  step_index = (step_index + 1) % 3;
  static const int tab[3][3] = {{0, 1, 2}, {2, 0, 1}, {1, 2, 0}};
  i_state = tab[step_index][0];
  i_old = tab[step_index][1];
  i_old_old = tab[step_index][2];
}

void Solver::prepare() {
  PrepareArgs a;
  a.N = N;
  a.c = constants;
  a.fs = fs;
  a.vol = d_vol;
  a.st = S();
  a.dp_out = dp_scratch;
  a.gp_out = gp_scratch;
  a.flux_s = flux_s;
  a.grad_u = grad_u;
  a.grad_v = grad_v;
  if (ref_racy) {  // test mode: in place, workgroups in order, the owners' fluxes
    a.dp_out = S().dp;
    a.gp_out = S().gp;
    launch_prepare_ordered(a, d_flux_mirror, (uint32_t)((size_t)topo.wf * N), stream);
    check_launch("prepare (reference semantics)");
    return;
  }
  launch_prepare(a, stream);
  check_launch("prepare");
  // commit d_p / grad_p (snapshot semantics): swap the scratch into the slot
  std::swap(S().dp, dp_scratch);
  std::swap(S().gp, gp_scratch);
  if (dist())  // assemble reads the neighbours' new d_p (and gradients for SOU/QUICK)
    halo(cell_plan, {{S().dp, 1}, {(float*)S().gp, 2}, {(float*)grad_u, 2}, {(float*)grad_v, 2}});
}

void Solver::assemble() {
  AssembleArgs a;
  a.N = N;
  a.ld = topo.ld;
  a.c = constants;
  a.fs = fs;
  a.vol = d_vol;
  a.st = S();
  a.u_old = ring[i_old].u;
  a.u_old_old = ring[i_old_old].u;
  a.flux_s = flux_s;
  a.grad_u = grad_u;
  a.grad_v = grad_v;
  a.srank_diag = d_sdrank;
  a.cslot_diag = d_tdrank8;
  a.cval_a = cval_a;
  a.cval_g = cval_g;
  a.cdiag2 = cdiag2;
  a.sval = sval;
  a.rhs = rhs;
  a.dinv_uv = dinv_uv;
  a.dinv_p = dinv_p;
  launch_assemble(a, stream);
  check_launch("assemble");
  if (dist()) halo(cell_plan, {{dinv_uv, 1}});  // the Schur prediction reads neighbours' D_u^-1
}

void Solver::ensure_fgmres() {  // coupled_solver_fgmres.rs:212-1280 (lazy)
  if (fgmres_ready) return;
  // Krylov vectors in the per-cell layout (ghost space: V_j and Z_j are read at
  // neighbours by the Schur prediction and the SpMV); 256-byte aligned slots
  stride = (3 * vlen + 63) & ~(size_t)63;
  float* braw = arena.alloc<float>((size_t)m1 * stride + 64);
  float* zraw = arena.alloc<float>((size_t)m * stride + 64);
  CFD_HIP(hipMemsetAsync(braw, 0, ((size_t)m1 * stride + 64) * sizeof(float), stream));
  CFD_HIP(hipMemsetAsync(zraw, 0, ((size_t)m * stride + 64) * sizeof(float), stream));
  basis = braw + 3 * (size_t)shift;
  zvec = zraw + 3 * (size_t)shift;
  w = valloc<float>(3);
  // pressure vectors: padded to a multiple of 64 owned rows (the AMG level-0
  // kernels process 4 rows per thread with 16-byte loads), plus ghosts
  temp = valloc<float>(1);
  temp_p = valloc<float>(1);
  p_sol = valloc<float>(1);
  partial = arena.alloc<float>((size_t)m1 * pstride);
  partial_n = arena.alloc<float>(pstride);
  const size_t nsc = kHOff + (size_t)m1 * m + 2 * (size_t)m + m1 + m + m + m1;
  dsc = arena.alloc<float>(nsc);
  CFD_HIP(hipMemsetAsync(dsc, 0, nsc * sizeof(float), stream));
  H = dsc + kHOff;
  givens = H + (size_t)m1 * m;
  g = givens + 2 * m;
  y = g + m1;
  resid_hist = y + m;
  binv = resid_hist + m;
  ev_iter.resize(2);  // the two pinned residual slots (Solver::solve)
  for (auto& e : ev_iter) CFD_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  fgmres_ready = true;
}

namespace {

// Device image of rows [r0, r0 + n) of the level matrix A (global numbering),
// off-diagonal columns mapped to local indices by `rel`; see AmgLevelDev.
template <class Rel>
void level_image(const HostCsr& A, uint64_t r0, uint32_t n, Rel rel, AmgGpuLevel& G, DeviceArena& arena,
                 hipStream_t stream, int wide_limit) {
  const uint32_t st = (n + 63) & ~63u;  // padded row count (16-byte row groups)
  int wmax = 0;
  bool small_delta = true;
  std::vector<uint8_t> len(st, 0), drank(st, 0);
  std::vector<uint16_t> len16(st, 0), drank16(st, 0);
  std::vector<float> dv(st, 0.0f), de(st, 1.0f);
  uint64_t nnz = 0;
  for (uint32_t i = 0; i < n; ++i) {
    const uint64_t gi = r0 + i;
    uint32_t off = 0, dr = 0;
    bool has = false;
    float diag = 1.0f, raw = 0.0f;
    for (uint32_t k = A.row[gi]; k < A.row[gi + 1]; ++k) {
      const uint32_t c = A.col[k];
      if (c == gi) {
        has = true;
        raw = A.val[k];
        diag = raw;
        dr = off;
      } else {
        ++off;
        const int64_t d = (int64_t)rel(c) - (int64_t)i;
        if (d < -32768 || d > 32767) small_delta = false;
      }
    }
    nnz += A.row[gi + 1] - A.row[gi];
    if (!has) dr = off;  // no diagonal entry: raw diag contributes nothing (dv = 0)
    if (std::fabs(diag) < 1e-14f) diag = 1.0f;  // amg.wgsl:46
    if (off > 65535) throw std::invalid_argument("AMG level row wider than 65535 entries (unsupported)");
    len[i] = (uint8_t)std::min(off, 255u);
    drank[i] = (uint8_t)std::min(dr, 255u);
    len16[i] = (uint16_t)off;
    drank16[i] = (uint16_t)dr;
    dv[i] = raw;
    de[i] = diag;
    wmax = std::max(wmax, (int)off);
  }
  const size_t slots = (size_t)std::max(wmax, 1) * st;
  std::vector<float> val(slots, 0.0f);
  std::vector<int16_t> col16(small_delta ? slots : 0, 0);
  std::vector<int32_t> col32(small_delta ? 0 : slots, 0);
  for (uint32_t i = 0; i < st; ++i) {
    uint32_t r = 0;
    if (i < n) {
      const uint64_t gi = r0 + i;
      for (uint32_t k = A.row[gi]; k < A.row[gi + 1]; ++k) {
        const uint32_t c = A.col[k];
        if (c == gi) continue;
        const size_t o = (size_t)r * st + i;
        val[o] = A.val[k];
        if (small_delta)
          col16[o] = (int16_t)((int64_t)rel(c) - (int64_t)i);
        else
          col32[o] = rel(c);
        ++r;
      }
    }
    // padding slots / rows: value 0, column = the row itself (allocated, zeroed)
    if (!small_delta)
      for (; r < (uint32_t)std::max(wmax, 1); ++r) col32[(size_t)r * st + i] = (int32_t)i;
  }
  G.nnz = nnz;
  G.dev.n = n;
  G.dev.r0 = 0;
  G.dev.r1 = n;
  G.dev.stride = st;
  G.dev.w = wmax;
  G.dev.use16 = small_delta ? 1 : 0;
  G.dev.val = arena.upload(val, stream);
  G.dev.col16 = small_delta ? arena.upload(col16, stream) : nullptr;
  G.dev.col32 = small_delta ? nullptr : arena.upload(col32, stream);
  G.dev.len = arena.upload(len, stream);
  G.dev.drank = arena.upload(drank, stream);
  G.dev.dv = arena.upload(dv, stream);
  G.dev.de = arena.upload(de, stream);
  G.wide = wmax > wide_limit;
  G.dev.len16 = G.wide ? arena.upload(len16, stream) : nullptr;
  G.dev.drank16 = G.wide ? arena.upload(drank16, stream) : nullptr;
}

}  // namespace

// ensure_amg_resources (coupled_solver_fgmres.rs:174-209): read back the live
// scalar matrix, build the frozen hierarchy on the host, upload it.  A
// distributed rank all-gathers the scalar matrix, builds the GLOBAL hierarchy
// (the one a single GPU builds, so results do not depend on the rank count)
// and keeps its rows of the levels with more than CFD_AMG_REPLICATE_ROWS rows
// (default kAmgReplicateRowsDefault); the small levels are replicated on every rank.
// Unconditional slot loads (kernels.hip gather_group) on level 0 (the face
// stencil: rows fill the ELL width) and on latency-bound small levels;
// predicated loads on the big coarse levels, whose row lengths vary (same-box
// A/B at C2: level 1 smoother 58 vs 66 us, small-level residual 6 vs 8.5 us).
std::vector<uint64_t> Solver::allgather_u64(uint64_t mine) {
  std::vector<uint64_t> all(R, mine);
  if (!dist()) return all;
  if (!d_u64) d_u64 = arena.alloc<uint64_t>((size_t)R + 1);
  CFD_HIP(hipMemcpyAsync(d_u64, &mine, sizeof(uint64_t), hipMemcpyHostToDevice, stream));
  comm->allgather(d_u64, d_u64 + 1, sizeof(uint64_t), stream);
  CFD_HIP(hipMemcpyAsync(all.data(), d_u64 + 1, (size_t)R * sizeof(uint64_t), hipMemcpyDeviceToHost, stream));
  sync();
  return all;
}

// Unconditional slot loads + vector gathers (MODE 1) where the rows fill the
// ELL width (level 0; the first coarse levels of the face-stencil meshes: mean
// off-diagonal count >= 3/4 of the width; C2 A/B: level-1 smoother 55.0 ->
// 50.2 us, level 2 15.1 -> 12.3) and on the small latency-bound levels;
// predicated loads on ragged big levels.
void Solver::set_amg_full_policy(AmgGpuLevel& G, int li) {
  const char* fe = knob(Knob::AmgFull);
  const double n = std::max<double>(G.dev.n, 1.0);
  const double offd = ((double)G.nnz - n) / n;  // mean off-diagonals per row
  const bool regular = G.dev.w > 0 && offd >= 0.75 * G.dev.w;
  G.dev.full = fe ? (fe[0] == '1') : (li == 0 || regular || G.dev.n <= (1u << 19));
}

// Host AMG setup (amg_setup.cpp): the assembled scalar matrix is downloaded,
// the whole hierarchy is built on the host and every level image uploaded
// (fallback of build_amg_device, or CFD_AMG_SETUP=host).
void Solver::build_amg_host() {
  const size_t ld = topo.ld;
  std::vector<float> ell((size_t)topo.ws * ld);
  CFD_HIP(hipMemcpyAsync(ell.data(), sval, ell.size() * sizeof(float), hipMemcpyDeviceToHost, stream));
  sync();
  std::vector<float> own(topo.scol.size());
  for (uint32_t i = 0; i < N; ++i)
    for (uint32_t k = topo.srow[i]; k < topo.srow[i + 1]; ++k) own[k] = ell[(size_t)(k - topo.srow[i]) * ld + i];
  HostCsr A0;
  std::vector<AmgHostLevel> H;
  if (!dist()) {
    A0.rows = A0.cols = N;
    A0.row = topo.srow;
    A0.col = topo.scol;
    A0.val = std::move(own);
    H = build_amg_hierarchy(A0, kMaxAmgLevels, {}, false, 0, cfg.log_level >= 2);
  } else {
    // all-gather the global pattern and the values (row order = global order, rank by rank)
    const std::vector<uint64_t> nz = allgather_u64(topo.scol.size());
    std::vector<uint64_t> eoff(R + 1, 0);
    for (int q = 0; q < R; ++q) eoff[q + 1] = eoff[q] + nz[q];
    std::vector<size_t> roff(R + 1), coff(R + 1);
    for (int q = 0; q <= R; ++q) {
      roff[q] = starts[q] * sizeof(uint32_t);
      coff[q] = eoff[q] * sizeof(uint32_t);
    }
    const size_t nnz_all = eoff[R];
    std::vector<uint32_t> lens(NG, 0);
    for (uint32_t i = 0; i < N; ++i) lens[starts[rk] + i] = topo.srow[i + 1] - topo.srow[i];
    uint32_t* d_lens = arena.alloc<uint32_t>(NG);
    uint32_t* d_cols = arena.alloc<uint32_t>(nnz_all);
    float* d_vals = arena.alloc<float>(nnz_all);
    CFD_HIP(hipMemcpyAsync(d_lens, lens.data(), (size_t)NG * 4, hipMemcpyHostToDevice, stream));
    CFD_HIP(hipMemcpyAsync(d_cols + eoff[rk], topo.scol.data(), topo.scol.size() * 4, hipMemcpyHostToDevice, stream));
    CFD_HIP(hipMemcpyAsync(d_vals + eoff[rk], own.data(), own.size() * 4, hipMemcpyHostToDevice, stream));
    comm->allgatherv_inplace(d_lens, roff, stream);
    comm->allgatherv_inplace(d_cols, coff, stream);
    comm->allgatherv_inplace(d_vals, coff, stream);
    A0.rows = A0.cols = NG;
    A0.row.assign((size_t)NG + 1, 0);
    A0.col.resize(nnz_all);
    A0.val.resize(nnz_all);
    CFD_HIP(hipMemcpyAsync(lens.data(), d_lens, (size_t)NG * 4, hipMemcpyDeviceToHost, stream));
    CFD_HIP(hipMemcpyAsync(A0.col.data(), d_cols, nnz_all * 4, hipMemcpyDeviceToHost, stream));
    CFD_HIP(hipMemcpyAsync(A0.val.data(), d_vals, nnz_all * 4, hipMemcpyDeviceToHost, stream));
    sync();
    for (uint32_t i = 0; i < NG; ++i) A0.row[i + 1] = A0.row[i] + lens[i];
    H = build_amg_hierarchy(A0, kMaxAmgLevels, starts, amg_local, amg_replicate_rows(), cfg.log_level >= 2 && rk == 0);
  }
  const int L = (int)H.size();
  // distributed levels [0, amg_g): the rest are replicated (all of them on one GPU)
  amg_g = 0;
  if (dist()) {
    const uint64_t rep = amg_replicate_rows();
    amg_g = L;
    for (int li = 1; li < L; ++li)
      if (H[li].A.rows <= rep) {
        amg_g = li;
        break;
      }
  }
  // Ghost lists of every rank on the distributed levels (the halo plans need
  // both directions): the matrix columns outside the rank's rows, plus on a
  // coarse level the aggregates of the rank's finer rows that another rank
  // owns (an aggregate belongs to its seed's rank and may reach into the next
  // ranks: the prolongation reads those coarse values, the restriction the
  // fine residuals of members owned by the next ranks, which are matrix
  // neighbours of the seed and so already ghosts of the seed's rank).
  std::vector<std::vector<std::vector<uint32_t>>> ghosts(amg_g);
  for (int li = 0; li < amg_g; ++li) {
    const AmgHostLevel& HL = H[li];
    ghosts[li].resize(R);
#pragma omp parallel for schedule(dynamic, 1)
    for (int q = 0; q < R; ++q) {
      auto& gq = ghosts[li][q];
      const uint64_t C0 = HL.part[q], C1 = HL.part[q + 1];
      for (uint64_t i = C0; i < C1; ++i)
        for (uint32_t k = HL.A.row[i]; k < HL.A.row[i + 1]; ++k) {
          const uint32_t c = HL.A.col[k];
          if (c < C0 || c >= C1) gq.push_back(c);
        }
      if (li > 0) {
        const AmgHostLevel& HF = H[li - 1];
        for (uint64_t i = HF.part[q]; i < HF.part[q + 1]; ++i) {
          const uint32_t a = HF.agg[i];
          if (a < C0 || a >= C1) gq.push_back(a);
        }
      }
      std::sort(gq.begin(), gq.end());
      gq.erase(std::unique(gq.begin(), gq.end()), gq.end());
    }
  }
  // signed local index of global row c of distributed level li on this rank
  auto rel_of = [&](int li, uint64_t c) -> int32_t {
    const AmgGpuLevel& G = levels[li];
    if (c >= G.C0 && c < G.C1) return (int32_t)(c - G.C0);
    const auto& gh = ghosts[li][rk];
    const auto it = std::lower_bound(gh.begin(), gh.end(), (uint32_t)c);
    if (it == gh.end() || *it != c) throw std::logic_error("AMG: row is neither owned nor a ghost");
    const uint32_t k = (uint32_t)(it - gh.begin());
    return k < G.glo ? (int32_t)k - (int32_t)G.glo : (int32_t)(G.npad + (k - G.glo));
  };
  levels.assign(L, AmgGpuLevel{});
  auto zeroed = [&](size_t cnt) {
    float* p = arena.alloc<float>(cnt + 64);
    CFD_HIP(hipMemsetAsync(p, 0, (cnt + 64) * sizeof(float), stream));
    return p;
  };
  for (int li = 0; li < L; ++li) {  // layouts first: P of level li needs level li + 1's
    const AmgHostLevel& HL = H[li];
    AmgGpuLevel& G = levels[li];
    G.nglob = HL.A.rows;
    G.part = HL.part;
    G.C0 = HL.part[rk];
    G.C1 = HL.part[rk + 1];
    if (li < amg_g) {
      G.dist = true;
      const auto& gh = ghosts[li][rk];
      G.glo = (uint32_t)(std::lower_bound(gh.begin(), gh.end(), (uint32_t)G.C0) - gh.begin());
      G.ghi = (uint32_t)gh.size() - G.glo;
      G.npad = (uint32_t)(((G.C1 - G.C0) + 63) & ~(uint64_t)63);
    }
  }
  for (int li = 0; li < L; ++li) {
    const AmgHostLevel& HL = H[li];
    AmgGpuLevel& G = levels[li];
    if (G.dist) {  // distributed level: owned rows + ghosts
      const uint32_t n = (uint32_t)(G.C1 - G.C0);
      std::vector<uint32_t> lrow(n + 1);
      for (uint32_t i = 0; i <= n; ++i) lrow[i] = HL.A.row[G.C0 + i] - HL.A.row[G.C0];
      const uint32_t* lcol = HL.A.col.data() + HL.A.row[G.C0];
      level_image(HL.A, G.C0, n, [&](uint32_t c) { return rel_of(li, c); }, G, arena, stream, amg_wide_limit);
      G.plan = build_halo_plan_lists(HL.part, rk, ghosts[li], G.glo, G.npad);
      interior_rows(HL.part, rk, lrow.data(), n, lcol, G.plan.lo_end, G.plan.hi_begin);
      make_plan_buffers(G.plan, 1);
      if (li == 0) {
        if (G.glo != topo.glo || G.ghi != topo.ghi || G.npad != topo.npad)
          throw std::logic_error("AMG level 0 ghosts differ from the cell ghosts");
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
    } else {  // replicated (or single-GPU) level, global numbering
      const uint32_t n = (uint32_t)HL.A.rows;
      level_image(HL.A, 0, n, [](uint32_t c) { return (int32_t)c; }, G, arena, stream, amg_wide_limit);
      G.npad = G.dev.stride;
      G.xt = zeroed(G.npad);
      G.r = zeroed(G.npad);
      if (li > 0) {
        G.x = zeroed(G.npad);
        G.b = zeroed(G.npad);
      }
    }
    set_amg_full_policy(G, li);
    // coarsening operators: P as an aggregate index per stored fine row
    // (signed local coarse index into a distributed next level, global id into
    // a replicated one), R = P^T rows of this rank's aggregates with local fine
    // members (owned, or ghosts of the next ranks)
    if (HL.has_op) {
      const AmgHostLevel& HC = H[li + 1];
      const bool next_dist = levels[li + 1].dist;
      std::vector<uint32_t> agg(G.dev.stride, 0), r_row, r_col;
      if (G.dist) {
        for (uint64_t i = G.C0; i < G.C1; ++i)
          agg[i - G.C0] = next_dist ? (uint32_t)rel_of(li + 1, HL.agg[i]) : HL.agg[i];
        const uint64_t I0 = HC.part[rk], I1 = HC.part[rk + 1];
        r_row.resize(I1 - I0 + 1);
        for (uint64_t I = I0; I <= I1; ++I) r_row[I - I0] = HL.r_row[I] - HL.r_row[I0];
        r_col.assign(HL.r_col.begin() + HL.r_row[I0], HL.r_col.begin() + HL.r_row[I1]);
        for (auto& f : r_col) {
          const int32_t lf = rel_of(li, f);
          if (lf < 0) throw std::logic_error("AMG: aggregate member below its seed's rank");
          f = (uint32_t)lf;
        }
        G.dev.nc = (uint32_t)(I1 - I0);
        // members live on this or higher ranks, seeds on this or lower ones: the
        // aggregates with ghost members come last, the fine rows of lower-rank
        // aggregates first
        const uint32_t nown = (uint32_t)(G.C1 - G.C0);
        G.rc_hi = G.dev.nc;
        for (uint32_t I = 0; I < G.dev.nc; ++I) {
          bool ghost = false;
          for (uint32_t k = r_row[I]; k < r_row[I + 1]; ++k) ghost |= r_col[k] >= nown;
          if (ghost) {
            G.rc_hi = I;
            break;
          }
        }
        G.pf_lo = 0;
        if (next_dist) {
          const uint32_t ncl = G.dev.nc;
          for (uint32_t i = 0; i < nown; ++i)
            if ((int32_t)agg[i] < 0 || agg[i] >= ncl) G.pf_lo = i + 1;
          G.pf_lo = std::min((G.pf_lo + 3) & ~3u, nown);
        }
      } else {
        std::copy(HL.agg.begin(), HL.agg.end(), agg.begin());
        r_row = HL.r_row;
        r_col = HL.r_col;
        G.dev.nc = HL.nc;
      }
      G.dev.agg = arena.upload(agg, stream, kAggSlack);
      G.dev.r_row = arena.upload(r_row, stream);
      G.dev.r_col = arena.upload(r_col, stream);
      {
        std::vector<int32_t> m4;
        build_r_m4(r_row, r_col, m4);
        G.dev.r_m4 = reinterpret_cast<const int4*>(arena.upload(m4, stream));
      }
    }
  }
}

// Drop the hierarchy (its device memory included); the next AMG solve builds
// a new one from the matrix of that moment (or from a loaded source).
void Solver::drop_amg() {
  CFD_HIP(hipSetDevice(device));
  sync();
  drop_graphs();  // they hold the hierarchy's pointers
  levels.clear();
  d_tail = nullptr;
  tail_blob_first = -1;
  d_tail_blob = nullptr;
  d_tail_desc = nullptr;
  tail_blob_words = tail_vec_floats = 0;
  amg_refresh.clear();
  rr_pair.clear();  // their block images lived in amg_arena
  up_pair.clear();
  amg_setup_flag = nullptr;
  amg_refresh_pending = false;
  amg_arena.release();
  amg_built = false;
  amg_setup_path = 0;
  amg_age = 0;
}

void Solver::ensure_amg() {
  if (amg_built) {
    if (amg_refresh_pending) {
      const Range range("amg refresh");
      refresh_amg();
      amg_refresh_pending = false;
      amg_age = 0;
    }
    return;
  }
  const Range range("amg setup");
  const bool timing = cfg.log_level >= 2 && rk == 0;
  const auto t_start = std::chrono::steady_clock::now();
  const char* se = knob(Knob::AmgSetup);
  if (se && std::strcmp(se, "host") && std::strcmp(se, "device") && std::strcmp(se, "rebuild"))
    throw std::invalid_argument(std::string("CFD_AMG_SETUP: expected device, host or rebuild, got ") + se);
  const bool device_setup = !(se && std::string(se) == "host");
  const char* how = "device";
  amg_setup_path = 2;
  const size_t slots_s = (size_t)topo.ws * topo.ld;
  if (!amg_src) amg_src = arena.alloc<float>(slots_s);
  const bool from_checkpoint = amg_src_loaded;  // then amg_age is the saved run's
  if (!from_checkpoint)  // keep the source matrix for cfd_state_save
    CFD_HIP(hipMemcpyAsync(amg_src, sval, slots_s * sizeof(float), hipMemcpyDeviceToDevice, stream));
  amg_src_loaded = false;
  // both setup paths read `sval`: point it at the source for the build; the
  // hierarchy's allocations go to amg_arena (arena swapped for the build)
  float* const live = sval;
  sval = amg_src;
  amg_arena.release();
  arena.swap(amg_arena);
  struct Restore {
    Solver* s;
    float* live;
    ~Restore() {
      s->sval = live;
      s->arena.swap(s->amg_arena);
    }
  } restore{this, live};
  if (!(device_setup && build_amg_device())) {
    how = "host";
    amg_setup_path = 1;
    levels.clear();
    arena.release();  // the device attempt's partial hierarchy
    build_amg_host();
  }
  const int L = (int)levels.size();
  set_resrestrict_blocks();
  // post-smoothers with the prolongation fused (single-GPU / replicated
  // levels of at most CFD_AMG_FUSED_PROLONG_ROWS rows; 0: never)
  fuse_prolong_rows = knob_u64(Knob::AmgFusedProlongRows, 1ull << 20);
  // the tail form: blob<K> (default blob2), lds, global
  {
    const char* tf = knob(Knob::AmgTail);
    tail_form = 2;
    tail_blob_shift = 2;
    if (tf && std::strncmp(tf, "blob", 4) == 0) {
      if (tf[4]) tail_blob_shift = std::max(0, (int)std::strtol(tf + 4, nullptr, 10));
    } else if (tf && std::strcmp(tf, "lds") == 0) {
      tail_form = 1;
    } else if (tf && std::strcmp(tf, "global") == 0) {
      tail_form = 0;
    } else if (tf) {
      throw std::invalid_argument(std::string("CFD_AMG_TAIL: expected blob<K>, lds or global, got ") + tf);
    }
  }
  // replicated levels from `tail_first` down run inside one single-workgroup kernel
  const uint32_t tail_rows = (uint32_t)knob_u64(Knob::AmgTailRows, 4096u);
  const int lo = std::max(amg_g, 1);
  tail_first = L;
  while (tail_first > lo && levels[tail_first - 1].dev.n <= tail_rows) --tail_first;
  // wide levels (16-bit row lengths) run only in the one-workgroup tail kernels
  {
    int bad = -1;  // first wide level the row kernels would run (level 0 or a row-partitioned level)
    for (int li = 0; li < L; ++li)
      if (levels[li].wide) {
        if (li < lo)
          bad = li;
        else
          tail_first = std::min(tail_first, li);
        break;
      }
    // the width of a row-partitioned level is per rank: every rank throws together
    uint64_t any_bad = bad >= 0 ? 1 : 0;
    if (dist())
      for (uint64_t f : allgather_u64(any_bad)) any_bad |= f;
    if (any_bad)
      throw std::invalid_argument("AMG: rows wider than 255 entries on a level the row kernels run (level 0 or a "
                                  "row-partitioned level): unsupported layout");
  }
  std::vector<AmgTailLevel> tl(L);
  for (int li = 0; li < L; ++li) {
    tl[li].L = levels[li].dev;
    tl[li].x = levels[li].x;
    tl[li].xt = levels[li].xt;
    tl[li].b = levels[li].b;
    tl[li].r = levels[li].r;
  }
  d_tail = arena.upload(tl, stream);
  check_launch("AMG setup");
  if (tail_form == 2) {
    // The LDS image of the tail (matrices included) is the fast tail; when it
    // does not fit in one CU's LDS, up to tail_blob_shift (CFD_AMG_TAIL=blob<K>,
    // default 2) more levels run with the row kernels so that it does (C1: the
    // 3.9 k-row level).
    const int shift = tail_blob_shift;
    const int t0 = std::max({tail_first, 1, dist() ? amg_g : 0});
    for (int t = t0; t < std::min(L, t0 + 1 + shift) && tail_blob_first < 0; ++t) {
      if (t > t0 && levels[t - 1].wide) break;  // wide levels run only in the tail kernels
      build_tail_blob(t);
      if (tail_blob_first >= 0) tail_first = t;
    }
  }
  build_rr_pairs();
  sync();
  amg_built = true;
  if (!from_checkpoint) amg_age = 0;
  if (timing) {
    std::string pairs;
    for (int li = 0; li < (int)rr_pair.size(); ++li)
      if (rr_pair[li].nblocks) pairs += " " + std::to_string(li) + "+" + std::to_string(li + 1);
    std::string ups;
    for (int li = 0; li < (int)up_pair.size(); ++li)
      if (up_pair[li].nblocks) ups += " " + std::to_string(li) + "+" + std::to_string(li - 1);
    std::fprintf(stderr,
                 "[amg setup] %s path: %d levels in %.3f s, tail from level %d (LDS image from level %d), "
                 "down-leg pairs:%s, up-leg pairs:%s\n",
                 how, L, std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count(),
                 tail_first, tail_blob_first, pairs.empty() ? " none" : pairs.c_str(), ups.empty() ? " none" : ups.c_str());
  }
}

// Aggregates per block of k_amg_resrestrict for the single-GPU / replicated
// levels with a coarse level and at most CFD_AMG_FUSED_RR_ROWS rows (default
// 2^18; distributed levels restrict ghost residuals and keep the two
// kernels): about 256 members per block, fewer aggregates while a block's
// members exceed its LDS capacity.  Its one-row-per-thread residual over
// permuted rows only pays on the latency-bound levels: same-box A/B
// (profiles/r03/ab_log.md) C2 level 0 129 vs 68 + 34 us, level 1 104 vs
// 56 + 13 us; C1 levels of 125 k rows and fewer 6-8 vs 10-11 us.
// CFD_AMG_FUSED_RR_ROWS=0 keeps the two kernels everywhere.
void Solver::set_resrestrict_blocks() {
  const uint64_t max_rows = knob_u64(Knob::AmgFusedRrRows, 1u << 18);
  for (AmgGpuLevel& G : levels) {
    AmgLevelDev& d = G.dev;
    d.rr_agg = 0;
    if (max_rows == 0 || G.dist || d.nc == 0 || d.n == 0 || d.n > max_rows || !d.r_row) continue;
    std::vector<uint32_t> rr((size_t)d.nc + 1);
    CFD_HIP(hipMemcpyAsync(rr.data(), d.r_row, rr.size() * 4, hipMemcpyDeviceToHost, stream));
    sync();
    uint32_t a = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(256, (uint64_t)256 * d.nc / d.n));
    for (; a >= 1; a /= 2) {
      uint32_t worst = 0;
      for (uint32_t I = 0; I < d.nc; I += a) worst = std::max(worst, rr[std::min(I + a, d.nc)] - rr[I]);
      if (worst <= kRRCap) break;
    }
    d.rr_agg = a;
  }
}

// Down-leg pairs (k_amg_resrestrict_pair): greedily from the top, two
// adjacent levels that both take k_amg_resrestrict and whose second level is
// pre-smoothed inside the V-cycle's down loop run as one launch.
void Solver::build_rr_pairs() {
  const int L = (int)levels.size();
  rr_pair.assign(L, AmgPairImage{});
  up_pair.assign(L, AmgUpPairImage{});
  pair_mode = (int)knob_u64(Knob::AmgFusedPair, 1);  // 0 off, 1 where cheap, 2 every candidate (tests)
  if (pair_mode == 0) return;
  const int D = dist() ? amg_g : 0;
  const int down = std::min(std::max({tail_first, 1, D}), L - 1);
  for (int i = 0; i + 1 < down;) {
    const AmgGpuLevel &F = levels[i], &M = levels[i + 1];
    const bool ok = !F.dist && !M.dist && !F.wide && !M.wide && F.dev.rr_agg && M.dev.rr_agg && M.dev.w >= 1;
    i += (ok && build_rr_pair(i)) ? 2 : 1;
  }
  // up-leg: from the bottom, post-smoothers of levels c and c - 1 that both
  // take the fused prolongation, fine level at most 2^18 rows
  for (int c = down - 1; c >= 1;) {
    const AmgGpuLevel &C = levels[c], &F = levels[c - 1];
    const bool ok = fused_prolong(c) && fused_prolong(c - 1) && !C.wide && !F.wide && F.dev.n <= (1u << 18) &&
                    F.dev.w >= 1 && C.dev.agg;
    c -= (ok && build_up_pair(c)) ? 2 : 1;
  }
}

// The up-leg pair image of levels (c, c - 1): blocks of kUpPairRows fine rows
// and the level-c rows T they need (kUpPairCap at most), with the T-local
// index of every fine slot's column aggregate.  Mode 1 pairs only while the
// blocks' T rows total at most 2.5x the level's rows (profiles/r06/ab_log.md,
// C1: levels 5+4 9.1 us against 7.5 + 6.3, in; 3+2 13.1 against 6.8 + 6.7,
// out).
bool Solver::build_up_pair(int c) {
  const AmgLevelDev &F = levels[c - 1].dev, &C = levels[c].dev;
  const uint32_t nf = F.n;
  const size_t slots = (size_t)F.w * F.stride;
  std::vector<uint8_t> flen(nf);
  std::vector<uint32_t> agg(nf);
  std::vector<int32_t> fc(slots);
  CFD_HIP(hipMemcpyAsync(flen.data(), F.len, nf, hipMemcpyDeviceToHost, stream));
  CFD_HIP(hipMemcpyAsync(agg.data(), F.agg, (size_t)nf * 4, hipMemcpyDeviceToHost, stream));
  if (F.use16) {
    std::vector<int16_t> c16(slots);
    CFD_HIP(hipMemcpyAsync(c16.data(), F.col16, slots * 2, hipMemcpyDeviceToHost, stream));
    sync();
    for (size_t k = 0; k < slots; ++k) fc[k] = (int32_t)(k % F.stride) + c16[k];
  } else {
    CFD_HIP(hipMemcpyAsync(fc.data(), F.col32, slots * 4, hipMemcpyDeviceToHost, stream));
    sync();
  }
  std::vector<uint32_t> frow(nf + 1, 0), fcol;
  for (uint32_t g = 0; g < nf; ++g) frow[g + 1] = frow[g] + flen[g];
  fcol.resize(frow[nf]);
  for (uint32_t g = 0; g < nf; ++g)
    for (uint32_t r = 0; r < flen[g]; ++r) fcol[frow[g] + r] = (uint32_t)fc[(size_t)r * F.stride + g];
  UpPairPartition up;
  if (!build_up_pair_partition(frow, fcol, agg, C.n, kUpPairRows, kUpPairCap, up)) return false;
  if (pair_mode < 2 && (double)up.t.size() > 2.5 * (double)C.n) return false;
  std::vector<uint16_t> lt(slots, 0), lto(F.stride, 0);
  for (uint32_t g = 0; g < nf; ++g) {
    lto[g] = up.lto[g];
    for (uint32_t r = 0; r < flen[g]; ++r) lt[(size_t)r * F.stride + g] = up.lt[frow[g] + r];
  }
  AmgUpPairImage& P = up_pair[c];
  P.nblocks = (uint32_t)up.tb.size() - 1;
  P.tb = arena.upload(up.tb, stream);
  P.t = arena.upload(up.t, stream);
  P.lt = arena.upload(lt, stream);
  P.lto = arena.upload(lto, stream);
  sync();
  return true;
}

// The pair image of levels (i, i+1): blocks of level-(i+2) aggregates whose
// level-(i+1) rows (members + ring: S) and level-i members of S each fit
// kPairThreads.  False (no pair) when one aggregate alone does not fit.
bool Solver::build_rr_pair(int i) {
  const AmgLevelDev &F = levels[i].dev, &M = levels[i + 1].dev;
  const uint32_t nm = M.n, nc = M.nc;
  auto down_u32 = [&](const uint32_t* d, size_t n) {
    std::vector<uint32_t> h(n);
    CFD_HIP(hipMemcpyAsync(h.data(), d, n * 4, hipMemcpyDeviceToHost, stream));
    return h;
  };
  const std::vector<uint32_t> fr_row = down_u32(F.r_row, (size_t)F.nc + 1), fr_col = down_u32(F.r_col, F.n);
  const std::vector<uint32_t> mr_row = down_u32(M.r_row, (size_t)nc + 1), mr_col = down_u32(M.r_col, nm);
  std::vector<uint8_t> mlen(nm);
  CFD_HIP(hipMemcpyAsync(mlen.data(), M.len, nm, hipMemcpyDeviceToHost, stream));
  const size_t slots = (size_t)M.w * M.stride;
  std::vector<int32_t> mcol(slots);
  if (M.use16) {
    std::vector<int16_t> c16(slots);
    CFD_HIP(hipMemcpyAsync(c16.data(), M.col16, slots * 2, hipMemcpyDeviceToHost, stream));
    sync();
    for (size_t k = 0; k < slots; ++k) mcol[k] = (int32_t)(k % M.stride) + c16[k];
  } else {
    CFD_HIP(hipMemcpyAsync(mcol.data(), M.col32, slots * 4, hipMemcpyDeviceToHost, stream));
    sync();
  }
  if (F.nc != nm) return false;
  // the off-diagonal pattern of level i + 1 as CSR in slot order
  std::vector<uint32_t> mrow(nm + 1, 0), mcsr;
  for (uint32_t g = 0; g < nm; ++g) mrow[g + 1] = mrow[g] + mlen[g];
  mcsr.resize(mrow[nm]);
  for (uint32_t g = 0; g < nm; ++g)
    for (uint32_t r = 0; r < mlen[g]; ++r) mcsr[mrow[g] + r] = (uint32_t)mcol[(size_t)r * M.stride + g];
  // 256-thread blocks (one CU each, like the k_amg_resrestrict launches they
  // replace) while the ring's redundant level-i rows stay within 50 %
  // (profiles/r06/ab_log.md, C1: levels 4+5 at 1.41x rows 7.8 us against
  // 5.5 + 5.1; levels 2+3 at 2.9x 16.1 us against 7.1 + 6.3; 1,024-thread
  // blocks -- less redundancy, a quarter of the CUs -- lost on both pairs)
  PairPartition pp;
  const uint32_t threads = 256;
  if (!build_pair_partition(fr_row, fr_col, mr_row, mr_col, mrow, mcsr, threads, pp)) return false;
  if (pair_mode < 2 && (double)pp.f.size() > 1.5 * (double)F.n) return false;
  std::vector<uint16_t> lc(slots, 0);
  for (uint32_t g = 0; g < nm; ++g)
    for (uint32_t r = 0; r < mlen[g]; ++r) lc[(size_t)r * M.stride + g] = pp.lc[mrow[g] + r];
  const uint32_t nb = (uint32_t)pp.jb.size() - 1;
  const std::vector<uint32_t>&jb = pp.jb, &sb = pp.sb, &sv = pp.s, &fo = pp.fo, &fv = pp.f;
  AmgPairImage& P = rr_pair[i];
  P.nblocks = nb;
  P.threads = threads;
  P.jb = arena.upload(jb, stream);
  P.sb = arena.upload(sb, stream);
  P.s = arena.upload(sv, stream);
  P.fo = arena.upload(fo, stream);
  P.f = arena.upload(fv, stream);
  P.lc = arena.upload(lc, stream);
  sync();
  return true;
}

// LDS image of the tail levels [tf, L) for k_amg_tail_blob: every array the
// tail V-cycle reads, compacted (off-diagonal CSR, u16 indices) from the
// level images, when vectors + blob fit in one CU's LDS.
void Solver::build_tail_blob(int tf, bool reuse) {
  const uint32_t old_words = tail_blob_words;
  tail_blob_first = -1;
  const int L = (int)levels.size();
  if (tf >= L) return;
  std::vector<uint32_t> blob;
  std::vector<TailBlobLevel> desc(L);
  auto align4 = [&] {
    while (blob.size() % 4) blob.push_back(0);
    return (uint32_t)blob.size();
  };
  auto put_f = [&](const float* v, size_t n) {
    const uint32_t o = align4();
    for (size_t i = 0; i < n; ++i) {
      uint32_t w;
      std::memcpy(&w, v + i, 4);
      blob.push_back(w);
    }
    return o;
  };
  auto put_u32 = [&](const std::vector<uint32_t>& v) {
    const uint32_t o = align4();
    blob.insert(blob.end(), v.begin(), v.end());
    return o;
  };
  auto put_u16 = [&](const std::vector<uint32_t>& v) {
    const uint32_t o = align4();
    for (size_t i = 0; i < v.size(); i += 2)
      blob.push_back((v[i] & 0xFFFFu) | ((i + 1 < v.size() ? v[i + 1] & 0xFFFFu : 0u) << 16));
    return o;
  };
  auto put_u8 = [&](const std::vector<uint8_t>& v) {
    const uint32_t o = align4();
    for (size_t i = 0; i < v.size(); i += 4) {
      uint32_t w = 0;
      for (size_t b = 0; b < 4 && i + b < v.size(); ++b) w |= (uint32_t)v[i + b] << (8 * b);
      blob.push_back(w);
    }
    return o;
  };
  auto d2h = [&](void* dst, const void* src, size_t bytes) {
    if (bytes) CFD_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, stream));
  };
  uint32_t vec = 0;
  for (int l = tf; l < L; ++l) {
    const AmgLevelDev& d = levels[l].dev;
    const uint32_t n = d.n, st = d.stride;
    if (n > 65535 || d.nc > 65535 || levels[l].wide) return;  // the blob keeps u8 diagonal ranks
    const size_t slots = (size_t)std::max(d.w, 1) * st;
    std::vector<uint8_t> len(n), drank(n);
    std::vector<float> dv(n), de(n), val(slots);
    std::vector<int16_t> c16(d.use16 ? slots : 0);
    std::vector<int32_t> c32(d.use16 ? 0 : slots);
    d2h(len.data(), d.len, n);
    d2h(drank.data(), d.drank, n);
    d2h(dv.data(), d.dv, (size_t)n * 4);
    d2h(de.data(), d.de, (size_t)n * 4);
    d2h(val.data(), d.val, slots * 4);
    if (d.use16) d2h(c16.data(), d.col16, slots * 2);
    else d2h(c32.data(), d.col32, slots * 4);
    std::vector<uint32_t> agg, rrow, rcol;
    if (d.nc) {
      agg.resize(n);
      rrow.resize((size_t)d.nc + 1);
      d2h(agg.data(), d.agg, (size_t)n * 4);
      d2h(rrow.data(), d.r_row, rrow.size() * 4);
    }
    sync();
    if (d.nc) {
      rcol.resize(rrow[d.nc]);
      d2h(rcol.data(), d.r_col, rcol.size() * 4);
      sync();
    }
    std::vector<uint32_t> ro(n + 1, 0), cols;
    std::vector<float> vals;
    for (uint32_t i = 0; i < n; ++i) {
      ro[i + 1] = ro[i] + len[i];
      for (uint32_t r = 0; r < len[i]; ++r) {
        const size_t o = (size_t)r * st + i;
        const int64_t c = d.use16 ? (int64_t)i + c16[o] : (int64_t)c32[o];
        if (c < 0 || c >= (int64_t)n) return;  // tail levels are replicated: global columns
        cols.push_back((uint32_t)c);
        vals.push_back(val[o]);
      }
    }
    TailBlobLevel& D = desc[l];
    D.n = n;
    D.nc = d.nc;
    D.maxlen = n ? *std::max_element(len.begin(), len.end()) : 0;
    D.de = put_f(de.data(), n);
    D.dv = put_f(dv.data(), n);
    D.rowoff = put_u32(ro);
    D.drank = put_u8(drank);
    D.val = put_f(vals.data(), vals.size());
    D.col = put_u16(cols);
    if (d.nc) {
      D.agg = put_u16(agg);
      D.r_row = put_u16(rrow);
      D.r_col = put_u16(rcol);
    }
    vec += 4 * ((n + 3) & ~3u);
  }
  align4();
  if (4 * ((size_t)vec + blob.size()) > lds_budget) return;
  if (reuse && d_tail_blob && blob.size() == old_words) {  // same structure: new values in place
    CFD_HIP(hipMemcpyAsync(d_tail_blob, blob.data(), blob.size() * 4, hipMemcpyHostToDevice, stream));
    CFD_HIP(hipMemcpyAsync(d_tail_desc, desc.data(), desc.size() * sizeof(TailBlobLevel), hipMemcpyHostToDevice,
                           stream));
    sync();  // the host staging vectors die here
  } else {
    if (reuse) throw std::logic_error("AMG refresh: tail blob layout changed");
    d_tail_blob = arena.upload(blob, stream);
    d_tail_desc = arena.upload(desc, stream);
  }
  tail_blob_words = (uint32_t)blob.size();
  tail_vec_floats = vec;
  tail_blob_first = tf;
}

// Timing of level-0 smoother launches (bench roofline): a pair of pool events
// per launch, recorded by the GPU at kernel start / end (hipExtLaunchKernel).
// The pool is created before the timed steps (cfd_profile_reset) and grows
// without synchronising; only at kProfPoolMax events is it drained (a stream
// synchronisation) into prof_ms.
std::pair<hipEvent_t, hipEvent_t> Solver::prof_pair() {
  if (prof_used + 2 > prof_ev.size()) {
    if (prof_ev.size() < kProfPoolMax) {
      prof_grow(prof_ev.size() + 1024);  // no synchronisation inside the timed steps
    } else {
      CFD_HIP(hipStreamSynchronize(stream));
      for (size_t k = 0; k + 1 < prof_used; k += 2) {
        float ms = 0.0f;
        CFD_HIP(hipEventElapsedTime(&ms, prof_ev[k], prof_ev[k + 1]));
        prof_ms += ms;
      }
      prof_used = 0;
    }
  }
  prof_used += 2;
  return {prof_ev[prof_used - 2], prof_ev[prof_used - 1]};
}

void Solver::prof_grow(size_t n) {
  while (prof_ev.size() < n) {
    hipEvent_t e;
    CFD_HIP(hipEventCreate(&e));
    prof_ev.push_back(e);
  }
}

void Solver::amg_smooth(size_t li, float*& xcur, const float* b, bool x_zero, bool nt) {
  AmgGpuLevel& L = levels[li];
  if (x_zero) {
    launch_amg_smooth_zero(L.dev, b, L.xt, stream);
  } else if (li == 0 && prof_take()) {
    if (capturing) {  // event nodes of the graph around the launch, read per replay (graph_harvest)
      hipEvent_t e0, e1;
      CFD_HIP(hipEventCreate(&e0));
      capturing->ev.push_back(e0);
      CFD_HIP(hipEventCreate(&e1));
      capturing->ev.push_back(e1);
      CFD_HIP(hipEventRecordWithFlags(e0, stream, hipEventRecordExternal));
      launch_amg_smooth(L.dev, xcur, b, L.xt, stream, nullptr, nullptr, nt);
      CFD_HIP(hipEventRecordWithFlags(e1, stream, hipEventRecordExternal));
    } else {
      const auto ev = prof_pair();
      launch_amg_smooth(L.dev, xcur, b, L.xt, stream, ev.first, ev.second, nt);
      prof_launches++;
    }
  } else {
    launch_amg_smooth(L.dev, xcur, b, L.xt, stream, nullptr, nullptr, nt);
  }
  std::swap(xcur, L.xt);  // out-of-place Jacobi: the partner buffer becomes current
}

// amg.rs:666-770, level 0 bound to (x = p_sol, b = temp_p).  Replicated levels
// from `tail_first` on run as one single-workgroup kernel (k_amg_tail).  On a
// distributed rank the levels below amg_g are row-partitioned: each smoother
// input gets a halo (the cleared coarse x needs none), the restriction into
// the first replicated level is all-gathered.
void Solver::v_cycle() {
  const int L = (int)levels.size();
  levels[0].x = p_sol;
  levels[0].b = temp_p;
  if (ref_inplace || ref_clamp) {
    v_cycle_reference();
    return;
  }
  const int D = dist() ? amg_g : 0;
  // the tail needs level >= 1 (level 0's x/b are bound per call) and is off
  // while the level-0 smoother is being timed on a one-level hierarchy
  const int tf = (prof && L == 1) ? L : std::max({tail_first, 1, D});
  const int down = std::min(tf, L - 1);
  // smoother sweep; on a distributed level the x halo overlaps the interior rows
  // post: the up-sweep's smoother (nontemporal matrix loads with nt_mask bit 1)
  auto sm = [&](int i, bool x_zero, bool post = false) {
    AmgGpuLevel& Lv = levels[i];
    const bool ntl = nt(post ? 1u : 16u);
    if (!Lv.dist || x_zero) {
      amg_smooth(i, Lv.x, Lv.b, x_zero, ntl);
      return;
    }
    const bool timed = i == 0 && prof_take();  // kernel time only: each part timed separately
    const CommScope cs(this, amg_cat(i));
    overlapped(Lv.plan, {{Lv.x, 1}}, Lv.dev.n, [&](uint32_t a, uint32_t b, uint32_t a2, uint32_t b2) {
      AmgLevelDev d = Lv.dev;
      d.r0 = a;
      d.r1 = b;
      d.r2 = a2;
      d.r3 = b2;
      if (timed) {
        const auto ev = prof_pair();
        launch_amg_smooth(d, Lv.x, Lv.b, Lv.xt, stream, ev.first, ev.second, ntl);
      } else {
        launch_amg_smooth(d, Lv.x, Lv.b, Lv.xt, stream, nullptr, nullptr, ntl);
      }
    });
    if (timed) prof_launches++;
    std::swap(Lv.x, Lv.xt);
  };
  auto res = [&](int i) {
    AmgGpuLevel& Lv = levels[i];
    auto f = [&](uint32_t a, uint32_t b, uint32_t a2, uint32_t b2) {
      AmgLevelDev d = Lv.dev;
      d.r0 = a;
      d.r1 = b;
      d.r2 = a2;
      d.r3 = b2;
      launch_amg_residual(d, Lv.x, Lv.b, Lv.r, stream, (i == 0 && nt(2)) || (i == 1 && nt(64)));
    };
    if (Lv.dist) {
      const CommScope cs(this, amg_cat(i));
      overlapped(Lv.plan, {{Lv.x, 1}}, Lv.dev.n, f);
    } else {
      f(0, Lv.dev.n, 0, 0);
    }
  };
  bool presmoothed = false;  // level i's zero-x pre-smoother already ran inside the restriction
  for (int i = 0; i < down; ++i) {
    AmgGpuLevel& Lv = levels[i];
    if (presmoothed)
      std::swap(Lv.x, Lv.xt);
    else
      sm(i, i > 0);  // coarse x was cleared by the restriction (ghosts too)
    AmgGpuLevel& C = levels[i + 1];
    // the next level is pre-smoothed by this loop: fuse its zero-x sweep into the restriction
    presmoothed = (i + 1 < down) && (!Lv.dist || C.dist);
    float* smo = presmoothed ? C.xt : nullptr;
    if (presmoothed && (size_t)i < rr_pair.size() && rr_pair[i].nblocks && i + 2 <= down) {
      // levels i and i + 1 in one launch; level i + 1 ends pre-smoothed (as
      // the next iteration's swap leaves it) and level i + 2 gets its rhs
      AmgGpuLevel& C2 = levels[i + 2];
      const bool pre2 = i + 2 < down;  // both replicated / single-GPU: as `presmoothed` below
      launch_amg_resrestrict_pair(Lv.dev, C.dev, rr_pair[i], Lv.x, Lv.b, C.b, C.xt, C2.b, C2.x,
                                  pre2 ? C2.xt : nullptr, C2.dev.de, stream);
      std::swap(C.x, C.xt);
      presmoothed = pre2;
      ++i;  // level i + 1 is done
      continue;
    }
    if (!Lv.dist && Lv.dev.rr_agg) {
      launch_amg_resrestrict(Lv.dev, Lv.x, Lv.b, C.b, C.x, smo, C.dev.de, stream);
    } else if (!Lv.dist) {
      res(i);
      launch_amg_restrict(Lv.dev, Lv.r, C.b, C.x, 0, 0, 0, stream, smo, C.dev.de);
    } else {
      res(i);
      // the restriction sums members owned by the next ranks too (their residuals
      // are ghosts): the aggregates without such members overlap the exchange
      const bool into_dist = C.dist;
      float* cb = into_dist ? C.b : C.b + C.C0;
      float* cx = into_dist ? C.x : C.x + C.C0;
      const uint32_t sc = into_dist ? C.npad : Lv.dev.nc;
      const uint32_t cg_lo = into_dist ? C.glo : (uint32_t)C.C0;
      const uint32_t cg_hi = into_dist ? C.ghi : (uint32_t)(C.nglob - C.C1);
      float* so = into_dist ? smo : nullptr;
      if (amg_local) {  // partition-aware: every member is owned, no residual halo
        launch_amg_restrict(Lv.dev, Lv.r, cb, cx, sc, cg_lo, cg_hi, stream, so, C.dev.de, 0, Lv.dev.nc, true);
      } else {
        const uint32_t split = Lv.dev.n >= overlap_min_rows ? Lv.rc_hi : 0u;  // as overlapped()
        const CommScope cs(this, amg_cat(i));
        halo_begin(Lv.plan, {{Lv.r, 1}});
        if (split > 0)
          launch_amg_restrict(Lv.dev, Lv.r, cb, cx, sc, cg_lo, cg_hi, stream, so, C.dev.de, 0, split, false);
        halo_end();
        launch_amg_restrict(Lv.dev, Lv.r, cb, cx, sc, cg_lo, cg_hi, stream, so, C.dev.de, split, Lv.dev.nc, true);
      }
    }
    if (Lv.dist && !C.dist) {  // into the first replicated level: own slice, all-gather
      std::vector<size_t> off(R + 1);
      for (int q = 0; q <= R; ++q) off[q] = C.part[q] * sizeof(float);
      timed_gather(kCommRepGather, off[rk + 1] - off[rk], [&] { comm->allgatherv_inplace(C.b, off, stream); });
    }
  }
  if (tf < L && tf == tail_blob_first) {
    launch_amg_tail_blob(d_tail, d_tail_desc, d_tail_blob, tail_blob_words, tail_vec_floats, tf, L, levels[tf].b,
                         levels[tf].dev.n, stream);
  } else if (tf < L) {
    size_t lds = 0;  // LDS-resident tail when its vectors fit (CFD_AMG_TAIL=global: never)
    for (int l = tf; l < L; ++l) lds += 4 * (((size_t)levels[l].dev.n + 3) & ~(size_t)3) * sizeof(float);
    if (lds > lds_budget || tail_form == 0) lds = 0;
    launch_amg_tail(d_tail, tf, L, lds, stream);
  } else {
    for (int s = 0; s < 10; ++s) sm(L - 1, s == 0 && L > 1);
  }
  for (int ii = down - 1; ii >= 0; --ii) {
    // the prolongation reads aggregates seeded on lower ranks (ghosts of the coarse x)
    if (levels[ii + 1].dist && amg_local) {  // partition-aware: every fine row's aggregate is owned
      AmgGpuLevel& F = levels[ii];
      launch_amg_prolong(F.dev, F.x, levels[ii + 1].x, stream, 0, F.dev.n, nt(32));
    } else if (levels[ii + 1].dist) {  // the rows of owned aggregates overlap the coarse-x exchange
      AmgGpuLevel& F = levels[ii];
      const uint32_t split = F.dev.n >= overlap_min_rows ? F.pf_lo : F.dev.n;  // as overlapped()
      const CommScope cs(this, amg_cat(ii + 1));
      halo_begin(levels[ii + 1].plan, {{levels[ii + 1].x, 1}});
      if (split < F.dev.n) launch_amg_prolong(F.dev, F.x, levels[ii + 1].x, stream, split, F.dev.n, nt(32));
      halo_end();
      if (split > 0) launch_amg_prolong(F.dev, F.x, levels[ii + 1].x, stream, 0, split, nt(32));
    } else if (ii >= 1 && (size_t)ii < up_pair.size() && up_pair[ii].nblocks) {
      // levels ii and ii - 1 post-smoothed in one launch; level ii's smoothed x
      // lives only in the kernel's LDS (nothing reads it after the up-leg), its
      // buffers swap as the separate launch would leave them
      AmgGpuLevel &Cl = levels[ii], &F = levels[ii - 1];
      launch_amg_prolong_smooth_pair(F.dev, Cl.dev, up_pair[ii], F.x, F.b, F.xt, Cl.x, Cl.b, levels[ii + 1].x, stream);
      std::swap(Cl.x, Cl.xt);
      std::swap(F.x, F.xt);
      --ii;  // level ii - 1 is done
      continue;
    } else if (fused_prolong(ii)) {
      // the prolongation applied inside the post-smoother's reads (x stays un-prolonged)
      AmgGpuLevel& F = levels[ii];
      launch_amg_smooth_prolong(F.dev, F.x, levels[ii + 1].x, F.b, F.xt, stream);
      std::swap(F.x, F.xt);
      continue;
    } else {
      launch_amg_prolong(levels[ii].dev, levels[ii].x, levels[ii + 1].x, stream, 0, 0, nt(32));
    }
    sm(ii, false, true);
  }
  // every level performs an even number of sweeps, so level 0 ends in p_sol
  if (levels[0].x != p_sol) throw std::logic_error("AMG level-0 ping-pong parity");
}

// FGMRES Preconditioner Step (coupled_solver_fgmres.rs:1911-1994)
void Solver::precondition(int j, float* z) {
  const CoupledMatrix A = cmat();
  const bool jacobi = constants.precond_type != 1;
  float* v = basis + (size_t)j * stride;  // V_j = binv[j] * W_j
  // the prediction reads neighbours' r_u, r_v
  const CommScope cs(this, kCommKrylovHalo);
  overlapped(cell_plan, {{v, 3}}, N, [&](uint32_t a, uint32_t b, uint32_t a2, uint32_t b2) {
    CoupledMatrix Ar = A;
    Ar.r0 = a;
    Ar.r1 = b;
    Ar.r2 = a2;
    Ar.r3 = b2;
    launch_precond_predict(Ar, v, binv, j, dinv_uv, dinv_p, temp_p, p_sol, jacobi ? temp : nullptr, stream, nt(4));
  });
  bool in_sol = true;
  if (!jacobi) {
    v_cycle();
  } else {
    // p_iters of coupled_solver_fgmres.rs:1949-1976 (global cell count)
    const size_t raw = 20u + (size_t)std::sqrt((float)NG) / 2u;
    const size_t p_iters = std::min<size_t>(raw, 200) == 0 ? 0 : std::min<size_t>(raw, 200) - 1;
    // small meshes: every sweep in one single-workgroup launch (same bits)
    if (!dist() && small_forms &&
        launch_relax_pressure_fused(N, topo.ld, (uint32_t)topo.ws, d_scol, d_slen, sval, dinv_p, temp_p, p_sol, temp,
                                    (uint32_t)p_iters, stream)) {
      if (p_iters & 1) in_sol = false;
    } else {
      AmgLevelDev rv{};  // the scalar ELL image (diagonal in the slots) as a row-kernel level
      rv.n = N;
      rv.r1 = N;
      rv.stride = topo.ld;
      rv.w = topo.ws;
      rv.use16 = topo.use16 ? 1 : 0;
      rv.full = 1;
      rv.val = sval;
      rv.col16 = d_scol16;
      rv.col32 = d_scol;
      rv.len = d_slen8;
      for (size_t it = 0; it < p_iters; ++it) {
        float* src = in_sol ? p_sol : temp;
        float* dst = in_sol ? temp : p_sol;
        if (dist()) halo(cell_plan, {{src, 1}});
        launch_relax_pressure4(rv, d_sdrank8, dinv_p, temp_p, src, dst, stream);
        in_sol = !in_sol;
      }
    }
  }
  float* ps = in_sol ? p_sol : temp;
  // the velocity correction reads neighbours' p_sol
  overlapped(cell_plan, {{ps, 1}}, N, [&](uint32_t a, uint32_t b, uint32_t a2, uint32_t b2) {
    CoupledMatrix Ar = A;
    Ar.r0 = a;
    Ar.r1 = b;
    Ar.r2 = a2;
    Ar.r3 = b2;
    launch_precond_correct(Ar, v, binv, j, ps, dinv_uv, z, stream);
  });
}

void Solver::set_reference_semantics(int flags) {
  if (flags & ~(1 | 2 | 4 | 8))
    throw std::invalid_argument("reference semantics on the GPU: flags 1 (in-place smoother), 2 (racy prepare), "
                                "4 (reduction order), 8 (restrict clamp) only");
  if (flags && dist()) throw std::invalid_argument("reference semantics: one GPU only");
  if ((flags & 2) && !d_flux_mirror) {  // each non-owner face slot -> the owner's slot of that face
    const size_t S = (size_t)topo.wf * N;
    size_t nfaces = 0;  // unused slots hold 0xFFFFFFFF: not a face
    for (size_t e = 0; e < S; ++e)
      if (topo.fs_face[e] != 0xFFFFFFFFu) nfaces = std::max(nfaces, (size_t)topo.fs_face[e] + 1);
    std::vector<int64_t> owner_slot(nfaces, -1);
    for (size_t e = 0; e < S; ++e)
      if (topo.fs_face[e] != 0xFFFFFFFFu && (topo.fs_meta[e] & kMetaOwner)) owner_slot[topo.fs_face[e]] = (int64_t)e;
    std::vector<int32_t> mirror(S, -1);
    for (size_t e = 0; e < S; ++e)
      if (topo.fs_face[e] != 0xFFFFFFFFu && topo.fs_other[e] != kNoCell && !(topo.fs_meta[e] & kMetaOwner)) {
        const int64_t o = owner_slot[topo.fs_face[e]];
        if (o < 0) throw std::logic_error("reference semantics: a face without its owner's slot");
        mirror[e] = (int32_t)o;
      }
    d_flux_mirror = arena.upload(mirror, stream);
  }
  if ((flags & 4) && !ref_part) {
    ref_ng = (uint32_t)((3 * (uint64_t)N + 63) / 64);
    ref_part = arena.alloc<float>((size_t)(m1 + 1) * ref_ng + 1);
    ref_norm = arena.alloc<float>((size_t)ref_ng + 1);
  }
  drop_graphs();  // captured iterations hold the other semantics' launches
  ref_red = (flags & 4) != 0;
  ref_inplace = (flags & 1) != 0;
  ref_clamp = (flags & 8) != 0;
  ref_racy = (flags & 2) != 0;
}

// amg.rs:666-770 dispatch by dispatch (test mode, flags 1 / 8): pre-smooth,
// residual + restriction (+ the clamped rows' store onto the last coarse
// entry), the coarse x cleared, 10 coarsest sweeps, prolongation +
// post-smooth -- no fused forms, no tail kernel.  In place (flag 1) the
// smoother runs its workgroups in order; else out-of-place Jacobi.
void Solver::v_cycle_reference() {
  const int L = (int)levels.size();
  auto smooth = [&](int i) {
    AmgGpuLevel& Lv = levels[i];
    if (ref_inplace) {
      launch_amg_smooth_ordered(Lv.dev, Lv.x, Lv.b, stream);
    } else {
      launch_amg_smooth(Lv.dev, Lv.x, Lv.b, Lv.xt, stream);
      std::swap(Lv.x, Lv.xt);
    }
  };
  for (int i = 0; i + 1 < L; ++i) {
    AmgGpuLevel &F = levels[i], &C = levels[i + 1];
    smooth(i);
    launch_amg_residual(F.dev, F.x, F.b, F.r, stream);
    launch_amg_restrict(F.dev, F.r, C.b, C.x, 0, 0, 0, stream);  // coarse b = R r, coarse x = 0
    const uint32_t nc = C.dev.n;
    if (ref_clamp && nc % 64 != 0) CFD_HIP(hipMemsetAsync(C.b + nc - 1, 0, sizeof(float), stream));
  }
  for (int s = 0; s < 10; ++s) smooth(L - 1);
  for (int i = L - 2; i >= 0; --i) {
    launch_amg_prolong(levels[i].dev, levels[i].x, levels[i + 1].x, stream);
    smooth(i);
  }
  if (levels[0].x != p_sol) throw std::logic_error("AMG level-0 ping-pong parity (reference semantics)");
}

void Solver::norm_launch(const float* v, int mode, int slot) {
  if (ref_red) {  // gpu_norm: norm_sq_partial + reduce_final (coupled_solver_fgmres.rs:1444-1588)
    launch_ref_norm_partials(v, 3 * N, ref_norm, stream);
    launch_reduce_final(ref_src(ref_norm, 1), mode, dsc + slot, binv, mode == 2 ? g : nullptr, m1, d_pin + slot,
                        stream);
    return;
  }
  launch_dot_partial(v, v, N, red.U, partial_n, stream);
  // the norm also lands in h_pin[slot] (mapped pinned memory): a blocking read needs no copy
  launch_reduce_final(combine(partial_n, 1), mode, dsc + slot, binv, mode == 2 ? g : nullptr, m1, d_pin + slot,
                      stream);
}

float Solver::norm_blocking(const float* v, int mode, int slot) {
  norm_launch(v, mode, slot);
  sync();
  return h_pin[slot];
}

// compute_residual_into (coupled_solver_fgmres.rs:1637-1667): V0 = b - A x, ||V0||
// V0 is stored unnormalised: binv[0] = 1/||r|| (the reference's scale_in_place),
// g = [||r||, 0, ...] (coupled_solver_fgmres.rs:1880-1890, 2380-2392).
float Solver::residual_into_v0_blocking() {
  residual_into_v0_launch();
  sync();
  return h_pin[1];
}

void Solver::residual_into_v0_launch() {
  // g = [||r||, 0, ...]: the zero fill is part of the norm's finishing kernel
  const CommScope cs(this, kCommKrylovHalo);
  overlapped(cell_plan, {{x, 3}}, N, [&](uint32_t a, uint32_t b, uint32_t a2, uint32_t b2) {
    CoupledMatrix A = cmat();
    A.r0 = a;
    A.r1 = b;
    A.r2 = a2;
    A.r3 = b2;
    launch_spmv(A, x, basis, stream, rhs, nt(8));  // V0 = 1 * b + -1 * (A x) as the SpMV stores it
  });
  norm_launch(basis, 2, 1);
}

// complete the lagged FGMRES residual read, if one is pending (async_buffer.rs)
void Solver::flush_inner() {
  if (inner.pending < 0) return;
  CFD_HIP(hipEventSynchronize(ev_iter[inner.pending]));
  inner.last = h_pin[64 + inner.pending];
  inner.has_last = true;
  inner.pending = -1;
}

// FGMRES iteration j (coupled_solver_fgmres.rs:1911-2283): Z_j = M^-1 V_j,
// w = A Z_j, CGS against V_0..V_j, ||w||, Hessenberg column + Givens.  The
// residual estimate also lands in pinned host memory at `pin` (natural
// schedule) -- no host reads in between, so the sequence is graph-capturable.
void Solver::iteration(int j, float* pin) {
  float* zj = zvec + (size_t)j * stride;
  precondition(j, zj);
  const CommScope cs(this, kCommKrylovHalo);
  overlapped(cell_plan, {{zj, 3}}, N, [&](uint32_t a, uint32_t b, uint32_t a2, uint32_t b2) {
    CoupledMatrix A = cmat();
    A.r0 = a;
    A.r1 = b;
    A.r2 = a2;
    A.r3 = b2;
    launch_spmv(A, zj, w, stream, nullptr, nt(8));
  });
  const bool lat = small_forms && cgs_latency_form(N);
  if (ref_red) {  // calc_dots_cgs / reduce_dots_cgs / update_w_cgs, then norm_sq_partial + finish
    launch_ref_cgs_dots(w, basis, binv, stride, j, 3 * N, ref_part, ref_ng, stream);
    launch_cgs_reduce(ref_src(ref_part, 2), j, H, m1, stream);
    launch_cgs_update_norm(w, basis, binv, stride, j, H, m1, N, red.U, partial_n, stream, cgs_keep_bytes > 0, true,
                           nullptr, lat);
    launch_ref_norm_partials(basis + (size_t)(j + 1) * stride, 3 * N, ref_norm, stream);
    launch_norm_givens(ref_src(ref_norm, 1), j, H, m1, givens, g, binv, resid_hist, pin, stream);
    check_launch("FGMRES iteration (reference reduction order)");
    return;
  }
  launch_cgs_dots(w, basis, binv, stride, j, N, red.U, partial, pstride, stream, cgs_keep_bytes, lat);
  const RedSrc dots = combine(partial, j + 1);
  const bool fuse_reduce = small_forms && cgs_reduce_fusable(dots);
  if (!fuse_reduce) launch_cgs_reduce(dots, j, H, m1, stream);
  // the whole restart basis and w within the kept bytes (small meshes): the
  // dots pass already reads every block with the default policy
  // (launch_cgs_dots), and the update reads / writes the basis with it too,
  // from the caches.  C0 21.2 -> 12.4 us per launch, -1.3 to -1.6 ms/step;
  // on C1's first iterations alone (the j + 2 vectors fitting) it lost
  // ≈ 0.1-0.2 ms/step, hence the whole-basis test (profiles/r05/ab_log.md).
  const bool basis_kept = (size_t)(m1 + 1) * 12u * N <= cgs_keep_bytes;
  launch_cgs_update_norm(w, basis, binv, stride, j, H, m1, N, red.U, partial_n, stream, cgs_keep_bytes > 0,
                         !basis_kept, fuse_reduce ? &dots : nullptr, lat);
  launch_norm_givens(combine(partial_n, 1), j, H, m1, givens, g, binv, resid_hist, pin, stream);
  check_launch("FGMRES iteration (Schur preconditioner, V-cycle, SpMV, CGS)");
}

void Solver::drop_graphs() {
  if (graphs.empty()) return;
  sync();
  for (IterGraph& G : graphs) {
    graph_harvest(G, false);
    if (G.exec) CFD_HIP(hipGraphExecDestroy(G.exec));
    for (auto e : G.ev) CFD_HIP(hipEventDestroy(e));
  }
  graphs.clear();
}

void Solver::graph_harvest(IterGraph& G, bool discard) {
  if (!G.pending) return;
  G.pending = false;
  if (G.ev.empty() || discard) return;
  CFD_HIP(hipEventSynchronize(G.ev.back()));
  for (size_t k = 0; k + 1 < G.ev.size(); k += 2) {
    float ms = 0.0f;
    CFD_HIP(hipEventElapsedTime(&ms, G.ev[k], G.ev[k + 1]));
    prof_ms += ms;
    prof_launches++;
  }
}

void Solver::graph_harvest_all(bool discard) {
  for (IterGraph& G : graphs) graph_harvest(G, discard);
}

void Solver::run_iteration(int j, float* pin, int variant) {
  const bool use = graph_on && !dist() && !check_sync && !comm_prof;
  if (!use) {
    iteration(j, pin);
    return;
  }
  if (graph_precond != (int)constants.precond_type) {
    drop_graphs();
    graph_precond = (int)constants.precond_type;
  }
  if (graphs.empty()) graphs.resize(3 * (size_t)m);
  IterGraph& G = graphs[3 * (size_t)j + variant];
  if (G.exec && G.prof != prof) {  // timing switched on / off: capture again
    sync();
    graph_harvest(G, false);
    CFD_HIP(hipGraphExecDestroy(G.exec));
    for (auto e : G.ev) CFD_HIP(hipEventDestroy(e));
    G = IterGraph{};
  }
  if (!G.exec) {
    hipGraph_t gr = nullptr;
    CFD_HIP(hipStreamBeginCapture(stream, hipStreamCaptureModeThreadLocal));
    capturing = &G;
    // a failed capture or instantiation leaves no timing pairs behind: they
    // were never recorded, and a later capture must not append after them
    auto reset_graph = [&] {
      for (auto ev : G.ev) (void)hipEventDestroy(ev);
      G = IterGraph{};
    };
    try {
      iteration(j, pin);
    } catch (...) {
      capturing = nullptr;
      (void)hipStreamEndCapture(stream, &gr);
      if (gr) (void)hipGraphDestroy(gr);
      reset_graph();
      throw;
    }
    capturing = nullptr;
    const hipError_t ec = hipStreamEndCapture(stream, &gr);
    const hipError_t e = ec == hipSuccess ? hipGraphInstantiate(&G.exec, gr, nullptr, nullptr, 0) : ec;
    if (gr) (void)hipGraphDestroy(gr);
    if (e != hipSuccess) {
      G.exec = nullptr;
      reset_graph();
      CFD_HIP(e);
    }
    G.prof = prof;
    graph_captures++;
  }
  graph_harvest(G, false);  // the previous replay's smoother times (complete by now: a solve start synchronised)
  CFD_HIP(hipGraphLaunch(G.exec, stream));
  G.pending = true;
  graph_replays++;
}

cfd_linear_stats Solver::solve() {  // coupled_solver_fgmres.rs:1728-2448
  const Range range("fgmres solve");
  // LinearSolverStats.time = start_time.elapsed() on every exit
  // (coupled_solver_fgmres.rs:1729,1840,1867,2446): host wall time of the solve
  const auto t_start = std::chrono::steady_clock::now();
  auto elapsed = [&] { return std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count(); };
  cfd_linear_stats st{};
  const size_t n = 3 * (size_t)N;
  const float tol = cfg.fgmres_rtol, abstol = cfg.fgmres_atol;
  const bool fixed = cfg.fixed_inner > 0;
  const int lag = cfg.convergence_lag;
  ensure_fgmres();
  if (constants.precond_type == 1) ensure_amg();
  // ||b|| and the initial residual V0 = b - A x, ||V0|| in one submission and
  // one readback: the reference reads ||b|| first and skips the residual on
  // its early exit; computing it anyway only writes solver scratch (V0,
  // binv[0], g) that the next solve rewrites, so the results are unchanged
  norm_launch(rhs, 1, 0);  // -> h_pin[0]
  residual_into_v0_launch();  // -> h_pin[1]
  sync();
  const float rhs_norm = h_pin[0];
  if (rhs_norm < abstol || !std::isfinite(rhs_norm)) {
    st.residual = rhs_norm;
    st.converged = rhs_norm < abstol;
    st.diverged = !std::isfinite(rhs_norm);
    st.time_s = elapsed();
    return st;
  }
  float residual_norm = h_pin[1];
  const float target = std::fmax(tol * rhs_norm, abstol);
  if (residual_norm < target) {
    log("FGMRES: Initial guess already converged (||r|| = %s < %s)\n", e2(residual_norm).c_str(), e2(target).c_str());
    st.residual = residual_norm;
    st.converged = 1;
    st.time_s = elapsed();
    return st;
  }
  log("FGMRES: Initial residual = %s\n", e2(residual_norm).c_str());
  uint32_t total = 0;
  float final_resid = residual_norm;
  bool converged = false;
  int stagnation = 0;
  float prev_resid = residual_norm;
  const int inner_max = fixed ? std::min(cfg.fixed_inner, m) : m;
  const int outer_max = fixed ? 1 : cfg.max_outer_restarts;
  for (int outer = 0; outer < outer_max; ++outer) {
    int basis_size = 0;
    for (int j = 0; j < inner_max; ++j) {
      const Range it_range("fgmres iteration");
      basis_size = j + 1;
      ++total;
      // the residual estimate goes to one of two pinned slots, never the slot
      // of a lagged read still pending (which may carry over from the previous
      // iteration, restart or solve: the reader is never reset)
      const int wslot = inner.pending == 0 ? 1 : 0;
      run_iteration(j, fixed ? nullptr : d_pin + 64 + wslot, fixed ? 0 : 1 + wslot);
      if (fixed) continue;
      // async residual read with the lag model (async_buffer.rs)
      flush_inner();
      // k_norm_givens wrote resid_hist[j] into h_pin[64 + wslot]; the event orders the read
      CFD_HIP(hipEventRecord(ev_iter[wslot], stream));
      bool have = false;
      float check = 0.0f;
      if (lag == 0) {
        CFD_HIP(hipEventSynchronize(ev_iter[wslot]));
        inner.last = h_pin[64 + wslot];
        inner.has_last = true;
        have = true;
        check = inner.last;
      } else {
        have = inner.has_last;
        check = inner.last;
        inner.pending = wslot;
      }
      if (have && (total % 10 == 0 || check < tol * rhs_norm))
        log("FGMRES iter %u: residual = %s (target %s)\n", total, e2(check).c_str(), e2(tol * rhs_norm).c_str());
      if (have && check < tol * rhs_norm) {
        converged = true;
        break;
      }
    }
    launch_solve_triangular(H, g, y, basis_size, m1, stream);
    launch_update_x(x, zvec, stride, y, basis_size, n, stream, small_forms);  // 0: the streaming form
    check_launch("FGMRES solution update");
    if (converged) {  // async_reader.flush()
      flush_inner();
      final_resid = inner.last;
      log("FGMRES restart %d: estimated residual = %s\n", outer + 1, e2(final_resid).c_str());
      break;
    }
    residual_norm = residual_into_v0_blocking();
    final_resid = residual_norm;
    if (fixed) {
      converged = residual_norm < tol * rhs_norm;
      break;
    }
    if (residual_norm < tol * rhs_norm) {
      converged = true;
      log("FGMRES restart %d: true residual = %s (converged)\n", outer + 1, e2(residual_norm).c_str());
      break;
    }
    if (residual_norm <= 0.0f) {
      log("FGMRES: residual vanished at restart %d\n", outer + 1);
      converged = true;
      break;
    }
    const float improvement = (prev_resid - residual_norm) / prev_resid;
    if (improvement < 1e-3f) {
      if (++stagnation >= 3) {
        log("FGMRES: Stagnation detected at restart %d (residual %s)\n", outer + 1, e2(residual_norm).c_str());
        converged = true;
        break;
      }
    } else {
      stagnation = 0;
    }
    prev_resid = residual_norm;
    log("FGMRES restart %d: residual = %s (target %s)\n", outer + 1, e2(residual_norm).c_str(),
        e2(tol * rhs_norm).c_str());
  }
  log("FGMRES finished: %u iterations, residual = %s, converged = %s\n", total, e2(final_resid).c_str(),
      tf(converged));
  st.iterations = total;
  st.residual = final_resid;
  st.converged = converged;
  st.diverged = std::isnan(final_resid);
  st.time_s = elapsed();
  return st;
}

// Reference reduction order (test mode): coupled_solver.rs:504-545 literally,
// on the host -- the AoS FluidState view (8 floats per cell: u, v, p, d_p,
// grad_p, grad_component = 0) read at floats 2i, 2i + 1 (the stride bug) and
// serial f64 loops.  tot: evolution, sum u, sum v, sum u^2, sum v^2.
void Solver::evolution_reference(double tot[5]) {
  auto aos = [&](const StateView& v, std::vector<float>& out) {
    std::vector<float2> u(N), gp(N);
    std::vector<float> p(N), dp(N);
    CFD_HIP(hipMemcpyAsync(u.data(), v.u, N * sizeof(float2), hipMemcpyDeviceToHost, stream));
    CFD_HIP(hipMemcpyAsync(p.data(), v.p, N * sizeof(float), hipMemcpyDeviceToHost, stream));
    CFD_HIP(hipMemcpyAsync(dp.data(), v.dp, N * sizeof(float), hipMemcpyDeviceToHost, stream));
    CFD_HIP(hipMemcpyAsync(gp.data(), v.gp, N * sizeof(float2), hipMemcpyDeviceToHost, stream));
    sync();
    out.assign(8 * (size_t)N, 0.0f);
    for (size_t c = 0; c < N; ++c) {
      float* r = out.data() + 8 * c;
      r[0] = u[c].x;
      r[1] = u[c].y;
      r[2] = p[c];
      r[3] = dp[c];
      r[4] = gp[c].x;
      r[5] = gp[c].y;
    }
  };
  std::vector<float> cur, old;
  aos(S(), cur);
  double e = 0.0, a = 0.0, b = 0.0, aa = 0.0, bb = 0.0;
  if (have_prev) {
    aos(prev, old);
    for (size_t k = 0; k < cur.size(); ++k) {
      const float d = cur[k] - old[k];
      e += (double)(d * d);
    }
  }
  for (size_t c = 0; c < N; ++c) {
    const double u = (double)cur[2 * c], v = (double)cur[2 * c + 1];
    a += u;
    b += v;
    aa += u * u;
    bb += v * v;
  }
  tot[0] = e;
  tot[1] = a;
  tot[2] = b;
  tot[3] = aa;
  tot[4] = bb;
}

// check_evolution (coupled_solver.rs:501-580), statistics on the GPU.  The
// stride bug (§0.1-12) makes index i read record i >> 2: a distributed rank
// first fetches the records [ev_a, ev_b) its indices read from their owners.
void Solver::check_evolution() {
  StateView var = S();
  uint64_t gbase = 0, rec0 = 0;
  if (dist()) {
    std::vector<Msg> msgs;
    StateView& cur = S();
    const uint64_t c0 = topo.c0, c1 = topo.c1;
    auto add = [&](int q, bool send, uint64_t lo, uint64_t hi) {
      const size_t n = hi - lo;
      if (send) {  // owned records [lo, hi) to rank q
        const size_t o = lo - c0;
        msgs.push_back({q, cur.u + o, n * sizeof(float2), nullptr, 0});
        msgs.push_back({q, cur.p + o, n * sizeof(float), nullptr, 0});
        msgs.push_back({q, cur.dp + o, n * sizeof(float), nullptr, 0});
        msgs.push_back({q, cur.gp + o, n * sizeof(float2), nullptr, 0});
      } else {  // records [lo, hi) of rank q
        const size_t o = lo - ev_a;
        msgs.push_back({q, nullptr, 0, evrec.u + o, n * sizeof(float2)});
        msgs.push_back({q, nullptr, 0, evrec.p + o, n * sizeof(float)});
        msgs.push_back({q, nullptr, 0, evrec.dp + o, n * sizeof(float)});
        msgs.push_back({q, nullptr, 0, evrec.gp + o, n * sizeof(float2)});
      }
    };
    for (int q = 0; q < R; ++q) {
      const uint64_t qa = starts[q] >> 2, qb = ((starts[q + 1] - 1) >> 2) + 1;  // q's record range
      // what q reads from me
      const uint64_t slo = std::max(qa, c0), shi = std::min(qb, c1);
      // what I read from q
      const uint64_t rlo = std::max(ev_a, starts[q]), rhi = std::min(ev_b, starts[q + 1]);
      if (q == rk) {
        if (rlo < rhi) {
          const size_t n = rhi - rlo, so = rlo - c0, ro = rlo - ev_a;
          CFD_HIP(hipMemcpyAsync(evrec.u + ro, cur.u + so, n * sizeof(float2), hipMemcpyDeviceToDevice, stream));
          CFD_HIP(hipMemcpyAsync(evrec.p + ro, cur.p + so, n * sizeof(float), hipMemcpyDeviceToDevice, stream));
          CFD_HIP(hipMemcpyAsync(evrec.dp + ro, cur.dp + so, n * sizeof(float), hipMemcpyDeviceToDevice, stream));
          CFD_HIP(hipMemcpyAsync(evrec.gp + ro, cur.gp + so, n * sizeof(float2), hipMemcpyDeviceToDevice, stream));
        }
        continue;
      }
      if (slo < shi) add(q, true, slo, shi);
      if (rlo < rhi) add(q, false, rlo, rhi);
    }
    comm->label = kCommStateHalo;
    comm->exchange(msgs, stream);
    var = evrec;
    gbase = topo.c0;
    rec0 = ev_a;
  }
  double tot[5];
  if (ref_red) {
    evolution_reference(tot);
  } else {
    launch_evolution_partial(S(), prev, have_prev ? 1 : 0, N, var, gbase, rec0, red.U, partial_d, pstride, stream);
    double* out5 = partial_d + 5 * (size_t)pstride;
    launch_evolution_final(combine_d(partial_d, 5), out5, stream);
    check_launch("check_evolution");
    CFD_HIP(hipMemcpyAsync(tot, out5, sizeof(tot), hipMemcpyDeviceToHost, stream));
  }
  copy_state(S(), prev, 0, N, stream);
  sync();
  const double nn = (double)NG;
  const double mean_u = tot[1] / nn, mean_v = tot[2] / nn;
  const double var_u = std::fmax(tot[3] / nn - mean_u * mean_u, 0.0);
  const double var_v = std::fmax(tot[4] / nn - mean_v * mean_v, 0.0);
  variance_history.push_back({var_u, var_v});
  if (variance_history.size() > 10) variance_history.erase(variance_history.begin());
  const double evo = have_prev ? std::sqrt(tot[0] / nn) : std::numeric_limits<double>::max();
  have_prev = true;
  if (evo < 1e-6) {
    if (var_u < 1e-10 && var_v < 1e-10) {
      info.degenerate_count++;
      info.steady_state_count = 0;
    } else {
      info.steady_state_count++;
      info.degenerate_count = 0;
    }
  } else {
    info.degenerate_count = 0;
    info.steady_state_count = 0;
  }
  if (info.degenerate_count > 10) {
    log("Solution is degenerate: Velocity field is uniform and not evolving. Variance U: %s, V: %s\n",
        e2(var_u).c_str(), e2(var_v).c_str());
    info.should_stop = 1;
  }
  if (info.steady_state_count > 10) {
    log("Steady state reached. Evolution diff: %s\n", e2(evo).c_str());
    info.should_stop = 1;
  }
}

void Solver::step() {  // coupled_solver.rs:33-499
  const Range range("cfd step");
  CFD_HIP(hipSetDevice(device));
  // opt-in deviation from the frozen hierarchy
  if (cfg.amg_rebuild_interval > 0 && amg_built && amg_age >= (uint32_t)cfg.amg_rebuild_interval) {
    // numeric re-setup over the kept structure when the device setup built it
    // (CFD_AMG_SETUP=rebuild: full rebuild; both give the same hierarchy)
    const char* se = knob(Knob::AmgSetup);  // "rebuild": a full setup instead of the refresh
    if (amg_setup_path == 2 && !amg_refresh.empty() && !(se && std::strcmp(se, "rebuild") == 0))
      amg_refresh_pending = true;
    else
      drop_amg();
  }
  rotate();
  constants.component = 0;
  const int fault_rank = debug_fault_after_prepare;  // test hook, one step only
  debug_fault_after_prepare = -1;
  if (dist()) halo_state(true);  // the rotated slot's ghosts (last written 3 steps ago)
  prepare();
  if (fault_rank == rk) throw std::runtime_error("injected fault after prepare");
  const bool fixed = cfg.fixed_outer > 0;
  const int max_iters = fixed ? cfg.fixed_outer : std::max(cfg.n_outer_correctors, 10);
  const double tol_u = 1e-5, tol_p = 1e-4;
  double prev_u = std::numeric_limits<double>::max(), prev_p = std::numeric_limits<double>::max();
  LagReader outer;  // reset per step (coupled_solver.rs:119-121)
  float last_u = 0.0f, last_p = 0.0f;
  int pend = -1;
  info.total_linear_iterations = 0;
  for (int iter = 0; iter < max_iters; ++iter) {
    const Range outer_range("picard iteration");
    log("Coupled Iteration: %d\n", iter + 1);
    if (iter > 0 || constants.scheme != 0) prepare();
    assemble();
    const cfd_linear_stats ls = solve();
    log("Coupled linear solve: %u iterations, residual %s, converged=%s\n", ls.iterations, e2(ls.residual).c_str(),
        tf(ls.converged));
    info.stats_p = ls;
    info.total_linear_iterations += ls.iterations;
    if (std::isnan(ls.residual)) throw std::domain_error("Coupled Linear Solver Diverged: NaN detected in linear residual");
    // the final max-diff pair also lands in this iteration's pinned host slot
    // (h_pin + 32 + 2 (iter & 1)): the lagged read below needs no copy launch
    uint32_t* host_slot = reinterpret_cast<uint32_t*>(d_pin + 32 + 2 * (iter & 1));
    launch_update_fields(N, constants.alpha_u, constants.alpha_p, x, S().u, S().p, blockmax, maxbits,
                         dist() ? nullptr : host_slot, stream);
    check_launch("update_fields");
    if (dist()) {
      halo_state(false);  // the next prepare reads neighbours' u, p
      timed_gather(kCommReduceGather, 2 * sizeof(uint32_t),
                   [&] { comm->allgather(maxbits, mx_gather, 2 * sizeof(uint32_t), stream); });
      launch_max_combine(mx_gather, R, maxbits, host_slot, stream);
    }
    if (iter == 0) {
      info.outer_residual_u = std::numeric_limits<float>::max();
      info.outer_residual_p = std::numeric_limits<float>::max();
      info.outer_iterations = 1;
      continue;
    }
    // async max-diff read (coupled_solver.rs:396-479) under the lag model
    float* slot = h_pin + 32 + 2 * (iter & 1);
    if (pend >= 0) {
      CFD_HIP(hipEventSynchronize(ev_outer[pend]));
      std::memcpy(&last_u, h_pin + 32 + 2 * pend, 4);
      std::memcpy(&last_p, h_pin + 32 + 2 * pend + 1, 4);
      outer.has_last = true;
      pend = -1;
    }
    CFD_HIP(hipEventRecord(ev_outer[iter & 1], stream));  // orders the read of slot
    bool have = false;
    float cu = 0.0f, cp = 0.0f;
    if (cfg.convergence_lag == 0) {
      CFD_HIP(hipEventSynchronize(ev_outer[iter & 1]));
      std::memcpy(&cu, slot, 4);
      std::memcpy(&cp, slot + 1, 4);
      have = true;
    } else {
      have = outer.has_last;
      cu = last_u;
      cp = last_p;
      pend = iter & 1;
    }
    if (!have) continue;
    const double du = cu, dp = cp;
    if (std::isnan(du) || std::isnan(dp)) throw std::domain_error("Coupled Solver Diverged: NaN detected in outer residuals");
    info.outer_residual_u = cu;
    info.outer_residual_p = cp;
    info.outer_iterations = iter + 1;
    log("Coupled Residuals - U: %s, P: %s\n", e2(du).c_str(), e2(dp).c_str());
    if (!fixed) {
      if (du < tol_u && dp < tol_p) {
        log("Coupled Solver Converged in %d iterations\n", iter + 1);
        break;
      }
      const double rel_u = (std::isfinite(prev_u) && std::fabs(prev_u) > 1e-14) ? std::fabs((du - prev_u) / prev_u)
                                                                                : std::numeric_limits<double>::infinity();
      const double rel_p = (std::isfinite(prev_p) && std::fabs(prev_p) > 1e-14) ? std::fabs((dp - prev_p) / prev_p)
                                                                                : std::numeric_limits<double>::infinity();
      if (rel_u < 1e-2 && rel_p < 1e-2 && iter > 2) {
        log("Coupled solver stagnated at iter %d: U=%s, P=%s\n", iter + 1, e2(du).c_str(), e2(dp).c_str());
        break;
      }
    }
    prev_u = du;
    prev_p = dp;
  }
  constants.time += constants.dt;
  if (amg_built) ++amg_age;
  check_evolution();
}

// ------------------------------------------------------------------ debug
void Solver::debug_prepare_assemble(bool asmb) {
  CFD_HIP(hipSetDevice(device));
  constants.component = 0;
  prepare();
  if (asmb) assemble();
  sync();
}

uint64_t Solver::amg_level_digest(int li) {
  if (li < 0 || li >= (int)levels.size()) throw std::invalid_argument("no such AMG level");
  CFD_HIP(hipSetDevice(device));
  const AmgLevelDev& d = levels[li].dev;
  uint64_t h = 1469598103934665603ull;
  auto mix = [&](const void* p, size_t bytes) {
    const unsigned char* b = static_cast<const unsigned char*>(p);
    for (size_t k = 0; k < bytes; ++k) h = (h ^ b[k]) * 1099511628211ull;
  };
  auto dev = [&](const void* src, size_t bytes) {
    if (!src || !bytes) return;
    std::vector<unsigned char> tmp(bytes);
    CFD_HIP(hipMemcpyAsync(tmp.data(), src, bytes, hipMemcpyDeviceToHost, stream));
    sync();
    mix(tmp.data(), bytes);
  };
  const uint32_t hdr[6] = {d.n, d.stride, (uint32_t)d.w, (uint32_t)d.use16, d.nc, (uint32_t)levels[li].nnz};
  mix(hdr, sizeof(hdr));
  const size_t slots = (size_t)std::max(d.w, 1) * d.stride;
  dev(d.val, slots * 4);
  dev(d.col16, d.use16 ? slots * 2 : 0);
  dev(d.col32, d.use16 ? 0 : slots * 4);
  dev(d.len, d.stride);
  dev(d.drank, d.stride);
  dev(d.dv, (size_t)d.stride * 4);
  dev(d.de, (size_t)d.stride * 4);
  if (d.nc) {
    dev(d.agg, (size_t)d.stride * 4);
    std::vector<uint32_t> rr((size_t)d.nc + 1);
    CFD_HIP(hipMemcpyAsync(rr.data(), d.r_row, rr.size() * 4, hipMemcpyDeviceToHost, stream));
    sync();
    mix(rr.data(), rr.size() * 4);
    dev(d.r_col, (size_t)rr[d.nc] * 4);
  }
  return h;
}

size_t Solver::debug_len(int id) const {
  const size_t n = N;
  switch (id) {
    case 0: return F;
    case 1: case 2: case 10: case 11: case 12: return 2 * n;
    case 3: case 4: return 3 * n;
    case 5: case 6: case 7: return n;
    case 8: return topo.scol.size();
    case 9: return 9 * topo.scol.size();
    default: return 0;
  }
}

void Solver::debug_buffer(int id, float* out) {
  CFD_HIP(hipSetDevice(device));
  if (dist() && (id == 0 || id == 8 || id == 9))
    throw std::invalid_argument("debug buffers 0/8/9 use the global face/CSR layout (single GPU only)");
  const size_t n = N;
  auto d2h = [&](void* dst, const void* src, size_t bytes) {
    CFD_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, stream));
    sync();
  };
  switch (id) {
    case 0: {  // fluxes[face] as written by the owner (prepare_coupled.wgsl:197-200)
      std::vector<float> fsv((size_t)topo.wf * n);
      d2h(fsv.data(), flux_s, fsv.size() * 4);
      std::fill(out, out + F, 0.0f);
      for (size_t e = 0; e < fsv.size(); ++e) {
        const uint32_t i = (uint32_t)(e % n), k = (uint32_t)(e / n);
        if (k < topo.nface[i] && (topo.fs_meta[e] & kMetaOwner)) out[topo.fs_face[e]] = fsv[e];
      }
      break;
    }
    case 1: d2h(out, grad_u, 2 * n * 4); break;
    case 2: d2h(out, grad_v, 2 * n * 4); break;
    case 3: d2h(out, rhs, 3 * n * 4); break;
    case 4: d2h(out, x, 3 * n * 4); break;
    case 5: case 6: d2h(out, dinv_uv, n * 4); break;
    case 7: d2h(out, dinv_p, n * 4); break;
    case 8: {
      const size_t ld = topo.ld;
      std::vector<float> ell((size_t)topo.ws * ld);
      d2h(ell.data(), sval, ell.size() * 4);
      for (uint32_t i = 0; i < N; ++i)
        for (uint32_t k = topo.srow[i]; k < topo.srow[i + 1]; ++k) out[k] = ell[(size_t)(k - topo.srow[i]) * ld + i];
      break;
    }
    case 9: {  // expand compressed blocks to the reference CSR (init/linear_solver/mod.rs:180-216)
      const size_t ld = topo.ld;
      std::vector<float2> ca((size_t)topo.ws * ld), cg((size_t)topo.ws * ld);
      std::vector<float2> d2(n);
      d2h(ca.data(), cval_a, ca.size() * sizeof(float2));
      d2h(cg.data(), cval_g, cg.size() * sizeof(float2));
      d2h(d2.data(), cdiag2, n * sizeof(float2));
      for (uint32_t i = 0; i < N; ++i) {
        const uint32_t so = topo.srow[i], nb = topo.srow[i + 1] - so;
        const uint32_t r0 = 9 * so, r1 = r0 + 3 * nb, r2 = r0 + 6 * nb;
        for (uint32_t r = 0; r < nb; ++r) {
          const size_t e = (size_t)topo.tslot[so + r] * ld + i;  // aligned slot of CSR entry r
          const float2 a = ca[e], gg = cg[e];
          const bool diag = (r == topo.ell_drank[i]);
          out[r0 + 3 * r + 0] = a.x;
          out[r0 + 3 * r + 1] = 0.0f;
          out[r0 + 3 * r + 2] = gg.x;
          out[r1 + 3 * r + 0] = 0.0f;
          out[r1 + 3 * r + 1] = a.x;
          out[r1 + 3 * r + 2] = gg.y;
          out[r2 + 3 * r + 0] = diag ? d2[i].x : gg.x;
          out[r2 + 3 * r + 1] = diag ? d2[i].y : gg.y;
          out[r2 + 3 * r + 2] = a.y;
        }
      }
      break;
    }
    case 10: d2h(out, S().gp, 2 * n * 4); break;
    case 11: d2h(out, ring[i_old].u, 2 * n * 4); break;
    case 12: d2h(out, ring[i_old_old].u, 2 * n * 4); break;
    default: throw std::invalid_argument("unknown debug buffer id");
  }
}

// ------------------------------------------------------------- accounting
// algorithmic bytes of one level-ℓ smoother sweep in the
// reference CSR/f32/u32 format: 4(n+1) + 8 nnz + 12 n.
double Solver::smoother_bytes() const {
  if (levels.empty()) return 0.0;
  const double n = levels[0].dev.n, nnz = (double)levels[0].nnz;
  return 4.0 * (n + 1.0) + 8.0 * nnz + 12.0 * n;
}

// Layout-true bytes of one level-0 sweep of k_amg_smooth: what the kernel
// must move in the AmgLevelDev image -- the u8 row lengths, every ELL slot's
// value and column (16-bit delta or i32) over the padded rows, b, x, the
// smoother diagonal and x_out (4 B each per row; the x gathers at the
// neighbours counted once, as SURVEY §8(d) counts them).  At C2 (w = 4,
// 16-bit deltas) 41 B per row against the reference format's 56.
double Solver::smoother_layout_bytes() const {
  if (levels.empty()) return 0.0;
  const AmgLevelDev& d = levels[0].dev;
  const double st = d.stride, n = d.n;
  return st + std::max(d.w, 1) * st * (4.0 + (d.use16 ? 2.0 : 4.0)) + 16.0 * n;
}

// Layout-true bytes of one step under the fixed schedule: per kernel, the
// bytes its arrays in THIS library's layouts must move (each element once:
// neighbour gathers counted once, as SURVEY §8(d) counts them), times its
// launches per step: the minimum traffic at kernel level.  It is not a lower
// bound of the HBM traffic: the kernel order is tuned so that some lines come
// from the Infinity Cache, so the PMC step traffic
// (step_counter_traffic) can be below it.
double Solver::layout_step_bytes() const {
  const double Nn = N;
  double S = 0.0, Sint = 0.0;  // used face slots, internal ones
  for (uint32_t i = 0; i < N; ++i) S += topo.nface[i];
  for (uint32_t li = 0; li < N; ++li) Sint += (double)(topo.srow[li + 1] - topo.srow[li]) - 1.0;
  const double ws = topo.ws;
  const int K = cfg.fixed_outer > 0 ? cfg.fixed_outer : std::max(cfg.n_outer_correctors, 10);
  const int M = cfg.fixed_inner > 0 ? std::min(cfg.fixed_inner, m) : m;
  const double prep = 40 * S + 60 * Nn;                    // 9 slot arrays + flux out; cell state in, gradients out
  const double asmb = 32 * S + 20 * Sint + 78 * Nn;        // 8 slot arrays; 3x3 block + Poisson entry out
  const double spmv = (35 + 16 * ws) * Nn;                 // headers, cval_a + cval_g slots, x, y
  const double predict = (39 + 8 * ws) * Nn;               // headers, cval_g slots, V_j, dinv, temp_p / p_sol out
  const double correct = (34 + 8 * ws) * Nn;               // lg, cval_g slots, p_sol, V_j, dinv, Z_j out
  // one V-cycle over the level images (as v_cycle launches them)
  double vc = 0.0;
  const int L = (int)levels.size();
  const int down = std::min(std::max(tail_first, 1), L - 1);
  auto row_image = [&](const AmgLevelDev& d) {  // ELL values + columns over the padded rows
    return std::max(d.w, 1) * (double)d.stride * (4.0 + (d.use16 ? 2.0 : 4.0));
  };
  for (int i = 0; i < L; ++i) {
    const AmgLevelDev& d = levels[i].dev;
    const double n = d.n, st = d.stride, img = row_image(d);
    const double smooth = st + img + 16 * n;
    if (i < down) {
      const double nc = levels[i + 1].dev.n;
      // pre-smoother (coarse: zero-x, elementwise; not launched when fused into
      // the previous level's restriction, whose 12 nc term counts it)
      const bool presmoothed = i > 0 && (!levels[i - 1].dist || levels[i].dist);
      vc += (i == 0 ? smooth : (presmoothed ? 0.0 : 12 * n));
      if (d.rr_agg && !levels[i].dist)
        vc += 4 * nc + 4 * n + 2 * st + img + 14 * n + 12 * nc;       // fused residual + restriction
      if (i > 0 && (size_t)i <= rr_pair.size() && rr_pair[i - 1].nblocks)
        vc -= 8 * n;  // second level of a k_amg_resrestrict_pair: its b and x stay in LDS
      if ((size_t)i < up_pair.size() && up_pair[i].nblocks)
        vc -= 8 * n;  // coarse level of a k_amg_prolong_smooth_pair: its smoothed x stays in LDS
      else
        vc += (2 * st + img + 16 * n) + (16 * nc + 4 * n + 12 * nc);  // residual, restriction
      if (fused_prolong(i))
        vc += smooth + 4 * n + 4 * nc;                                 // post-smoother reading x + P xc
      else
        vc += (12 * n + 4 * nc) + smooth;                              // prolongation, post-smoother
    } else if (i == down) {
      vc += 4.0 * tail_blob_words + 16.0 * tail_vec_floats;            // single-workgroup tail (LDS image in)
    }
  }
  double inner = 0.0;
  for (int j = 0; j < M; ++j) {
    inner += predict + vc + correct + spmv;
    inner += (j + 2) * 12.0 * Nn + (j + 3) * 12.0 * Nn;    // CGS dots, CGS update + norm
  }
  const double residual = spmv + 12 * Nn + 12 * Nn;       // SpMV storing b - A x (b read), norm
  const double solve = 12 * Nn + residual + inner + (M + 2) * 12.0 * Nn + residual;
  return K * (prep + asmb + solve + 36 * Nn);  // prepare: once per Picard iteration (scheme 0)
}

double Solver::algorithmic_step_bytes() const {
  const double Nn = N, Fn = F, S = (double)topo.srow[N] - 0.0;  // nnz_s
  double Sfaces = 0.0;
  for (uint32_t i = 0; i < N; ++i) Sfaces += topo.nface[i];
  const double nnz_s = S;
  const double prep = 84 * Nn + 4 * Sfaces + 36 * Fn;
  const double asmb = 68 * Nn + 8 * Sfaces + 36 * Fn + 40 * nnz_s;
  const int K = cfg.fixed_outer > 0 ? cfg.fixed_outer : std::max(cfg.n_outer_correctors, 10);
  const int M = cfg.fixed_inner > 0 ? std::min(cfg.fixed_inner, m) : m;
  // V-cycle bytes
  double vc = 0.0;
  for (size_t li = 0; li < levels.size(); ++li) {
    const double n = levels[li].dev.n, nnz = (double)levels[li].nnz;
    const double bs = 4 * (n + 1) + 8 * nnz + 12 * n;
    if (li + 1 < levels.size()) {
      const double nc = levels[li + 1].dev.n;
      const double br = 4 * (n + 1) + 8 * nnz + 8 * n + 4 * (nc + 1) + 8 * n + 4 * nc;
      const double bp = 4 * (n + 1) + 8 * n + 8 * n + 4 * nc;
      vc += 2 * bs + br + bp + 4 * nc;
    } else {
      vc += 10 * bs;
    }
  }
  double inner = 0.0;
  for (int j = 0; j < M; ++j) {
    inner += 36 * Nn + 72 * nnz_s;                       // SpMV
    inner += (j + 1) * 24.0 * Nn + 36 * Nn;              // CGS
    inner += 12 * Nn + 24 * Nn;                          // norm + scale
    inner += 52 * Nn + 24 * nnz_s + 48 * Nn + 48 * nnz_s + vc;  // preconditioner
  }
  const double solve = inner + M * 36.0 * Nn + 2 * (36 * Nn + 72 * nnz_s) + 36 * Nn + 3 * 12 * Nn;
  return prep + K * (prep + asmb + solve + 36 * Nn);
}

}  // namespace cfd2
