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
#include <cmath>
#include <cstdio>
#include <cstring>
#include <limits>

#include "solver_impl.hpp"

namespace cfd2 {

namespace {
constexpr int kScalBase = 0;   // dsc[0..15]: rhs_norm, resid, inv_resid, wnorm, inv_w, resid_est
constexpr int kHOff = 16;
}  // namespace

Solver::Solver(const cfd_mesh_view& mesh, const cfd_config& c, int dev) : cfg(c), device(dev) {
  if (cfg.max_restart < 1 || cfg.max_restart > 63) throw std::invalid_argument("max_restart must be 1..63");
  m = cfg.max_restart;
  m1 = m + 1;
  build_topology(mesh, topo);
  N = topo.N;
  F = topo.F;
  nchunks = (N + kRedChunkCells - 1) / kRedChunkCells;
  CFD_HIP(hipSetDevice(device));
  CFD_HIP(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
  const size_t Nz = N;
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
  // fields (init/fields.rs:62-139): zero-initialised
  auto zeros_state = [&](StateView& v) {
    v.u = arena.alloc<float2>(Nz);
    v.p = arena.alloc<float>(Nz);
    v.dp = arena.alloc<float>(Nz);
    v.gp = arena.alloc<float2>(Nz);
    CFD_HIP(hipMemsetAsync(v.u, 0, Nz * sizeof(float2), stream));
    CFD_HIP(hipMemsetAsync(v.p, 0, Nz * sizeof(float), stream));
    CFD_HIP(hipMemsetAsync(v.dp, 0, Nz * sizeof(float), stream));
    CFD_HIP(hipMemsetAsync(v.gp, 0, Nz * sizeof(float2), stream));
  };
  for (auto& r : ring) zeros_state(r);
  zeros_state(prev);
  dp_scratch = arena.alloc<float>(Nz);
  gp_scratch = arena.alloc<float2>(Nz);
  const size_t slots_f = (size_t)topo.wf * Nz, slots_s = (size_t)topo.ws * Nz;
  flux_s = arena.alloc<float>(slots_f);
  CFD_HIP(hipMemsetAsync(flux_s, 0, slots_f * sizeof(float), stream));
  grad_u = arena.alloc<float2>(Nz);
  grad_v = arena.alloc<float2>(Nz);
  CFD_HIP(hipMemsetAsync(grad_u, 0, Nz * sizeof(float2), stream));
  CFD_HIP(hipMemsetAsync(grad_v, 0, Nz * sizeof(float2), stream));
  cval_a = arena.alloc<float2>(slots_s);
  cval_g = arena.alloc<float2>(slots_s);
  CFD_HIP(hipMemsetAsync(cval_a, 0, slots_s * sizeof(float2), stream));
  CFD_HIP(hipMemsetAsync(cval_g, 0, slots_s * sizeof(float2), stream));
  cdiag2 = arena.alloc<float2>(Nz);
  CFD_HIP(hipMemsetAsync(cdiag2, 0, Nz * sizeof(float2), stream));
  sval = arena.alloc<float>(slots_s);
  CFD_HIP(hipMemsetAsync(sval, 0, slots_s * sizeof(float), stream));
  rhs = arena.alloc<float>(3 * Nz);
  x = arena.alloc<float>(3 * Nz);
  CFD_HIP(hipMemsetAsync(rhs, 0, 3 * Nz * sizeof(float), stream));
  CFD_HIP(hipMemsetAsync(x, 0, 3 * Nz * sizeof(float), stream));
  dinv_uv = arena.alloc<float>(Nz);
  dinv_p = arena.alloc<float>(Nz);
  CFD_HIP(hipMemsetAsync(dinv_uv, 0, Nz * sizeof(float), stream));
  CFD_HIP(hipMemsetAsync(dinv_p, 0, Nz * sizeof(float), stream));
  partial_d = arena.alloc<double>(5 * (size_t)nchunks + 5);
  maxbits = arena.alloc<uint32_t>(4);
  blockmax = arena.alloc<uint32_t>(2 * (((size_t)N + 255) / 256) + 2);
  CFD_HIP(hipHostMalloc((void**)&h_pin, 4096 * sizeof(float), hipHostMallocDefault));
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
  for (auto e : ev_iter) (void)hipEventDestroy(e);
  for (auto e : ev_outer)
    if (e) (void)hipEventDestroy(e);
  for (auto e : prof_ev) (void)hipEventDestroy(e);
  if (h_pin) (void)hipHostFree(h_pin);
  arena.release();
  if (stream) (void)hipStreamDestroy(stream);
}

CoupledMatrix Solver::cmat() const {
  CoupledMatrix A;
  A.N = N;
  A.ws = topo.ws;
  A.col = d_scol;
  A.len = d_slen;
  A.drank = d_sdrank;
  A.cval_a = cval_a;
  A.cval_g = cval_g;
  A.cdiag2 = cdiag2;
  return A;
}

// ---------------------------------------------------------------- state API
void Solver::set_u(const double* uv) {  // solver.rs:9-21 (clobbers the whole state)
  std::vector<float2> u(N);
  for (uint32_t i = 0; i < N; ++i) u[i] = make_float2((float)uv[2 * i], (float)uv[2 * i + 1]);
  StateView& s = S();
  CFD_HIP(hipMemcpyAsync(s.u, u.data(), N * sizeof(float2), hipMemcpyHostToDevice, stream));
  CFD_HIP(hipMemsetAsync(s.p, 0, N * sizeof(float), stream));
  CFD_HIP(hipMemsetAsync(s.dp, 0, N * sizeof(float), stream));
  CFD_HIP(hipMemsetAsync(s.gp, 0, N * sizeof(float2), stream));
  sync();
}

void Solver::set_p(const double* pv) {  // solver.rs:23-34
  std::vector<float> p(N);
  for (uint32_t i = 0; i < N; ++i) p[i] = (float)pv[i];
  StateView& s = S();
  CFD_HIP(hipMemsetAsync(s.u, 0, N * sizeof(float2), stream));
  CFD_HIP(hipMemcpyAsync(s.p, p.data(), N * sizeof(float), hipMemcpyHostToDevice, stream));
  CFD_HIP(hipMemsetAsync(s.dp, 0, N * sizeof(float), stream));
  CFD_HIP(hipMemsetAsync(s.gp, 0, N * sizeof(float2), stream));
  sync();
}

static void copy_state(const StateView& src, StateView& dst, uint32_t N, hipStream_t s) {
  CFD_HIP(hipMemcpyAsync(dst.u, src.u, N * sizeof(float2), hipMemcpyDeviceToDevice, s));
  CFD_HIP(hipMemcpyAsync(dst.p, src.p, N * sizeof(float), hipMemcpyDeviceToDevice, s));
  CFD_HIP(hipMemcpyAsync(dst.dp, src.dp, N * sizeof(float), hipMemcpyDeviceToDevice, s));
  CFD_HIP(hipMemcpyAsync(dst.gp, src.gp, N * sizeof(float2), hipMemcpyDeviceToDevice, s));
}

void Solver::initialize_history() {  // solver.rs:276-294
  copy_state(ring[i_state], ring[i_old], N, stream);
  copy_state(ring[i_state], ring[i_old_old], N, stream);
  sync();
}

void Solver::get_u(double* uv) {
  std::vector<float2> u(N);
  CFD_HIP(hipMemcpyAsync(u.data(), S().u, N * sizeof(float2), hipMemcpyDeviceToHost, stream));
  sync();
  for (uint32_t i = 0; i < N; ++i) {
    uv[2 * i] = u[i].x;
    uv[2 * i + 1] = u[i].y;
  }
}

void Solver::get_p(double* out) {
  std::vector<float> p(N);
  CFD_HIP(hipMemcpyAsync(p.data(), S().p, N * sizeof(float), hipMemcpyDeviceToHost, stream));
  sync();
  for (uint32_t i = 0; i < N; ++i) out[i] = p[i];
}

void Solver::get_d_p(double* out) {
  std::vector<float> p(N);
  CFD_HIP(hipMemcpyAsync(p.data(), S().dp, N * sizeof(float), hipMemcpyDeviceToHost, stream));
  sync();
  for (uint32_t i = 0; i < N; ++i) out[i] = p[i];
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
  launch_prepare(a, stream);
  // commit d_p / grad_p (snapshot semantics): swap the scratch into the slot
  std::swap(S().dp, dp_scratch);
  std::swap(S().gp, gp_scratch);
}

void Solver::assemble() {
  AssembleArgs a;
  a.N = N;
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
  a.cval_a = cval_a;
  a.cval_g = cval_g;
  a.cdiag2 = cdiag2;
  a.sval = sval;
  a.rhs = rhs;
  a.dinv_uv = dinv_uv;
  a.dinv_p = dinv_p;
  launch_assemble(a, stream);
}

void Solver::ensure_fgmres() {  // coupled_solver_fgmres.rs:212-1280 (lazy)
  if (fgmres_ready) return;
  const size_t n = 3 * (size_t)N;
  stride = (n + 63) & ~(size_t)63;  // 256-byte aligned basis rows
  basis = arena.alloc<float>((size_t)m1 * stride);
  zvec = arena.alloc<float>((size_t)m * stride);
  w = arena.alloc<float>(n);
  // pressure vectors are padded to a multiple of 64 (zeroed): the AMG level-0
  // kernels process 4 rows per thread with 16-byte loads
  const size_t np = ((size_t)N + 63) & ~(size_t)63;
  temp = arena.alloc<float>(np);
  temp_p = arena.alloc<float>(np);
  p_sol = arena.alloc<float>(np);
  CFD_HIP(hipMemsetAsync(basis, 0, (size_t)m1 * stride * sizeof(float), stream));
  CFD_HIP(hipMemsetAsync(zvec, 0, (size_t)m * stride * sizeof(float), stream));
  CFD_HIP(hipMemsetAsync(w, 0, n * sizeof(float), stream));
  CFD_HIP(hipMemsetAsync(temp, 0, np * sizeof(float), stream));
  CFD_HIP(hipMemsetAsync(temp_p, 0, np * sizeof(float), stream));
  CFD_HIP(hipMemsetAsync(p_sol, 0, np * sizeof(float), stream));
  partial = arena.alloc<float>((size_t)m1 * nchunks);
  partial_n = arena.alloc<float>(nchunks);
  const size_t nsc = kHOff + (size_t)m1 * m + 2 * (size_t)m + m1 + m + m + m1;
  dsc = arena.alloc<float>(nsc);
  CFD_HIP(hipMemsetAsync(dsc, 0, nsc * sizeof(float), stream));
  H = dsc + kHOff;
  givens = H + (size_t)m1 * m;
  g = givens + 2 * m;
  y = g + m1;
  resid_hist = y + m;
  binv = resid_hist + m;
  ev_iter.resize(m);
  for (auto& e : ev_iter) CFD_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  fgmres_ready = true;
}

// ensure_amg_resources (coupled_solver_fgmres.rs:174-209): read back the live
// scalar matrix, build the frozen hierarchy on the host, upload it.
void Solver::ensure_amg() {
  if (amg_built) return;
  std::vector<float> ell((size_t)topo.ws * N);
  CFD_HIP(hipMemcpyAsync(ell.data(), sval, ell.size() * sizeof(float), hipMemcpyDeviceToHost, stream));
  sync();
  HostCsr A0;
  A0.rows = A0.cols = N;
  A0.row = topo.srow;
  A0.col = topo.scol;
  A0.val.resize(topo.scol.size());
  for (uint32_t i = 0; i < N; ++i)
    for (uint32_t k = topo.srow[i]; k < topo.srow[i + 1]; ++k)
      A0.val[k] = ell[(size_t)(k - topo.srow[i]) * N + i];
  std::vector<AmgHostLevel> H0 = build_amg_hierarchy(A0, kMaxAmgLevels);
  levels.clear();
  for (size_t li = 0; li < H0.size(); ++li) {
    const AmgHostLevel& L = H0[li];
    const uint32_t n = (uint32_t)L.A.rows;
    const uint32_t st = (n + 63) & ~63u;  // padded row count (16-byte row groups)
    int wmax = 0;
    bool small_delta = true;
    std::vector<uint8_t> len(st, 0), drank(st, 0);
    std::vector<float> dv(st, 0.0f), de(st, 1.0f);
    for (uint32_t i = 0; i < n; ++i) {
      uint32_t off = 0, dr = 0;
      bool has = false;
      float diag = 1.0f, raw = 0.0f;
      for (uint32_t k = L.A.row[i]; k < L.A.row[i + 1]; ++k) {
        const uint32_t c = L.A.col[k];
        if (c == i) {
          has = true;
          raw = L.A.val[k];
          diag = raw;
          dr = off;
        } else {
          ++off;
          const int64_t d = (int64_t)c - (int64_t)i;
          if (d < -32768 || d > 32767) small_delta = false;
        }
      }
      if (!has) dr = off;  // no diagonal entry: raw diag contributes nothing (dv = 0)
      if (std::fabs(diag) < 1e-14f) diag = 1.0f;  // amg.wgsl:46
      if (off > 255) throw std::domain_error("AMG level row wider than 255 entries");
      len[i] = (uint8_t)off;
      drank[i] = (uint8_t)dr;
      dv[i] = raw;
      de[i] = diag;
      wmax = std::max(wmax, (int)off);
    }
    const size_t slots = (size_t)std::max(wmax, 1) * st;
    std::vector<float> val(slots, 0.0f);
    std::vector<int16_t> col16(small_delta ? slots : 0, 0);
    std::vector<uint32_t> col32(small_delta ? 0 : slots, 0);
    for (uint32_t i = 0; i < st; ++i) {
      uint32_t r = 0;
      if (i < n)
        for (uint32_t k = L.A.row[i]; k < L.A.row[i + 1]; ++k) {
          const uint32_t c = L.A.col[k];
          if (c == i) continue;
          const size_t o = (size_t)r * st + i;
          val[o] = L.A.val[k];
          if (small_delta)
            col16[o] = (int16_t)((int64_t)c - (int64_t)i);
          else
            col32[o] = c;
          ++r;
        }
      // padding slots: value 0, column = own row (delta 0; padding rows read x[i],
      // which is allocated and zero-initialised)
      if (!small_delta)
        for (; r < (uint32_t)std::max(wmax, 1); ++r) col32[(size_t)r * st + i] = std::min(i, n - 1);
    }
    if (small_delta)  // padding rows must not point past n-1 either
      for (uint32_t i = n; i < st; ++i)
        for (int r = 0; r < std::max(wmax, 1); ++r) col16[(size_t)r * st + i] = 0;
    AmgGpuLevel G;
    G.nnz = L.A.col.size();
    G.dev.n = n;
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
    G.dev.nc = L.has_op ? L.nc : 0;
    if (L.has_op) {
      std::vector<uint32_t> agg(st, 0);
      std::copy(L.agg.begin(), L.agg.end(), agg.begin());
      G.dev.agg = arena.upload(agg, stream);
      G.dev.r_row = arena.upload(L.r_row, stream);
      G.dev.r_col = arena.upload(L.r_col, stream);
    }
    auto zeroed = [&](size_t cnt) {
      float* p = arena.alloc<float>(cnt);
      CFD_HIP(hipMemsetAsync(p, 0, cnt * sizeof(float), stream));
      return p;
    };
    G.xt = zeroed(st);
    G.r = zeroed(st);
    if (li > 0) {
      G.x = zeroed(st);
      G.b = zeroed(st);
    }
    levels.push_back(G);
  }
  // levels from `tail_first` down run inside one single-workgroup kernel
  const char* env = std::getenv("CFD_AMG_TAIL_ROWS");
  const uint32_t tail_rows = env ? (uint32_t)std::strtoul(env, nullptr, 10) : 4096u;
  tail_first = (int)levels.size();
  while (tail_first > 1 && levels[tail_first - 1].dev.n <= tail_rows) --tail_first;
  std::vector<AmgTailLevel> tl(levels.size());
  for (size_t li = 0; li < levels.size(); ++li) {
    tl[li].L = levels[li].dev;
    tl[li].x = levels[li].x;
    tl[li].xt = levels[li].xt;
    tl[li].b = levels[li].b;
    tl[li].r = levels[li].r;
  }
  d_tail = arena.upload(tl, stream);
  sync();
  amg_built = true;
}

void Solver::amg_smooth(size_t li, float*& xcur, const float* b) {
  AmgGpuLevel& L = levels[li];
  const bool timed = prof && li == 0;
  if (timed) {
    if (prof_used + 2 > prof_ev.size()) {  // drain the pool
      CFD_HIP(hipStreamSynchronize(stream));
      for (size_t k = 0; k + 1 < prof_used; k += 2) {
        float ms = 0.0f;
        CFD_HIP(hipEventElapsedTime(&ms, prof_ev[k], prof_ev[k + 1]));
        prof_ms += ms;
      }
      prof_used = 0;
      while (prof_ev.size() < 512) {
        hipEvent_t e;
        CFD_HIP(hipEventCreate(&e));
        prof_ev.push_back(e);
      }
    }
    CFD_HIP(hipEventRecord(prof_ev[prof_used], stream));
  }
  launch_amg_smooth(L.dev, xcur, b, L.xt, stream);
  if (timed) {
    CFD_HIP(hipEventRecord(prof_ev[prof_used + 1], stream));
    prof_used += 2;
    prof_launches++;
  }
  std::swap(xcur, L.xt);  // out-of-place Jacobi: the partner buffer becomes current
}

// amg.rs:666-770, level 0 bound to (x = p_sol, b = temp_p).  Levels below
// `tail_first` (all small) run as one single-workgroup kernel (k_amg_tail).
void Solver::v_cycle() {
  const int L = (int)levels.size();
  levels[0].x = p_sol;
  levels[0].b = temp_p;
  // the tail needs level >= 1 (level 0's x/b are bound per call) and is off
  // while the level-0 smoother is being timed on a one-level hierarchy
  const int tf = (prof && L == 1) ? L : std::max(tail_first, 1);
  const int down = std::min(tf, L - 1);
  for (int i = 0; i < down; ++i) {
    amg_smooth(i, levels[i].x, levels[i].b);
    launch_amg_residual(levels[i].dev, levels[i].x, levels[i].b, levels[i].r, stream);
    launch_amg_restrict(levels[i].dev, levels[i].r, levels[i + 1].b, levels[i + 1].x, stream);
  }
  if (tf < L) {
    launch_amg_tail(d_tail, tf, L, stream);
  } else {
    for (int s = 0; s < 10; ++s) amg_smooth(L - 1, levels[L - 1].x, levels[L - 1].b);
  }
  for (int ii = down - 1; ii >= 0; --ii) {
    launch_amg_prolong(levels[ii].dev, levels[ii].x, levels[ii + 1].x, stream);
    amg_smooth(ii, levels[ii].x, levels[ii].b);
  }
  // every level performs an even number of sweeps, so level 0 ends in p_sol
  if (levels[0].x != p_sol) throw std::logic_error("AMG level-0 ping-pong parity");
}

// FGMRES Preconditioner Step (coupled_solver_fgmres.rs:1911-1994)
void Solver::precondition(int j, float* z) {
  const CoupledMatrix A = cmat();
  const bool jacobi = constants.precond_type != 1;
  const float* v = basis + (size_t)j * stride;  // V_j = binv[j] * W_j
  launch_precond_predict(A, v, binv, j, dinv_uv, dinv_p, temp_p, p_sol, jacobi ? temp : nullptr, stream);
  bool in_sol = true;
  if (!jacobi) {
    v_cycle();
  } else {
    const size_t raw = 20u + (size_t)std::sqrt((float)N) / 2u;
    const size_t p_iters = std::min<size_t>(raw, 200) == 0 ? 0 : std::min<size_t>(raw, 200) - 1;
    for (size_t it = 0; it < p_iters; ++it) {
      if (in_sol)
        launch_relax_pressure(N, topo.ws, d_scol, d_slen, sval, dinv_p, temp_p, p_sol, temp, stream);
      else
        launch_relax_pressure(N, topo.ws, d_scol, d_slen, sval, dinv_p, temp_p, temp, p_sol, stream);
      in_sol = !in_sol;
    }
  }
  launch_precond_correct(A, v, binv, j, in_sol ? p_sol : temp, dinv_uv, z, stream);
}

float Solver::norm_blocking(const float* v, int mode, int slot) {
  launch_dot_partial(v, v, N, partial_n, stream);
  launch_reduce_final(partial_n, nchunks, mode, dsc + slot, binv, mode == 2 ? g : nullptr, stream);
  CFD_HIP(hipMemcpyAsync(h_pin, dsc + slot, sizeof(float), hipMemcpyDeviceToHost, stream));
  sync();
  return h_pin[0];
}

// compute_residual_into (coupled_solver_fgmres.rs:1637-1667): V0 = b - A x, ||V0||
// V0 is stored unnormalised: binv[0] = 1/||r|| (the reference's scale_in_place),
// g = [||r||, 0, ...] (coupled_solver_fgmres.rs:1880-1890, 2380-2392).
float Solver::residual_into_v0_blocking() {
  CFD_HIP(hipMemsetAsync(g, 0, m1 * sizeof(float), stream));
  launch_spmv(cmat(), x, w, stream);
  launch_residual_axpby(rhs, w, basis, 3 * (size_t)N, stream);
  return norm_blocking(basis, 2, 1);
}

cfd_linear_stats Solver::solve() {  // coupled_solver_fgmres.rs:1728-2448
  cfd_linear_stats st{};
  const size_t n = 3 * (size_t)N;
  const float tol = cfg.fgmres_rtol, abstol = cfg.fgmres_atol;
  const bool fixed = cfg.fixed_inner > 0;
  const int lag = cfg.convergence_lag;
  ensure_fgmres();
  if (constants.precond_type == 1) ensure_amg();
  const float rhs_norm = norm_blocking(rhs, 1, 0);
  if (rhs_norm < abstol || !std::isfinite(rhs_norm)) {
    st.residual = rhs_norm;
    st.converged = rhs_norm < abstol;
    st.diverged = !std::isfinite(rhs_norm);
    return st;
  }
  float residual_norm = residual_into_v0_blocking();
  const float target = std::fmax(tol * rhs_norm, abstol);
  if (residual_norm < target) {
    st.residual = residual_norm;
    st.converged = 1;
    return st;
  }
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
      basis_size = j + 1;
      ++total;
      float* zj = zvec + (size_t)j * stride;
      precondition(j, zj);
      launch_spmv(cmat(), zj, w, stream);
      launch_cgs_dots(w, basis, binv, stride, j, N, partial, nchunks, stream);
      launch_cgs_reduce(partial, nchunks, j, H, m1, stream);
      launch_cgs_update_norm(w, basis, binv, stride, j, H, m1, N, partial_n, stream);
      launch_norm_givens(partial_n, nchunks, j, H, m1, givens, g, binv, resid_hist, stream);
      if (fixed) continue;
      // async residual read with the lag model (async_buffer.rs)
      if (inner.pending >= 0) {
        CFD_HIP(hipEventSynchronize(ev_iter[inner.pending]));
        inner.last = h_pin[64 + inner.pending];
        inner.has_last = true;
        inner.pending = -1;
      }
      CFD_HIP(hipMemcpyAsync(h_pin + 64 + j, resid_hist + j, sizeof(float), hipMemcpyDeviceToHost, stream));
      CFD_HIP(hipEventRecord(ev_iter[j], stream));
      bool have = false;
      float check = 0.0f;
      if (lag == 0) {
        CFD_HIP(hipEventSynchronize(ev_iter[j]));
        inner.last = h_pin[64 + j];
        inner.has_last = true;
        have = true;
        check = inner.last;
      } else {
        have = inner.has_last;
        check = inner.last;
        inner.pending = j;
      }
      if (have && check < tol * rhs_norm) {
        converged = true;
        break;
      }
    }
    launch_solve_triangular(H, g, y, basis_size, m1, stream);
    launch_update_x(x, zvec, stride, y, basis_size, n, stream);
    if (converged) {  // async_reader.flush()
      if (inner.pending >= 0) {
        CFD_HIP(hipEventSynchronize(ev_iter[inner.pending]));
        inner.last = h_pin[64 + inner.pending];
        inner.has_last = true;
        inner.pending = -1;
      }
      final_resid = inner.last;
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
      break;
    }
    if (residual_norm <= 0.0f) {
      converged = true;
      break;
    }
    const float improvement = (prev_resid - residual_norm) / prev_resid;
    if (improvement < 1e-3f) {
      if (++stagnation >= 3) {
        converged = true;
        break;
      }
    } else {
      stagnation = 0;
    }
    prev_resid = residual_norm;
  }
  st.iterations = total;
  st.residual = final_resid;
  st.converged = converged;
  st.diverged = std::isnan(final_resid);
  return st;
}

// check_evolution (coupled_solver.rs:501-580), statistics on the GPU
void Solver::check_evolution() {
  launch_evolution_partial(S(), prev, have_prev ? 1 : 0, N, partial_d, stream);
  double* out5 = partial_d + 5 * (size_t)nchunks;
  launch_evolution_final(partial_d, nchunks, out5, stream);
  double tot[5];
  CFD_HIP(hipMemcpyAsync(tot, out5, sizeof(tot), hipMemcpyDeviceToHost, stream));
  copy_state(S(), prev, N, stream);
  sync();
  const double nn = (double)N;
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
  if (info.degenerate_count > 10 || info.steady_state_count > 10) info.should_stop = 1;
}

void Solver::step() {  // coupled_solver.rs:33-499
  rotate();
  constants.component = 0;
  prepare();
  const bool fixed = cfg.fixed_outer > 0;
  const int max_iters = fixed ? cfg.fixed_outer : std::max(cfg.n_outer_correctors, 10);
  const double tol_u = 1e-5, tol_p = 1e-4;
  double prev_u = std::numeric_limits<double>::max(), prev_p = std::numeric_limits<double>::max();
  LagReader outer;  // reset per step (coupled_solver.rs:119-121)
  float last_u = 0.0f, last_p = 0.0f;
  int pend = -1;
  info.total_linear_iterations = 0;
  for (int iter = 0; iter < max_iters; ++iter) {
    if (iter > 0 || constants.scheme != 0) prepare();
    assemble();
    const cfd_linear_stats ls = solve();
    info.stats_p = ls;
    info.total_linear_iterations += ls.iterations;
    if (std::isnan(ls.residual)) throw std::domain_error("Coupled Linear Solver Diverged: NaN detected in linear residual");
    launch_update_fields(N, constants.alpha_u, constants.alpha_p, x, S().u, S().p, blockmax, maxbits, stream);
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
    CFD_HIP(hipMemcpyAsync(slot, maxbits, 2 * sizeof(uint32_t), hipMemcpyDeviceToHost, stream));
    CFD_HIP(hipEventRecord(ev_outer[iter & 1], stream));
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
    if (!fixed) {
      if (du < tol_u && dp < tol_p) break;
      const double rel_u = (std::isfinite(prev_u) && std::fabs(prev_u) > 1e-14) ? std::fabs((du - prev_u) / prev_u)
                                                                                : std::numeric_limits<double>::infinity();
      const double rel_p = (std::isfinite(prev_p) && std::fabs(prev_p) > 1e-14) ? std::fabs((dp - prev_p) / prev_p)
                                                                                : std::numeric_limits<double>::infinity();
      if (rel_u < 1e-2 && rel_p < 1e-2 && iter > 2) break;
    }
    prev_u = du;
    prev_p = dp;
  }
  constants.time += constants.dt;
  check_evolution();
}

// ------------------------------------------------------------------ debug
void Solver::debug_prepare_assemble(bool asmb) {
  constants.component = 0;
  prepare();
  if (asmb) assemble();
  sync();
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
      std::vector<float> ell((size_t)topo.ws * n);
      d2h(ell.data(), sval, ell.size() * 4);
      for (uint32_t i = 0; i < N; ++i)
        for (uint32_t k = topo.srow[i]; k < topo.srow[i + 1]; ++k) out[k] = ell[(size_t)(k - topo.srow[i]) * n + i];
      break;
    }
    case 9: {  // expand compressed blocks to the reference CSR (init/linear_solver/mod.rs:180-216)
      std::vector<float2> ca((size_t)topo.ws * n), cg((size_t)topo.ws * n);
      std::vector<float2> d2(n);
      d2h(ca.data(), cval_a, ca.size() * sizeof(float2));
      d2h(cg.data(), cval_g, cg.size() * sizeof(float2));
      d2h(d2.data(), cdiag2, n * sizeof(float2));
      for (uint32_t i = 0; i < N; ++i) {
        const uint32_t so = topo.srow[i], nb = topo.srow[i + 1] - so;
        const uint32_t r0 = 9 * so, r1 = r0 + 3 * nb, r2 = r0 + 6 * nb;
        for (uint32_t r = 0; r < nb; ++r) {
          const float2 a = ca[(size_t)r * n + i], gg = cg[(size_t)r * n + i];
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
