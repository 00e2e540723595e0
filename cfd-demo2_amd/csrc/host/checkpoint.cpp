// Checkpoint / resume of the solver state (cfd_state_file_header in
// include/cfd2_amd.h; SURVEY §5 "Checkpoint / resume").  The reference has no
// equivalent -- its FluidState ring lives only in wgpu buffers
// (src/solver/gpu/structs.rs, coupled_solver.rs:43-71) -- so the format is
// ours: every value a step reads from earlier steps, f32 bit patterns as the
// device holds them, in GLOBAL cell order so a file written by R ranks loads
// into any rank count.
//
// Carried across steps, hence saved:
//   ring[3] (u, p, d_p, grad_p) + step_index    coupled_solver.rs:43-71
//   x (the next solve's initial guess)          coupled_solver_fgmres.rs:1728+
//   prev + have_prev + variance history + info  coupled_solver.rs:501-580
//   the lagged FGMRES residual read             async_buffer.rs
//   constants                                   structs.rs:86-101
//   the scalar matrix the AMG hierarchy was built from (the hierarchy is built
//   once, on the first AMG solve, and never refreshed: a resumed solver must
//   rebuild it from the same matrix, not from its first assembled one)
// Scratch that every step rewrites before reading (fluxes, gradients, the
// coupled matrix, FGMRES basis, AMG level vectors) is not saved.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <cstdio>
#include <cstddef>
#include <cstring>

#include "solver_impl.hpp"

namespace cfd2 {

static_assert(sizeof(cfd_state_file_header) == 512, "cfd_state_file_header layout");
static_assert(offsetof(cfd_state_file_header, variance) == 64, "cfd_state_file_header layout");
static_assert(offsetof(cfd_state_file_header, constants) == 224, "cfd_state_file_header layout");
static_assert(offsetof(cfd_state_file_header, info) == 280, "cfd_state_file_header layout");
static_assert(offsetof(cfd_state_file_header, amg_age) == 336, "cfd_state_file_header layout");
static_assert(offsetof(cfd_state_file_header, nranks) == 344, "cfd_state_file_header layout");

namespace {

constexpr char kMagic[8] = {'C', 'F', 'D', '2', 'S', 'T', 'A', 'T'};
constexpr uint32_t kVersion = 1;
constexpr uint64_t kCellFloats = 6;  // u(2) p d_p grad_p(2) per cell per FluidState

// byte offsets of the sections (all derived from num_cells and amg_nnz)
struct Layout {
  uint64_t ng, nnz;
  uint64_t state(int slot) const { return 512 + (uint64_t)slot * kCellFloats * 4 * ng; }  // slot 3 = prev
  // within a FluidState block: u[2N], p[N], d_p[N], grad_p[2N]
  static uint64_t u_off(uint64_t) { return 0; }
  static uint64_t p_off(uint64_t n) { return 8 * n; }
  static uint64_t dp_off(uint64_t n) { return 12 * n; }
  static uint64_t gp_off(uint64_t n) { return 16 * n; }
  uint64_t x() const { return state(4); }
  uint64_t rowptr() const { return x() + 12 * ng; }
  uint64_t val() const { return rowptr() + (nnz ? 8 * (ng + 1) : 0); }
  uint64_t total() const { return val() + 4 * nnz; }
};

void pwrite_all(int fd, const void* p, size_t bytes, uint64_t off) {
  const char* c = static_cast<const char*>(p);
  while (bytes) {
    const ssize_t w = ::pwrite(fd, c, bytes, (off_t)off);
    if (w < 0) {
      if (errno == EINTR) continue;
      throw std::runtime_error(std::string("state save: write failed: ") + std::strerror(errno));
    }
    c += w;
    bytes -= (size_t)w;
    off += (uint64_t)w;
  }
}

}  // namespace

void Solver::save_state(const char* path) {
  const Range range("state save");
  CFD_HIP(hipSetDevice(device));
  sync();
  // a lagged residual read still pending is part of the state: complete it
  // now (the value is the one the next read would take)
  flush_inner();
  // collective: every rank learns the AMG source size and its value offset
  // a pending refresh stands for a dropped hierarchy (the next AMG solve re-makes it)
  const bool have_amg = (amg_built && !amg_refresh_pending) || amg_src_loaded;
  const uint64_t my_nnz = have_amg ? (uint64_t)topo.scol.size() : 0;
  const std::vector<uint64_t> nz = allgather_u64(my_nnz);
  uint64_t nnz = 0, e0 = 0;
  for (int q = 0; q < R; ++q) {
    if (q == rk) e0 = nnz;
    nnz += nz[q];
  }
  const Layout L{NG, nnz};
  const uint64_t c0 = topo.c0;
  std::string err;
  int fd = ::open(path, O_WRONLY | O_CREAT, 0644);
  if (fd < 0) err = std::string("state save: cannot open ") + path + ": " + std::strerror(errno);
  try {
    if (fd >= 0) {
      if (rk == 0) {
        if (::ftruncate(fd, (off_t)L.total()) != 0)
          throw std::runtime_error(std::string("state save: ftruncate: ") + std::strerror(errno));
        cfd_state_file_header h;
        std::memset(&h, 0, sizeof(h));
        std::memcpy(h.magic, kMagic, 8);
        h.version = kVersion;
        h.header_bytes = sizeof(h);
        h.num_cells = NG;
        h.num_faces = F;
        h.amg_nnz = nnz;
        h.step_index = step_index;
        h.have_prev = have_prev ? 1 : 0;
        h.inner_has_last = inner.has_last ? 1 : 0;
        h.inner_last = inner.last;
        h.n_variance = (uint32_t)variance_history.size();
        for (size_t k = 0; k < variance_history.size(); ++k) {
          h.variance[k][0] = variance_history[k].first;
          h.variance[k][1] = variance_history[k].second;
        }
        h.constants = constants;
        h.info = info;
        h.amg_age = amg_refresh_pending ? 0 : amg_age;
        h.amg_local_aggregation = amg_local ? 1 : 0;
        h.nranks = R;
        pwrite_all(fd, &h, sizeof(h), 0);
      }
      // owned rows of every per-cell array at their global offsets
      std::vector<float> buf(3 * (size_t)N);
      auto put = [&](const void* dev, int comps, uint64_t sec) {
        const size_t bytes = (size_t)N * comps * sizeof(float);
        CFD_HIP(hipMemcpyAsync(buf.data(), dev, bytes, hipMemcpyDeviceToHost, stream));
        sync();
        pwrite_all(fd, buf.data(), bytes, sec + c0 * comps * sizeof(float));
      };
      for (int s = 0; s < 4; ++s) {
        const StateView& v = s < 3 ? ring[s] : prev;
        const uint64_t b = L.state(s);
        put(v.u, 2, b + Layout::u_off(NG));
        put(v.p, 1, b + Layout::p_off(NG));
        put(v.dp, 1, b + Layout::dp_off(NG));
        put(v.gp, 2, b + Layout::gp_off(NG));
      }
      put(x, 3, L.x());
      if (nnz) {
        // ELL image -> CSR rows (topo.srow order = ascending columns)
        const size_t ld = topo.ld;
        std::vector<float> ell((size_t)topo.ws * ld);
        CFD_HIP(hipMemcpyAsync(ell.data(), amg_src, ell.size() * sizeof(float), hipMemcpyDeviceToHost, stream));
        sync();
        std::vector<float> own(topo.scol.size());
        std::vector<uint64_t> rp((size_t)N + (rk == R - 1 ? 1 : 0));
        for (uint32_t i = 0; i < N; ++i) {
          rp[i] = e0 + topo.srow[i];
          for (uint32_t k = topo.srow[i]; k < topo.srow[i + 1]; ++k) own[k] = ell[(size_t)(k - topo.srow[i]) * ld + i];
        }
        if (rk == R - 1) rp[N] = nnz;
        pwrite_all(fd, rp.data(), rp.size() * 8, L.rowptr() + c0 * 8);
        pwrite_all(fd, own.data(), own.size() * 4, L.val() + e0 * 4);
      }
    }
  } catch (const HipError&) {
    if (fd >= 0) ::close(fd);
    throw;  // device failure: not recoverable, no point in keeping the ranks in step
  } catch (const std::exception& e) {
    err = e.what();
  }
  if (fd >= 0 && ::close(fd) != 0 && err.empty())
    err = std::string("state save: close: ") + std::strerror(errno);
  // barrier: the file is complete on every rank's return; a failure anywhere fails everywhere
  const std::vector<uint64_t> bad = allgather_u64(err.empty() ? 0 : 1);
  if (!err.empty()) throw std::runtime_error(err);
  for (int q = 0; q < R; ++q)
    if (bad[q]) throw std::runtime_error("state save failed on rank " + std::to_string(q));
}

void Solver::load_state(const char* path) {
  const Range range("state load");
  CFD_HIP(hipSetDevice(device));
  const int fd = ::open(path, O_RDONLY);
  if (fd < 0) throw std::invalid_argument(std::string("state load: cannot open ") + path + ": " + std::strerror(errno));
  struct stat st;
  if (::fstat(fd, &st) != 0 || (size_t)st.st_size < sizeof(cfd_state_file_header)) {
    ::close(fd);
    throw std::invalid_argument(std::string("state load: not a state file: ") + path);
  }
  const size_t fsize = (size_t)st.st_size;
  void* map = ::mmap(nullptr, fsize, PROT_READ, MAP_PRIVATE, fd, 0);
  ::close(fd);
  if (map == MAP_FAILED) throw std::runtime_error(std::string("state load: mmap: ") + std::strerror(errno));
  struct Unmap {
    void* p;
    size_t n;
    ~Unmap() { ::munmap(p, n); }
  } unmap{map, fsize};
  const char* base = static_cast<const char*>(map);
  cfd_state_file_header h;
  std::memcpy(&h, base, sizeof(h));
  if (std::memcmp(h.magic, kMagic, 8) != 0 || h.version != kVersion || h.header_bytes != sizeof(h))
    throw std::invalid_argument("state load: bad magic / version");
  if (h.num_cells != NG || h.num_faces != F)
    throw std::invalid_argument("state load: the file belongs to a different mesh (cells / faces differ)");
  const Layout L{NG, h.amg_nnz};
  if (L.total() != fsize) throw std::invalid_argument("state load: truncated or oversized file");
  if (h.step_index < 0 || h.step_index > 2 || h.n_variance > 10)
    throw std::invalid_argument("state load: corrupt header");
  // AMG source rows first (validates the pattern before anything is touched)
  std::vector<float> ell;
  if (h.amg_nnz) {
    const uint64_t* rp = reinterpret_cast<const uint64_t*>(base + L.rowptr());
    const float* val = reinterpret_cast<const float*>(base + L.val());
    const uint64_t c0 = topo.c0;
    if (rp[NG] != h.amg_nnz) throw std::invalid_argument("state load: corrupt AMG row pointers");
    const size_t ld = topo.ld;
    ell.assign((size_t)topo.ws * ld, 0.0f);
    for (uint32_t i = 0; i < N; ++i) {
      const uint64_t a = rp[c0 + i], b = rp[c0 + i + 1];
      if (b < a || b > h.amg_nnz || b - a != topo.srow[i + 1] - topo.srow[i])
        throw std::invalid_argument("state load: AMG source pattern does not match the mesh");
      for (uint64_t k = a; k < b; ++k) ell[(size_t)(k - a) * ld + i] = val[k];
    }
  }
  std::vector<float> img;
  auto put = [&](void* dev, int comps, uint64_t sec) {  // owned + ghosts
    local_image(reinterpret_cast<const float*>(base + sec), comps, img);
    CFD_HIP(hipMemcpyAsync(static_cast<float*>(dev) - (size_t)shift * comps, img.data(), img.size() * sizeof(float),
                           hipMemcpyHostToDevice, stream));
    sync();
  };
  for (int s = 0; s < 3; ++s) {
    const uint64_t b = L.state(s);
    put(ring[s].u, 2, b + Layout::u_off(NG));
    put(ring[s].p, 1, b + Layout::p_off(NG));
    put(ring[s].dp, 1, b + Layout::dp_off(NG));
    put(ring[s].gp, 2, b + Layout::gp_off(NG));
  }
  {  // prev: owned cells only (check_evolution copies S() -> prev over [0, N))
    const uint64_t b = L.state(3), c0 = topo.c0;
    auto own = [&](void* dev, int comps, uint64_t sec) {
      CFD_HIP(hipMemcpyAsync(dev, base + sec + c0 * comps * 4, (size_t)N * comps * 4, hipMemcpyHostToDevice, stream));
      sync();
    };
    own(prev.u, 2, b + Layout::u_off(NG));
    own(prev.p, 1, b + Layout::p_off(NG));
    own(prev.dp, 1, b + Layout::dp_off(NG));
    own(prev.gp, 2, b + Layout::gp_off(NG));
  }
  put(x, 3, L.x());
  if (h.amg_nnz) {
    if (!amg_src) amg_src = arena.alloc<float>(ell.size());
    CFD_HIP(hipMemcpyAsync(amg_src, ell.data(), ell.size() * sizeof(float), hipMemcpyHostToDevice, stream));
    sync();
  }
  if (amg_built) drop_amg();  // the saved run's hierarchy replaces this solver's
  // the hierarchy is rebuilt under THIS solver's mode and rank count: the same
  // as the saving run's unless a partition-aware hierarchy is involved
  if (h.amg_nnz && h.nranks > 0 && rk == 0 &&
      ((h.amg_local_aggregation != 0) != amg_local || (amg_local && h.nranks != R)))
    std::fprintf(stderr,
                 "cfd_state_load: the file was saved with amg_local_aggregation=%d on %d rank(s); this solver "
                 "runs amg_local_aggregation=%d on %d: the AMG hierarchy rebuilt from the saved matrix differs, "
                 "so the continuation is not bit-identical to the saving run\n",
                 (int)h.amg_local_aggregation, (int)h.nranks, amg_local ? 1 : 0, R);
  amg_src_loaded = h.amg_nnz != 0;
  amg_age = h.amg_age;
  step_index = (h.step_index + 2) % 3;  // rotate() advances it back to the saved slot triple
  rotate();
  have_prev = h.have_prev != 0;
  inner = LagReader{};
  inner.has_last = h.inner_has_last != 0;
  inner.last = h.inner_last;
  variance_history.clear();
  for (uint32_t k = 0; k < h.n_variance; ++k) variance_history.push_back({h.variance[k][0], h.variance[k][1]});
  constants = h.constants;
  info = h.info;
}

}  // namespace cfd2
