// Mesh -> device-ready static topology and per-face-slot geometric factors.
//
// Restates init/mesh.rs:24-212 (f64 -> f32 upload, scalar CSR, face -> matrix
// slot, diagonal indices) and hoists every purely geometric sub-expression of
// prepare_coupled.wgsl / coupled_assembly_merged.wgsl out of the per-step
// kernels.  Each factor is computed in f32 with the same operations, in the
// same order, as the WGSL expression it replaces (compiled -ffp-contract=off),
// so the kernels reading it produce identical bits.
#include <algorithm>
#include <cstdlib>
#include <unordered_map>
#include <cmath>
#include <stdexcept>

#include "solver_impl.hpp"

namespace cfd2 {

namespace {
inline float wdistance(float ax, float ay, float bx, float by) {
  const float dx = ax - bx, dy = ay - by;
  return std::sqrt(dx * dx + dy * dy);
}
}  // namespace

void build_topology(const cfd_mesh_view& m, Topology& t) { build_topology(m, t, 0, m.num_cells); }

void build_topology(const cfd_mesh_view& m, Topology& t, uint32_t c0, uint32_t c1) {
  const uint32_t NG = m.num_cells, F = m.num_faces;
  if (NG == 0) throw std::invalid_argument("mesh has no cells");
  if (c0 >= c1 || c1 > NG) throw std::invalid_argument("empty or invalid owned cell range");
  const uint32_t N = c1 - c0;
  t.N = N;
  t.F = F;
  t.NG = NG;
  t.c0 = c0;
  t.c1 = c1;
  t.npad = (N + 63) & ~63u;
  const uint32_t NONE = 0xFFFFFFFFu;
  for (uint32_t f = 0; f < F; ++f) {
    if (m.face_owner[f] >= NG) throw std::invalid_argument("face_owner out of range");
    if (m.face_neighbor[f] != NONE && m.face_neighbor[f] >= NG)
      throw std::invalid_argument("face_neighbor out of range");
  }

  // f32 geometry (init/mesh.rs:93-155); centres of every cell (ghost geometry)
  std::vector<float> cx(NG), cy(NG);
  for (uint32_t i = 0; i < NG; ++i) {
    cx[i] = (float)m.cell_cx[i];
    cy[i] = (float)m.cell_cy[i];
  }
  t.vol.resize(N);
  for (uint32_t li = 0; li < N; ++li) t.vol[li] = (float)m.cell_vol[c0 + li];

  // scalar CSR rows of the owned cells (init/mesh.rs:27-53): adjacency from the
  // face list, + diagonal, sorted, deduplicated; GLOBAL column ids
  int ws = 0;
  {
    auto owned = [&](uint32_t c) { return c >= c0 && c < c1; };
    std::vector<uint32_t> deg(N + 1, 1);
    for (uint32_t f = 0; f < F; ++f) {
      const uint32_t o = m.face_owner[f], n = m.face_neighbor[f];
      if (n == NONE) continue;
      if (owned(o)) deg[o - c0]++;
      if (owned(n)) deg[n - c0]++;
    }
    std::vector<uint32_t> aoff(N + 1, 0);
    for (uint32_t li = 0; li < N; ++li) aoff[li + 1] = aoff[li] + deg[li];
    std::vector<uint32_t> adj(aoff[N]);
    std::vector<uint32_t> pos(aoff.begin(), aoff.end() - 1);
    for (uint32_t li = 0; li < N; ++li) adj[pos[li]++] = c0 + li;
    for (uint32_t f = 0; f < F; ++f) {
      const uint32_t o = m.face_owner[f], n = m.face_neighbor[f];
      if (n == NONE) continue;
      if (owned(o)) adj[pos[o - c0]++] = n;
      if (owned(n)) adj[pos[n - c0]++] = o;
    }
    t.srow.assign(N + 1, 0);
    t.scol.clear();
    t.scol.reserve(aoff[N]);
    for (uint32_t li = 0; li < N; ++li) {
      auto bb = adj.begin() + aoff[li], ee = adj.begin() + aoff[li + 1];
      std::sort(bb, ee);
      ee = std::unique(bb, ee);
      t.srow[li] = (uint32_t)t.scol.size();
      t.scol.insert(t.scol.end(), bb, ee);
      ws = std::max(ws, (int)(ee - bb));
    }
    t.srow[N] = (uint32_t)t.scol.size();
  }
  t.ws = ws;
  // one validated width limit for every row layout: the coupled-matrix ELL
  // header keeps a row's slots-in-use in 7 bits (kLgUsedMask), the scalar
  // image and the Jacobi relaxation u8 lengths
  if (ws > (int)kLgUsedMask)
    throw std::invalid_argument("cell with more than " + std::to_string(kLgUsedMask - 1) +
                                " neighbours (scalar row width " + std::to_string(ws) + " > " +
                                std::to_string(kLgUsedMask) + ")");
  // ghosts: off-range neighbours, ascending global id
  t.ghost.clear();
  for (uint32_t c : t.scol)
    if (c < c0 || c >= c1) t.ghost.push_back(c);
  std::sort(t.ghost.begin(), t.ghost.end());
  t.ghost.erase(std::unique(t.ghost.begin(), t.ghost.end()), t.ghost.end());
  t.glo = (uint32_t)(std::lower_bound(t.ghost.begin(), t.ghost.end(), c0) - t.ghost.begin());
  t.ghi = (uint32_t)t.ghost.size() - t.glo;

  // scalar-row ELL image (signed local columns) + diagonal rank (init/mesh.rs:201-212),
  // slot stride ld = npad (16-byte groups of 4 rows); 16-bit column deltas and
  // u8 lengths / ranks for the 4-rows-per-thread Krylov kernels
  const uint32_t ld = t.npad;
  t.ld = ld;
  t.ell_col.assign((size_t)ws * ld, 0);
  t.ell_len.assign(ld, 0);
  t.ell_drank.assign(ld, 0);
  t.ell_len8.assign(ld, 0);
  t.ell_drank8.assign(ld, 0);
  bool small = true;
  for (uint32_t li = 0; li < ld; ++li) {
    const uint32_t a = li < N ? t.srow[li] : 0, b = li < N ? t.srow[li + 1] : 0;
    t.ell_len[li] = b - a;
    bool found = li >= N;
    for (uint32_t k = a; k < b; ++k) {
      const uint32_t r = k - a;
      const int32_t c = t.rel(t.scol[k]);
      t.ell_col[(size_t)r * ld + li] = c;
      const int64_t d = (int64_t)c - (int64_t)li;
      if (d < -32768 || d > 32767) small = false;
      if (t.scol[k] == c0 + li) {
        t.ell_drank[li] = r;
        found = true;
      }
    }
    if (!found) throw std::invalid_argument("Diagonal not found in CSR cols");
    // unused ELL slots / padding rows hold the row's own index (never read)
    for (uint32_t r = b - a; r < (uint32_t)ws; ++r) t.ell_col[(size_t)r * ld + li] = (int32_t)li;
    t.ell_len8[li] = (uint8_t)t.ell_len[li];
    t.ell_drank8[li] = (uint8_t)t.ell_drank[li];
  }
  // coupled-matrix ELL with aligned slots (Topology::tslot)
  {
    // aligned slots up to 8 slots per row (the gap mask is 8 bits); wider
    // meshes (the Voronoi meshes: up to 9 neighbours) keep the positional layout
    const bool typed = ws <= 8;
    t.tmode.assign(ws, 0);
    if (typed) {
      const uint32_t step = N > (1u << 20) ? 7u : 1u;  // a sample is enough for a mode
      for (int r = 0; r < ws; ++r) {
        std::unordered_map<int32_t, uint32_t> cnt;
        for (uint32_t li = 0; li < N; li += step)
          if (t.ell_len[li] == (uint32_t)ws) ++cnt[t.ell_col[(size_t)r * ld + li] - (int32_t)li];
        uint32_t best = 0;
        for (const auto& kv : cnt)
          if (kv.second > best || (kv.second == best && kv.first < t.tmode[r])) {
            best = kv.second;
            t.tmode[r] = kv.first;
          }
      }
    }
    const int32_t vlo = -(int32_t)t.glo, vhi = (int32_t)(t.npad + t.ghi) - 1;
    t.tslot.assign(t.scol.size(), 0);
    t.tcol.assign((size_t)ws * ld, 0);
    t.tlg.assign(ld, 0);
    t.tdrank8.assign(ld, 0);
    for (uint32_t li = 0; li < ld; ++li) {
      const uint32_t a = li < N ? t.srow[li] : 0, len = li < N ? t.srow[li + 1] - a : 0;
      std::vector<int> slot(len);
      int prev = -1;
      for (uint32_t q = 0; q < len; ++q) {
        const int32_t d = t.ell_col[(size_t)q * ld + li] - (int32_t)li;
        const int lo = prev + 1, hi = ws - (int)(len - q);
        int s = lo;
        if (typed && len < (uint32_t)ws)
          for (int c = lo; c <= hi; ++c)
            if (t.tmode[c] == d) {
              s = c;
              break;
            }
        slot[q] = prev = s;
      }
      // slots in use; the gap mask exists only for the typed layout (ws <= 8):
      // untyped rows fill slots 0..len-1 and have no gaps
      uint32_t used = 0, on = 0;
      for (uint32_t q = 0; q < len; ++q) {
        t.tslot[a + q] = (uint8_t)slot[q];
        if (typed) on |= 1u << slot[q];
        used = (uint32_t)slot[q] + 1;
        t.tcol[(size_t)slot[q] * ld + li] = t.ell_col[(size_t)q * ld + li];
      }
      const uint32_t gap = typed ? ((1u << used) - 1u) & ~on : 0u;
      for (int r = 0; r < ws; ++r) {
        if (typed ? (on >> r & 1u) : (uint32_t)r < len) continue;
        const int32_t v = li < N ? (int32_t)li + t.tmode[r] : (int32_t)li;
        t.tcol[(size_t)r * ld + li] = std::min(std::max(v, vlo), vhi);
        const int64_t dd = (int64_t)t.tcol[(size_t)r * ld + li] - (int64_t)li;
        if (dd < -32768 || dd > 32767) small = false;
      }
      // regular row: every slot's column is row + tmode[slot] (the kernels
      // then derive the columns instead of loading them)
      bool regular = typed && li < N;
      for (int r = 0; r < ws && regular; ++r) regular = t.tcol[(size_t)r * ld + li] == (int32_t)li + t.tmode[r];
      t.tlg[li] = (uint16_t)(used | (regular ? 0x80u : 0u) | gap << 8);
      if (li < N) t.tdrank8[li] = (uint8_t)slot[t.ell_drank[li]];
    }
  }
  t.use16 = small;
  t.ell_col16.clear();
  t.tcol16.clear();
  if (small) {
    t.ell_col16.resize(t.ell_col.size());
    for (size_t e = 0; e < t.ell_col.size(); ++e)
      t.ell_col16[e] = (int16_t)(t.ell_col[e] - (int32_t)(e % ld));
    t.tcol16.resize(t.tcol.size());
    for (size_t e = 0; e < t.tcol.size(); ++e) t.tcol16[e] = (int16_t)(t.tcol[e] - (int32_t)(e % ld));
  }

  // face slots
  int wf = 0;
  t.nface.resize(N);
  for (uint32_t li = 0; li < N; ++li) {
    const uint32_t i = c0 + li;
    const uint32_t nfc = m.cell_face_offsets[i + 1] - m.cell_face_offsets[i];
    t.nface[li] = nfc;
    wf = std::max(wf, (int)nfc);
  }
  t.wf = wf;
  const size_t S = (size_t)wf * N;
  t.fs_other.assign(S, kNoCell);
  t.fs_meta.assign(S, 0);
  t.fs_face.assign(S, NONE);
  for (auto* v : {&t.fs_area, &t.fs_nx, &t.fs_ny, &t.fs_lam_s, &t.fs_lam_f, &t.fs_dist_a,
                  &t.fs_dist_e, &t.fs_dvx, &t.fs_dvy, &t.fs_rx, &t.fs_ry, &t.fs_rox, &t.fs_roy})
    v->assign(S, 0.0f);
  for (uint32_t li = 0; li < N; ++li) {
    const uint32_t i = c0 + li;
    const float ci_x = cx[i], ci_y = cy[i];
    for (uint32_t k = 0; k < t.nface[li]; ++k) {
      const uint32_t f = m.cell_faces[m.cell_face_offsets[i] + k];
      if (f >= F) throw std::invalid_argument("cell_faces out of range");
      const uint32_t o = m.face_owner[f], nb = m.face_neighbor[f];
      const bool own = (o == i);
      const bool internal = (nb != NONE);
      if (!internal && !own) throw std::invalid_argument("boundary face listed by a non-owner cell");
      if (internal && !own && nb != i)
        throw std::invalid_argument("cell lists a face it does not own or neighbour");
      const uint32_t bt = internal ? 0u : (m.face_boundary[f] & 3u);
      const float Nx = (float)m.face_nx[f], Ny = (float)m.face_ny[f];
      const float area = (float)m.face_area[f];
      const float fcx = (float)m.face_cx[f], fcy = (float)m.face_cy[f];
      const float nx = own ? Nx : -Nx, ny = own ? Ny : -Ny;
      // prepare_coupled.wgsl:124-130 geometric flip of the flux normal
      const float cox = cx[o], coy = cy[o];
      const float dxv = fcx - cox, dyv = fcy - coy;
      const bool flip = (dxv * Nx + dyv * Ny < 0.0f);
      const uint32_t other = internal ? (own ? nb : o) : NONE;
      const float ocx = internal ? cx[other] : fcx, ocy = internal ? cy[other] : fcy;
      const float dvx = ocx - ci_x, dvy = ocy - ci_y;
      const float dist_e = std::sqrt(dvx * dvx + dvy * dvy);            // prepare :224-226
      const float dist_a = std::fmax(std::fabs(dvx * nx + dvy * ny), 1e-6f);  // assembly :176-179
      uint32_t meta = bt | (own ? kMetaOwner : 0u) | (flip ? kMetaFluxFlip : 0u);
      float lam_s = 0.5f, lam_f = 0.5f;
      uint32_t rank = 0xFFu;
      if (internal) {
        const float d_c = wdistance(ci_x, ci_y, fcx, fcy);
        const float d_o = wdistance(ocx, ocy, fcx, fcy);
        const float tot = d_c + d_o;
        if (tot > 1e-6f)
          lam_s = d_o / tot;
        else
          meta |= kMetaDegen;
        const float cnx = cx[nb], cny = cy[nb];
        const float d_own = wdistance(cox, coy, fcx, fcy);
        const float d_ngh = wdistance(cnx, cny, fcx, fcy);
        const float total = d_own + d_ngh;
        if (total > 1e-6f) lam_f = d_ngh / total;
        // cell_face_matrix_indices (init/mesh.rs:157-193) as a row rank
        const uint32_t* b = t.scol.data() + t.srow[li];
        const uint32_t* e = t.scol.data() + t.srow[li + 1];
        const uint32_t* it = std::lower_bound(b, e, other);
        if (it == e || *it != other) throw std::invalid_argument("neighbour missing from CSR row");
        rank = (uint32_t)(it - b);
      }
      meta |= rank << kMetaRankShift;
      if (internal) meta |= (uint32_t)t.tslot[t.srow[li] + rank] << kMetaTSlotShift;
      const size_t e = (size_t)k * N + li;
      t.fs_other[e] = internal ? t.rel(other) : kNoCell;
      t.fs_meta[e] = meta;
      t.fs_face[e] = f;
      t.fs_area[e] = area;
      t.fs_nx[e] = nx;
      t.fs_ny[e] = ny;
      t.fs_lam_s[e] = lam_s;
      t.fs_lam_f[e] = lam_f;
      t.fs_dist_a[e] = dist_a;
      t.fs_dist_e[e] = dist_e;
      t.fs_dvx[e] = dvx;
      t.fs_dvy[e] = dvy;
      t.fs_rx[e] = fcx - ci_x;
      t.fs_ry[e] = fcy - ci_y;
      t.fs_rox[e] = fcx - ocx;
      t.fs_roy[e] = fcy - ocy;
    }
  }
}

}  // namespace cfd2
