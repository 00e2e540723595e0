// Deterministic cut-cell mesher + Laplacian smoothing (host, f64).
//
// Restatement of src/solver/mesh/{cut_cell.rs:10-510, quadtree.rs:39-103,
// geometry.rs:24-260, utils.rs:1-29, structs.rs:61-320}.  The reference runs
// the per-vertex / per-face loops with rayon; every one of them is a pure map
// (or a max-reduction), so the OpenMP loops below produce the same bits.
#include "mesh.hpp"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <stdexcept>

namespace cfd2 {

namespace {

// nalgebra Vector2::norm(): (x*x + y*y).sqrt()  (dotx special case for U2).
inline double norm2(double x, double y) { return std::sqrt(x * x + y * y); }

// Rust f64::signum: +1 for +0/positive, -1 for -0/negative, NaN for NaN.
inline double rsignum(double v) { return std::isnan(v) ? v : std::copysign(1.0, v); }

inline double box_sdf(double dx, double dy) {
  // dx.max(dy).min(0.0) + Vector2::new(dx.max(0.0), dy.max(0.0)).norm()
  return std::fmin(std::fmax(dx, dy), 0.0) + norm2(std::fmax(dx, 0.0), std::fmax(dy, 0.0));
}

}  // namespace

double Geometry::sdf(double x, double y) const {
  switch (kind) {
    case kChannelWithObstacle: {  // geometry.rs:46-58
      const double length = p[0], height = p[1], cx = p[2], cy = p[3], r = p[4];
      const double dx = std::fabs(x - length / 2.0) - length / 2.0;
      const double dy = std::fabs(y - height / 2.0) - height / 2.0;
      const double box_dist = box_sdf(dx, dy);
      const double circle_dist = norm2(x - cx, y - cy) - r;
      return std::fmax(box_dist, -circle_dist);
    }
    case kBackwardsStep: {  // geometry.rs:138-162
      const double length = p[0], h_in = p[1], h_out = p[2], step_x = p[3];
      const double obx = std::fabs(x - length / 2.0) - length / 2.0;
      const double oby = std::fabs(y - h_out / 2.0) - h_out / 2.0;
      const double outer_dist = box_sdf(obx, oby);
      const double step_h = h_out - h_in;
      const double step_w = step_x;
      const double block_cx = step_w / 2.0;
      const double block_cy = step_h / 2.0;
      const double bdx = std::fabs(x - block_cx) - step_w / 2.0;
      const double bdy = std::fabs(y - block_cy) - step_h / 2.0;
      const double block_dist = box_sdf(bdx, bdy);
      return std::fmax(outer_dist, -block_dist);
    }
    case kRectangularChannel: {  // geometry.rs:228-232
      const double length = p[0], height = p[1];
      const double dx = std::fabs(x - length / 2.0) - length / 2.0;
      const double dy = std::fabs(y - height / 2.0) - height / 2.0;
      return box_sdf(dx, dy);
    }
    case kCircleObstacle: {  // src/solver/mesh/tests.rs:17-27
      const double cx = p[0], cy = p[1], r = p[2], x0 = p[3], y0 = p[4], x1 = p[5], y1 = p[6];
      const double dx = std::fabs(x - (x0 + x1) / 2.0) - (x1 - x0) / 2.0;
      const double dy = std::fabs(y - (y0 + y1) / 2.0) - (y1 - y0) / 2.0;
      const double box_dist = box_sdf(dx, dy);
      const double circle_dist = norm2(x - cx, y - cy) - r;
      return std::fmax(box_dist, -circle_dist);
    }
    default:
      throw std::runtime_error("unknown geometry kind");
  }
}

namespace {

// ---------------------------------------------------------------------------
// Open-addressing hash maps (the reference uses AHashMap; only lookups/inserts
// are observable, never iteration order, so any exact map is equivalent).
// Open-addressing hash map (u64, u64) -> u32 with linear probing.  One
// 24-byte slot per entry (key pair, value, in-use flag) so a probe touches one
// cache line, not four separate arrays.
struct PairMap {
  struct Slot {
    uint64_t a, b;
    uint32_t v, used;
  };
  std::vector<Slot> slots;
  size_t mask = 0, count = 0;
  explicit PairMap(size_t expect) { rehash(std::max<size_t>(64, expect * 2)); }
  static uint64_t mix(uint64_t a, uint64_t b) {
    uint64_t h = a * 0x9E3779B97F4A7C15ull ^ (b + 0x632BE59BD9B4E019ull + (a << 6) + (a >> 2));
    h ^= h >> 31;
    h *= 0xBF58476D1CE4E5B9ull;
    h ^= h >> 29;
    return h;
  }
  void rehash(size_t cap) {
    size_t c = 1;
    while (c < cap) c <<= 1;
    std::vector<Slot> old = std::move(slots);
    slots.assign(c, Slot{0, 0, 0, 0});
    mask = c - 1;
    count = 0;
    for (const Slot& o : old)
      if (o.used) insert(o.a, o.b, o.v);
  }
  // Returns pointer to the value slot for key, or nullptr if absent.
  uint32_t* find(uint64_t a, uint64_t b) {
    size_t h = mix(a, b) & mask;
    while (slots[h].used) {
      if (slots[h].a == a && slots[h].b == b) return &slots[h].v;
      h = (h + 1) & mask;
    }
    return nullptr;
  }
  void insert(uint64_t a, uint64_t b, uint32_t v) {
    if ((count + 1) * 2 > mask + 1) rehash((mask + 1) * 2);
    size_t h = mix(a, b) & mask;
    while (slots[h].used) {
      if (slots[h].a == a && slots[h].b == b) {
        slots[h].v = v;
        return;
      }
      h = (h + 1) & mask;
    }
    slots[h] = Slot{a, b, v, 1};
    ++count;
  }
};

// Faces by their vertex pair (kmin, kmax), for the finalize pass: the first
// two faces of each kmin live in a per-vertex array (vertices of a cell are
// numbered close together, so these accesses stay in cache), further ones in
// a PairMap.  Same answers as one PairMap over all pairs.
struct EdgeMap {
  std::vector<uint64_t> inl;  // [2 v + s] = kmax << 32 | face, or kEmpty
  PairMap extra;
  static constexpr uint64_t kEmpty = ~0ull;
  explicit EdgeMap(size_t nverts) : inl(2 * nverts, kEmpty), extra(64) {}
  bool find(uint32_t kmin, uint32_t kmax, uint32_t* face) {
    for (int q = 0; q < 2; ++q) {
      const uint64_t e = inl[2 * (size_t)kmin + q];
      if (e == kEmpty) return false;  // slots fill in order: no later entry
      if ((uint32_t)(e >> 32) == kmax) {
        *face = (uint32_t)e;
        return true;
      }
    }
    if (uint32_t* f = extra.find(kmin, kmax)) {
      *face = *f;
      return true;
    }
    return false;
  }
  void insert(uint32_t kmin, uint32_t kmax, uint32_t face) {
    for (int q = 0; q < 2; ++q) {
      uint64_t& e = inl[2 * (size_t)kmin + q];
      if (e == kEmpty) {
        e = ((uint64_t)kmax << 32) | face;
        return;
      }
    }
    extra.insert(kmin, kmax, face);
  }
};

struct Pt {
  double x, y;
};

// quadtree.rs:39-93 (refine) + 95-103 (collect leaves, depth-first c0..c3).
void refine_collect(const Geometry& geo, Pt mn, Pt mx, double min_size, double growth_rate,
                    std::vector<std::pair<Pt, Pt>>& leaves) {
  const double size = std::fmax(mx.x - mn.x, mx.y - mn.y);
  if (size <= min_size * 1.001) {
    leaves.push_back({mn, mx});
    return;
  }
  const double d00 = geo.sdf(mn.x, mn.y);
  const double d10 = geo.sdf(mx.x, mn.y);
  const double d11 = geo.sdf(mx.x, mx.y);
  const double d01 = geo.sdf(mn.x, mx.y);
  const bool has_inside = d00 < 0.0 || d10 < 0.0 || d11 < 0.0 || d01 < 0.0;
  const bool has_outside = d00 >= 0.0 || d10 >= 0.0 || d11 >= 0.0 || d01 >= 0.0;
  bool should_split = has_inside && has_outside;
  if (!should_split) {
    const double dist =
        std::fmin(std::fmin(std::fmin(std::fabs(d00), std::fabs(d10)), std::fabs(d11)), std::fabs(d01));
    const double slope = std::fmax(growth_rate - 1.0, 0.0);
    const double max_allowed = min_size + slope * dist;
    if (size > max_allowed) should_split = true;
  }
  if (!should_split) {
    leaves.push_back({mn, mx});
    return;
  }
  const Pt c{(mn.x + mx.x) / 2.0, (mn.y + mx.y) / 2.0};
  refine_collect(geo, mn, c, min_size, growth_rate, leaves);
  refine_collect(geo, Pt{c.x, mn.y}, Pt{mx.x, c.y}, min_size, growth_rate, leaves);
  refine_collect(geo, Pt{mn.x, c.y}, Pt{c.x, mx.y}, min_size, growth_rate, leaves);
  refine_collect(geo, c, mx, min_size, growth_rate, leaves);
}

// utils.rs:4-10
Pt compute_normal(const Geometry& geo, Pt p) {
  const double eps = 1e-6;
  const double dx = geo.sdf(p.x + eps, p.y) - geo.sdf(p.x - eps, p.y);
  const double dy = geo.sdf(p.x, p.y + eps) - geo.sdf(p.x, p.y - eps);
  const double n = norm2(dx, dy);
  return Pt{dx / n, dy / n};
}

// utils.rs:12-29
bool intersect_lines(Pt p1, Pt n1, Pt p2, Pt n2, Pt* out) {
  const double det = n1.x * n2.y - n1.y * n2.x;
  if (std::fabs(det) < 1e-6) return false;
  const double d1 = p1.x * n1.x + p1.y * n1.y;
  const double d2 = p2.x * n2.x + p2.y * n2.y;
  out->x = (d1 * n2.y - d2 * n1.y) / det;
  out->y = (d2 * n1.x - d1 * n2.x) / det;
  return true;
}

}  // namespace

Mesh generate_cut_cell_mesh(const Geometry& geo, double min_cell_size, double max_cell_size,
                            double growth_rate, double domain_x, double domain_y) {
  std::vector<double> vx, vy;
  std::vector<uint8_t> v_fixed;
  std::vector<std::vector<uint32_t>> cells;

  const size_t nx = (size_t)std::ceil(domain_x / max_cell_size);
  const size_t ny = (size_t)std::ceil(domain_y / max_cell_size);
  PairMap vertex_map(nx * ny + 16);

  auto quantize = [](double v) -> int64_t { return (int64_t)std::round(v * 100000.0); };
  auto add_vertex = [&](Pt p, bool fixed) -> uint32_t {
    const int64_t kx = quantize(p.x), ky = quantize(p.y);
    if (uint32_t* idx = vertex_map.find((uint64_t)kx, (uint64_t)ky)) {
      if (fixed && !v_fixed[*idx]) v_fixed[*idx] = 1;
      return *idx;
    }
    const uint32_t idx = (uint32_t)vx.size();
    vx.push_back(p.x);
    vy.push_back(p.y);
    v_fixed.push_back(fixed ? 1 : 0);
    vertex_map.insert((uint64_t)kx, (uint64_t)ky, idx);
    return idx;
  };

  // 1. Base mesh (cut_cell.rs:47-207).  The vertex numbering is
  // order-dependent, so it stays serial; the polygons themselves (quadtree
  // refinement, SDF bisection, corner reconstruction: the bulk of the work)
  // are built in parallel over a band of base columns, then inserted in the
  // serial (column, row, leaf) order -- the same vertices, numbers and cells.
  cells.reserve(nx * ny);
  struct PV {
    Pt p;
    bool inter;
  };
  // one base column: its cells' polygons, concatenated (sizes in `len`)
  struct Column {
    std::vector<PV> verts;
    std::vector<uint32_t> len;
  };
  auto build_column = [&](size_t i, Column& col) {
    col.verts.clear();
    col.len.clear();
    std::vector<std::pair<Pt, Pt>> leaves;
    std::vector<PV> poly, recon;
    for (size_t j = 0; j < ny; ++j) {
      const double x0 = (double)i * max_cell_size;
      const double y0 = (double)j * max_cell_size;
      const double x1 = std::fmin(x0 + max_cell_size, domain_x);
      const double y1 = std::fmin(y0 + max_cell_size, domain_y);
      leaves.clear();
      refine_collect(geo, Pt{x0, y0}, Pt{x1, y1}, min_cell_size, growth_rate, leaves);
      for (const auto& leaf : leaves) {
        const Pt mn = leaf.first, mx = leaf.second;
        const Pt p00 = mn, p10{mx.x, mn.y}, p11 = mx, p01{mn.x, mx.y};
        const double d00 = geo.sdf(p00.x, p00.y);
        const double d10 = geo.sdf(p10.x, p10.y);
        const double d11 = geo.sdf(p11.x, p11.y);
        const double d01 = geo.sdf(p01.x, p01.y);
        const double tol = 1e-9;
        if (d00 >= -tol && d10 >= -tol && d11 >= -tol && d01 >= -tol) continue;
        poly.clear();
        if (d00 < -tol && d10 < -tol && d11 < -tol && d01 < -tol) {
          poly.push_back({p00, false});
          poly.push_back({p10, false});
          poly.push_back({p11, false});
          poly.push_back({p01, false});
        } else {
          const Pt corners[4] = {p00, p10, p11, p01};
          const double dists[4] = {d00, d10, d11, d01};
          for (int k = 0; k < 4; ++k) {
            const Pt pc = corners[k], pn = corners[(k + 1) % 4];
            const double dc = dists[k], dn = dists[(k + 1) % 4];
            if (dc < -tol) poly.push_back({pc, false});
            if ((dc < -tol && dn >= -tol) || (dc >= -tol && dn < -tol)) {
              double t_a = 0.0, t_b = 1.0, d_a = dc, d_b = dn;
              double t = t_a - d_a * (t_b - t_a) / (d_b - d_a);
              for (int it = 0; it < 10; ++it) {
                const Pt pi{pc.x + (pn.x - pc.x) * t, pc.y + (pn.y - pc.y) * t};
                const double di = geo.sdf(pi.x, pi.y);
                if (std::fabs(di) < 1e-12) break;
                if (rsignum(di) == rsignum(d_a)) {
                  t_a = t;
                  d_a = di;
                } else {
                  t_b = t;
                  d_b = di;
                }
                const double denom = d_b - d_a;
                if (std::fabs(denom) < 1e-20) break;
                t = t_a - d_a * (t_b - t_a) / denom;
              }
              poly.push_back({Pt{pc.x + (pn.x - pc.x) * t, pc.y + (pn.y - pc.y) * t}, true});
            }
          }
        }
        if (poly.size() >= 3) {
          recon.clear();
          const size_t n = poly.size();
          for (size_t k = 0; k < n; ++k) {
            const PV cur = poly[k], nxt = poly[(k + 1) % n];
            recon.push_back(cur);
            if (cur.inter && nxt.inter) {
              const Pt n1 = compute_normal(geo, cur.p);
              const Pt n2 = compute_normal(geo, nxt.p);
              if (n1.x * n2.x + n1.y * n2.y < 0.7) {
                Pt pcor;
                if (intersect_lines(cur.p, n1, nxt.p, n2, &pcor)) {
                  const double ctol = 1e-5;
                  if (std::fabs(geo.sdf(pcor.x, pcor.y)) <= 1e-4) {
                    if (pcor.x >= mn.x - ctol && pcor.x <= mx.x + ctol && pcor.y >= mn.y - ctol &&
                        pcor.y <= mx.y + ctol)
                      recon.push_back({pcor, true});
                  }
                }
              }
            }
          }
          col.verts.insert(col.verts.end(), recon.begin(), recon.end());
          col.len.push_back((uint32_t)recon.size());
        }
      }
    }
  };
  constexpr size_t kBand = 64;  // base columns built in parallel per band
  std::vector<Column> band(kBand);
  for (size_t i0 = 0; i0 < nx; i0 += kBand) {
    const size_t nb = std::min(kBand, nx - i0);
#pragma omp parallel for schedule(dynamic, 1)
    for (long q = 0; q < (long)nb; ++q) build_column(i0 + (size_t)q, band[q]);
    for (size_t q = 0; q < nb; ++q) {
      const Column& col = band[q];
      size_t at = 0;
      for (const uint32_t n : col.len) {
        std::vector<uint32_t> idxs;
        idxs.reserve(n);
        for (uint32_t k = 0; k < n; ++k, ++at) idxs.push_back(add_vertex(col.verts[at].p, col.verts[at].inter));
        cells.push_back(std::move(idxs));
      }
    }
  }

  // 2-6. Imprint hanging nodes (cut_cell.rs:209-404).
  const double grid_size = max_cell_size;
  const size_t grid_nx = (size_t)std::ceil(domain_x / grid_size) + 1;
  const size_t grid_ny = (size_t)std::ceil(domain_y / grid_size) + 1;
  const size_t grid_len = grid_nx * grid_ny;
  const size_t nv = vx.size();
  std::vector<size_t> grid_counts(grid_len, 0), grid_idx(nv);
  for (size_t i = 0; i < nv; ++i) {
    const size_t gx = (size_t)std::fmax(std::floor(vx[i] / grid_size), 0.0);
    const size_t gy = (size_t)std::fmax(std::floor(vy[i] / grid_size), 0.0);
    if (gx < grid_nx && gy < grid_ny) {
      grid_idx[i] = gy * grid_nx + gx;
      grid_counts[grid_idx[i]]++;
    } else {
      grid_idx[i] = grid_len;
    }
  }
  std::vector<size_t> grid_starts(grid_len + 1, 0);
  {
    size_t cur = 0;
    for (size_t i = 0; i < grid_len; ++i) {
      grid_starts[i] = cur;
      cur += grid_counts[i];
    }
    grid_starts[grid_len] = cur;
  }
  std::vector<double> sxs(nv, 0.0), sys(nv, 0.0);
  std::vector<uint32_t> sidx(nv, 0);
  {
    std::vector<size_t> cs = grid_starts;
    for (size_t i = 0; i < nv; ++i) {
      const size_t g = grid_idx[i];
      if (g < grid_len) {
        const size_t pos = cs[g]++;
        sxs[pos] = vx[i];
        sys[pos] = vy[i];
        sidx[pos] = (uint32_t)i;
      }
    }
  }
  const long ncells_poly = (long)cells.size();
#pragma omp parallel for schedule(dynamic, 4096)
  for (long ci = 0; ci < ncells_poly; ++ci) {
    std::vector<uint32_t>& cell = cells[ci];
    std::vector<uint32_t> new_cell;
    std::vector<std::pair<double, uint32_t>> on_seg;
    const size_t n = cell.size();
    for (size_t k = 0; k < n; ++k) {
      const uint32_t ic = cell[k], in = cell[(k + 1) % n];
      new_cell.push_back(ic);
      const double pcx = vx[ic], pcy = vy[ic], pnx = vx[in], pny = vy[in];
      const double sgx = pnx - pcx, sgy = pny - pcy;
      const double seg_len_sq = sgx * sgx + sgy * sgy;
      if (seg_len_sq < 1e-12) continue;
      on_seg.clear();
      const double min_x = std::fmin(pcx, pnx), max_x = std::fmax(pcx, pnx);
      const double min_y = std::fmin(pcy, pny), max_y = std::fmax(pcy, pny);
      const size_t min_gx = (size_t)std::fmax(std::floor(min_x / grid_size), 0.0);
      const size_t max_gx = (size_t)std::fmax(std::floor(max_x / grid_size), 0.0);
      const size_t min_gy = (size_t)std::fmax(std::floor(min_y / grid_size), 0.0);
      const size_t max_gy = (size_t)std::fmax(std::floor(max_y / grid_size), 0.0);
      const size_t gy_end = std::min(max_gy, grid_ny - 1), gx_end = std::min(max_gx, grid_nx - 1);
      for (size_t gy = min_gy; gy <= gy_end; ++gy) {
        for (size_t gx = min_gx; gx <= gx_end; ++gx) {
          const size_t g = gy * grid_nx + gx;
          for (size_t q = grid_starts[g]; q < grid_starts[g + 1]; ++q) {
            const double vxq = sxs[q], vyq = sys[q];
            const double dxc = vxq - pcx, dyc = vyq - pcy;
            const double d_curr = dxc * dxc + dyc * dyc;
            const double dxn = vxq - pnx, dyn = vyq - pny;
            const double d_next = dxn * dxn + dyn * dyn;
            if (d_curr < 1e-10 || d_next < 1e-10) continue;
            const double t = (dxc * sgx + dyc * sgy) / seg_len_sq;
            if (t > 1e-6 && t < 1.0 - 1e-6) {
              const double prx = pcx + sgx * t, pry = pcy + sgy * t;
              const double ex = vxq - prx, ey = vyq - pry;
              if (ex * ex + ey * ey < 1e-10) on_seg.push_back({t, sidx[q]});
            }
          }
        }
      }
      std::stable_sort(on_seg.begin(), on_seg.end(),
                       [](const std::pair<double, uint32_t>& a, const std::pair<double, uint32_t>& b) {
                         return a.first < b.first;
                       });
      for (const auto& e : on_seg) new_cell.push_back(e.second);
    }
    cell.swap(new_cell);
  }

  // 7. Finalize (cut_cell.rs:406-496).
  Mesh mesh;
  mesh.vx = std::move(vx);
  mesh.vy = std::move(vy);
  mesh.v_fixed = std::move(v_fixed);
  mesh.cell_face_offsets.push_back(0);
  mesh.cell_vertex_offsets.push_back(0);
  {
    size_t nvs = 0;
    for (const auto& cv : cells) nvs += cv.size();
    const size_t nfe = nvs / 2 + cells.size() + 16;  // ~2 faces per quad cell, boundary extra
    for (auto* v : {&mesh.face_v1, &mesh.face_v2, &mesh.face_owner, &mesh.face_neighbor, &mesh.face_boundary})
      v->reserve(nfe);
    for (auto* v : {&mesh.face_nx, &mesh.face_ny, &mesh.face_area, &mesh.face_cx, &mesh.face_cy}) v->reserve(nfe);
    for (auto* v : {&mesh.cell_cx, &mesh.cell_cy, &mesh.cell_vol}) v->reserve(cells.size());
    mesh.cell_face_offsets.reserve(cells.size() + 1);
    mesh.cell_vertex_offsets.reserve(cells.size() + 1);
    mesh.cell_faces.reserve(nvs);
    mesh.cell_vertices.reserve(nvs);
  }
  EdgeMap face_map(mesh.vx.size());
  for (const auto& cv : cells) {
    double ccx = 0.0, ccy = 0.0, area = 0.0;
    const size_t n = cv.size();
    for (size_t k = 0; k < n; ++k) {
      const uint32_t a = cv[k], b = cv[(k + 1) % n];
      const double pix = mesh.vx[a], piy = mesh.vy[a], pjx = mesh.vx[b], pjy = mesh.vy[b];
      const double cross = pix * pjy - pjx * piy;
      area += cross;
      ccx += (pix + pjx) * cross;
      ccy += (piy + pjy) * cross;
    }
    area *= 0.5;
    if (std::fabs(area) < 1e-9) continue;
    const double six_a = 6.0 * area;
    ccx /= six_a;
    ccy /= six_a;
    const uint32_t cell_idx = (uint32_t)mesh.cell_cx.size();
    for (size_t k = 0; k < n; ++k) {
      const uint32_t v1 = cv[k], v2 = cv[(k + 1) % n];
      if (v1 == v2) continue;
      const double p1x = mesh.vx[v1], p1y = mesh.vy[v1], p2x = mesh.vx[v2], p2y = mesh.vy[v2];
      const double ex = p2x - p1x, ey = p2y - p1y;
      const double elen = norm2(ex, ey);
      if (elen < 1e-9) continue;
      const uint32_t kmin = std::min(v1, v2), kmax = std::max(v1, v2);
      uint32_t fidx;
      if (face_map.find(kmin, kmax, &fidx)) {
        mesh.face_neighbor[fidx] = cell_idx;
        mesh.face_boundary[fidx] = kNone;
        mesh.cell_faces.push_back(fidx);
      } else {
        const double fcx = (p1x + p2x) * 0.5, fcy = (p1y + p2y) * 0.5;
        // Vector2::new(edge.y, -edge.x).normalize()
        const double nlen = norm2(ey, -ex);
        const double nxv = ey / nlen, nyv = -ex / nlen;
        uint32_t btype;
        if (fcx < 1e-6)
          btype = kInlet;
        else if (std::fabs(fcx - domain_x) < 1e-6)
          btype = kOutlet;
        else
          btype = kWall;
        const uint32_t face_idx = (uint32_t)mesh.face_cx.size();
        mesh.face_v1.push_back(v1);
        mesh.face_v2.push_back(v2);
        mesh.face_owner.push_back(cell_idx);
        mesh.face_neighbor.push_back(kNoNeighbor);
        mesh.face_boundary.push_back(btype);
        mesh.face_nx.push_back(nxv);
        mesh.face_ny.push_back(nyv);
        mesh.face_area.push_back(elen);
        mesh.face_cx.push_back(fcx);
        mesh.face_cy.push_back(fcy);
        face_map.insert(kmin, kmax, face_idx);
        mesh.cell_faces.push_back(face_idx);
      }
    }
    mesh.cell_cx.push_back(ccx);
    mesh.cell_cy.push_back(ccy);
    mesh.cell_vol.push_back(std::fabs(area));
    mesh.cell_face_offsets.push_back((uint32_t)mesh.cell_faces.size());
    mesh.cell_vertices.insert(mesh.cell_vertices.end(), cv.begin(), cv.end());
    mesh.cell_vertex_offsets.push_back((uint32_t)mesh.cell_vertices.size());
  }
  return mesh;
}

// structs.rs:61-155
void Mesh::recalculate_geometry() {
  const long nf = (long)face_cx.size();
#pragma omp parallel for schedule(static)
  for (long i = 0; i < nf; ++i) {
    const uint32_t a = face_v1[i], b = face_v2[i];
    const double v0x = vx[a], v0y = vy[a], v1x = vx[b], v1y = vy[b];
    face_cx[i] = (v0x + v1x) * 0.5;
    face_cy[i] = (v0y + v1y) * 0.5;
    const double ex = v1x - v0x, ey = v1y - v0y;
    const double len = norm2(ex, ey);
    face_area[i] = len;
    const double tx = ex / len, ty = ey / len;  // edge_vec.normalize()
    double nx = ty, ny = -tx;
    if (nx * face_nx[i] + ny * face_ny[i] < 0.0) {
      nx = -nx;
      ny = -ny;
    }
    face_nx[i] = nx;
    face_ny[i] = ny;
  }
  const long nc = (long)cell_cx.size();
#pragma omp parallel for schedule(static)
  for (long i = 0; i < nc; ++i) {
    const uint32_t start = cell_vertex_offsets[i], end = cell_vertex_offsets[i + 1];
    const uint32_t n = end - start;
    double signed_area = 0.0, c_x = 0.0, c_y = 0.0;
    for (uint32_t k = 0; k < n; ++k) {
      const uint32_t i0 = cell_vertices[start + k], i1 = cell_vertices[start + (k + 1) % n];
      const double p0x = vx[i0], p0y = vy[i0], p1x = vx[i1], p1y = vy[i1];
      const double cross = p0x * p1y - p1x * p0y;
      signed_area += cross;
      c_x += (p0x + p1x) * cross;
      c_y += (p0y + p1y) * cross;
    }
    signed_area *= 0.5;
    const double area = std::fabs(signed_area);
    double cx, cy;
    if (area > 1e-12) {
      cx = c_x / (6.0 * signed_area);
      cy = c_y / (6.0 * signed_area);
    } else {
      cx = 0.0;
      cy = 0.0;
      for (uint32_t k = 0; k < n; ++k) {
        cx += vx[cell_vertices[start + k]];
        cy += vy[cell_vertices[start + k]];
      }
      cx /= (double)n;
      cy /= (double)n;
    }
    cell_cx[i] = cx;
    cell_cy[i] = cy;
    cell_vol[i] = area;
  }
}

// structs.rs:294-320
double Mesh::calculate_max_skewness() const {
  const long nf = (long)face_cx.size();
  double best = 0.0;
#pragma omp parallel for schedule(static) reduction(max : best)
  for (long i = 0; i < nf; ++i) {
    const uint32_t o = face_owner[i];
    double dx, dy;
    if (face_neighbor[i] != kNoNeighbor) {
      const uint32_t n = face_neighbor[i];
      dx = cell_cx[n] - cell_cx[o];
      dy = cell_cy[n] - cell_cy[o];
    } else {
      dx = face_cx[i] - cell_cx[o];
      dy = face_cy[i] - cell_cy[o];
    }
    double nx = 0.0, ny = 0.0;
    if (dx * dx + dy * dy > 1e-12) {
      const double l = norm2(dx, dy);
      nx = dx / l;
      ny = dy / l;
    }
    const double s = 1.0 - std::fabs(nx * face_nx[i] + ny * face_ny[i]);
    best = std::fmax(best, s);
  }
  return best;
}

// structs.rs:159-292
int Mesh::smooth(const Geometry& geo, double target_skew, int max_iterations) {
  const size_t n_verts = vx.size();
  // adjacency in face order (both directions), as Vec<Vec<usize>>
  std::vector<uint32_t> adj_cnt(n_verts + 1, 0);
  const size_t nf = face_cx.size();
  for (size_t i = 0; i < nf; ++i) {
    adj_cnt[face_v1[i]]++;
    adj_cnt[face_v2[i]]++;
  }
  std::vector<uint32_t> adj_off(n_verts + 1, 0);
  for (size_t i = 0; i < n_verts; ++i) adj_off[i + 1] = adj_off[i] + adj_cnt[i];
  std::vector<uint32_t> adj(adj_off[n_verts]);
  {
    std::vector<uint32_t> pos(adj_off.begin(), adj_off.end() - 1);
    for (size_t i = 0; i < nf; ++i) {
      const uint32_t a = face_v1[i], b = face_v2[i];
      adj[pos[a]++] = b;
      adj[pos[b]++] = a;
    }
  }
  double minx = 1.7976931348623157e308, miny = 1.7976931348623157e308;
  double maxx = -1.7976931348623157e308, maxy = -1.7976931348623157e308;
  for (size_t i = 0; i < n_verts; ++i) {
    if (vx[i] < minx) minx = vx[i];
    if (vy[i] < miny) miny = vy[i];
    if (vx[i] > maxx) maxx = vx[i];
    if (vy[i] > maxy) maxy = vy[i];
  }
  auto is_on_box = [&](double x, double y) {
    const double eps = 1e-6;
    return std::fabs(x - minx) < eps || std::fabs(x - maxx) < eps || std::fabs(y - miny) < eps ||
           std::fabs(y - maxy) < eps;
  };
  std::vector<double> nvx(n_verts), nvy(n_verts);
  for (int iter = 0; iter < max_iterations; ++iter) {
    recalculate_geometry();
    if (calculate_max_skewness() < target_skew) return iter;
#pragma omp parallel for schedule(static)
    for (long i = 0; i < (long)n_verts; ++i) {
      const double x_old = vx[i], y_old = vy[i];
      nvx[i] = x_old;
      nvy[i] = y_old;
      if (is_on_box(x_old, y_old)) continue;
      const uint32_t a0 = adj_off[i], a1 = adj_off[i + 1];
      if (a0 == a1) continue;
      double sx = 0.0, sy = 0.0;
      int count = 0;
      for (uint32_t q = a0; q < a1; ++q) {
        sx += vx[adj[q]];
        sy += vy[adj[q]];
        ++count;
      }
      const double avg_x = sx / (double)count, avg_y = sy / (double)count;
      const double alpha = 0.5;
      double x_new = x_old + (avg_x - x_old) * alpha;
      double y_new = y_old + (avg_y - y_old) * alpha;
      if (v_fixed[i]) {
        const double d = geo.sdf(x_new, y_new);
        const double eps = 1e-6;
        const double gdx = geo.sdf(x_new + eps, y_new) - geo.sdf(x_new - eps, y_new);
        const double gdy = geo.sdf(x_new, y_new + eps) - geo.sdf(x_new, y_new - eps);
        const double gl = norm2(gdx, gdy);
        const double gx = gdx / gl, gy = gdy / gl;
        x_new = x_new - gx * d;
        y_new = y_new - gy * d;
      }
      bool bad = false;
      for (uint32_t q = a0; q < a1; ++q) {
        const double ddx = x_new - vx[adj[q]], ddy = y_new - vy[adj[q]];
        if (ddx * ddx + ddy * ddy < 1e-8) {
          bad = true;
          break;
        }
      }
      if (!bad) {
        nvx[i] = x_new;
        nvy[i] = y_new;
      }
    }
    vx.swap(nvx);
    vy.swap(nvy);
  }
  recalculate_geometry();
  return max_iterations;
}

}  // namespace cfd2
