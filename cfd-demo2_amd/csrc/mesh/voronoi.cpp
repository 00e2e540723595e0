// Seeded polygonal (Voronoi) mesher: SURVEY §8(f) rank 4, a behavioural
// restatement of src/solver/mesh/delaunay.rs + voronoi.rs.  Those use an
// unseeded thread_rng, so their meshes cannot be reproduced; this one follows
// the same pipeline with a seeded generator:
//   1. generators: the geometry's boundary points (geometry.rs
//      get_boundary_points, fixed) + variable-radius Poisson-disk interior
//      points (delaunay.rs:195-333, Bridson with r = min + (growth-1)|sdf|,
//      capped at max), Morton-ordered;
//   2. Delaunay triangulation, Bowyer-Watson (delaunay.rs:483-729), keeping
//      the triangles that touch an interior generator or whose centroid is in
//      the fluid;
//   3. 20 sweeps of size-weighted Laplacian generator smoothing, each followed
//      by a re-triangulation (delaunay.rs:170-190, 335-460);
//   4. the dual (voronoi.rs:23-388): one cell per generator; a face per
//      Delaunay edge between the dual points of its triangles (a hull edge:
//      dual point -> edge midpoint, plus two boundary half-faces midpoint ->
//      generator); boundary type by position (x = 0 inlet, x = L outlet, else
//      wall).
// Where the reference repairs concave boundary cells afterwards
// (voronoi.rs:390-782), the dual point of a triangle here is its
// circumcentre only when that lies inside the triangle, else its centroid:
// every face then stays inside its two triangles, so every cell is a simple
// CCW polygon star-shaped about its generator and no repair is needed.
// Zero-length faces (cocircular generators) are dropped.  Geometry is then
// derived from the vertices by Mesh::recalculate_geometry (centroids, areas,
// face normals), as the reference does.
#include <algorithm>
#include <array>
#include <cmath>
#include <cstdint>
#include <map>
#include <stdexcept>
#include <unordered_map>
#include <vector>

#include "mesh.hpp"

namespace cfd2 {

namespace {

struct P {
  double x, y;
};

struct Rng {  // splitmix64: platform-independent doubles in [0, 1)
  uint64_t s;
  uint64_t next() {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  double uniform() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }
};

bool inside(const Geometry& g, P p) { return g.sdf(p.x, p.y) < 0.0; }

void box_points(double x0, double y0, double x1, double y1, double spacing, std::vector<P>& out) {
  const size_t nx = (size_t)std::ceil((x1 - x0) / spacing), ny = (size_t)std::ceil((y1 - y0) / spacing);
  for (size_t i = 0; i <= nx; ++i) {
    const double x = std::min(x0 + (double)i * spacing, x1);
    out.push_back({x, y0});
    out.push_back({x, y1});
  }
  for (size_t i = 0; i <= ny; ++i) {
    const double y = std::min(y0 + (double)i * spacing, y1);
    out.push_back({x0, y});
    out.push_back({x1, y});
  }
}

void circle_points(double cx, double cy, double r, double spacing, std::vector<P>& out) {
  const size_t n = (size_t)std::ceil(2.0 * M_PI * r / spacing);
  for (size_t i = 0; i < n; ++i) {
    const double t = 2.0 * M_PI * (double)i / (double)n;
    out.push_back({cx + r * std::cos(t), cy + r * std::sin(t)});
  }
}

// geometry.rs get_boundary_points (ChannelWithObstacle :72-110, BackwardsStep
// :173-215, RectangularChannel :243-258; CircleObstacle as the channel one)
std::vector<P> boundary_points(const Geometry& g, double spacing) {
  std::vector<P> out;
  switch (g.kind) {
    case kChannelWithObstacle:
      box_points(0.0, 0.0, g.p[0], g.p[1], spacing, out);
      circle_points(g.p[2], g.p[3], g.p[4], spacing, out);
      break;
    case kRectangularChannel:
      box_points(0.0, 0.0, g.p[0], g.p[1], spacing, out);
      break;
    case kCircleObstacle:
      box_points(g.p[3], g.p[4], g.p[5], g.p[6], spacing, out);
      circle_points(g.p[0], g.p[1], g.p[2], spacing, out);
      break;
    case kBackwardsStep: {
      const double L = g.p[0], h_in = g.p[1], h_out = g.p[2], sx = g.p[3], sh = h_out - h_in;
      const P seg[6][2] = {{{0.0, h_out}, {L, h_out}}, {{L, h_out}, {L, 0.0}}, {{L, 0.0}, {sx, 0.0}},
                           {{sx, 0.0}, {sx, sh}},      {{sx, sh}, {0.0, sh}},   {{0.0, sh}, {0.0, h_out}}};
      for (const auto& s : seg) {
        const double d = std::hypot(s[1].x - s[0].x, s[1].y - s[0].y);
        const size_t n = (size_t)std::ceil(d / spacing);
        for (size_t i = 0; i < n; ++i) {
          const double t = (double)i / (double)n;
          out.push_back({s[0].x + (s[1].x - s[0].x) * t, s[0].y + (s[1].y - s[0].y) * t});
        }
      }
      break;
    }
    default:
      throw std::invalid_argument("voronoi mesher: unsupported geometry kind");
  }
  return out;
}

struct Sizing {
  const Geometry& g;
  double mn, mx, growth;
  double operator()(P p) const { return std::min(mn + std::max(growth - 1.0, 0.0) * std::fabs(g.sdf(p.x, p.y)), mx); }
};

// Bridson Poisson-disk sampling with the variable radius (delaunay.rs:195-333)
std::vector<P> poisson_points(const std::vector<P>& bnd, const Sizing& size, double dx, double dy, Rng& rng) {
  const double cell = size.mn / std::sqrt(2.0);
  const long gw = (long)std::ceil(dx / cell), gh = (long)std::ceil(dy / cell);
  std::vector<int64_t> grid((size_t)(gw * gh), -1);
  std::vector<P> pts(bnd);
  std::vector<size_t> active;
  auto put = [&](size_t idx) {
    const long gx = (long)std::floor(pts[idx].x / cell), gy = (long)std::floor(pts[idx].y / cell);
    if (gx >= 0 && gx < gw && gy >= 0 && gy < gh) grid[(size_t)(gy * gw + gx)] = (int64_t)idx;
  };
  for (size_t i = 0; i < pts.size(); ++i) {
    active.push_back(i);
    put(i);
  }
  const long search = (long)std::ceil(size.mx / cell);
  while (!active.empty()) {
    const size_t ai = (size_t)(rng.uniform() * (double)active.size()) % active.size();
    const P p = pts[active[ai]];
    const double r = size(p);
    bool found = false;
    for (int k = 0; k < 30 && !found; ++k) {
      const double ang = rng.uniform() * 2.0 * M_PI, dist = r + rng.uniform() * r;
      const P q{p.x + dist * std::cos(ang), p.y + dist * std::sin(ang)};
      if (q.x < 0.0 || q.x > dx || q.y < 0.0 || q.y > dy || !inside(size.g, q)) continue;
      const double rq = size(q);
      const long gx = (long)std::floor(q.x / cell), gy = (long)std::floor(q.y / cell);
      bool conflict = false;
      for (long oy = -search; oy <= search && !conflict; ++oy)
        for (long ox = -search; ox <= search && !conflict; ++ox) {
          const long nx = gx + ox, ny = gy + oy;
          if (nx < 0 || nx >= gw || ny < 0 || ny >= gh) continue;
          const int64_t j = grid[(size_t)(ny * gw + nx)];
          if (j < 0) continue;
          const double ddx = pts[(size_t)j].x - q.x, ddy = pts[(size_t)j].y - q.y;
          conflict = ddx * ddx + ddy * ddy < rq * rq;
        }
      if (conflict) continue;
      pts.push_back(q);
      active.push_back(pts.size() - 1);
      put(pts.size() - 1);
      found = true;
    }
    if (!found) {
      active[ai] = active.back();
      active.pop_back();
    }
  }
  return std::vector<P>(pts.begin() + (ptrdiff_t)bnd.size(), pts.end());
}

uint64_t morton(double x, double y, double dx, double dy) {
  auto spread = [](uint64_t v) {
    v &= 0xFFFFFFFFull;
    v = (v | (v << 16)) & 0x0000FFFF0000FFFFull;
    v = (v | (v << 8)) & 0x00FF00FF00FF00FFull;
    v = (v | (v << 4)) & 0x0F0F0F0F0F0F0F0Full;
    v = (v | (v << 2)) & 0x3333333333333333ull;
    v = (v | (v << 1)) & 0x5555555555555555ull;
    return v;
  };
  const double s = 65535.0;
  const uint64_t ix = (uint64_t)std::clamp(x / dx * s, 0.0, s), iy = (uint64_t)std::clamp(y / dy * s, 0.0, s);
  return spread(ix) | (spread(iy) << 1);
}

double orient(P a, P b, P c) { return (b.x - a.x) * (c.y - a.y) - (b.y - a.y) * (c.x - a.x); }

// p strictly inside the circumcircle of CCW (a, b, c)
bool in_circle(P a, P b, P c, P p) {
  const long double adx = a.x - p.x, ady = a.y - p.y, bdx = b.x - p.x, bdy = b.y - p.y, cdx = c.x - p.x,
                    cdy = c.y - p.y;
  const long double al = adx * adx + ady * ady, bl = bdx * bdx + bdy * bdy, cl = cdx * cdx + cdy * cdy;
  const long double det = adx * (bdy * cl - cdy * bl) - ady * (bdx * cl - cdx * bl) + al * (bdx * cdy - cdx * bdy);
  return det > 0.0L;
}

struct Tri {
  uint32_t v[3];   // CCW
  int64_t nb[3];   // neighbour across edge k = v[k] -> v[(k+1)%3] (-1: none)
  bool alive;
};

// Bowyer-Watson over pts (+3 super-triangle vertices); returns the CCW
// triangles of the input points with their adjacency.
std::vector<Tri> delaunay(const std::vector<P>& in, double dx, double dy) {
  std::vector<P> pts(in);
  const size_t n = in.size();
  const double m = 10.0 * std::hypot(dx, dy);
  pts.push_back({-m, -m});
  pts.push_back({2.0 * m + dx, -m});
  pts.push_back({-m, 2.0 * m + dy});
  std::vector<Tri> T;
  std::vector<size_t> free_slots;
  T.push_back({{(uint32_t)n, (uint32_t)n + 1, (uint32_t)n + 2}, {-1, -1, -1}, true});
  size_t last = 0;
  std::vector<size_t> cav, stack;
  std::vector<uint32_t> mark;  // mark[t] == i + 1: triangle t is in point i's cavity (no per-point reset)
  struct BEdge {
    uint32_t a, b;
    int64_t out;
  };
  std::vector<BEdge> bedges;
  for (size_t i = 0; i < n; ++i) {
    const P p = pts[i];
    // locate by walking; linear scan as fallback
    size_t cur = T[last].alive ? last : 0;
    while (!T[cur].alive) ++cur;
    bool located = false;
    for (size_t it = 0; it < T.size() + 8 && !located; ++it) {
      const Tri& t = T[cur];
      int go = -1;
      for (int k = 0; k < 3 && go < 0; ++k)
        if (orient(pts[t.v[k]], pts[t.v[(k + 1) % 3]], p) < 0.0 && t.nb[k] >= 0) go = k;
      if (go < 0)
        located = true;
      else
        cur = (size_t)t.nb[go];
    }
    if (!located) {
      for (size_t t = 0; t < T.size(); ++t)
        if (T[t].alive && orient(pts[T[t].v[0]], pts[T[t].v[1]], p) >= 0.0 &&
            orient(pts[T[t].v[1]], pts[T[t].v[2]], p) >= 0.0 && orient(pts[T[t].v[2]], pts[T[t].v[0]], p) >= 0.0) {
          cur = t;
          break;
        }
    }
    // cavity: triangles whose circumcircle holds p, grown from the containing one
    const uint32_t stamp = (uint32_t)i + 1;
    if (mark.size() < T.size()) mark.resize(T.size(), 0);
    auto in_cav = [&](size_t t) { return mark[t] == stamp; };
    cav.clear();
    stack.assign(1, cur);
    mark[cur] = stamp;
    while (!stack.empty()) {
      const size_t t = stack.back();
      stack.pop_back();
      cav.push_back(t);
      for (int k = 0; k < 3; ++k) {
        const int64_t nb = T[t].nb[k];
        if (nb < 0 || in_cav((size_t)nb)) continue;
        const Tri& u = T[(size_t)nb];
        if (in_circle(pts[u.v[0]], pts[u.v[1]], pts[u.v[2]], p)) {
          mark[(size_t)nb] = stamp;
          stack.push_back((size_t)nb);
        }
      }
    }
    // the cavity must be star-shaped from p: drop triangles whose outer edge p cannot see
    for (bool changed = true; changed;) {
      changed = false;
      bedges.clear();
      for (size_t t : cav) {
        if (!in_cav(t)) continue;
        for (int k = 0; k < 3; ++k) {
          const int64_t nb = T[t].nb[k];
          if (nb >= 0 && in_cav((size_t)nb)) continue;
          const uint32_t a = T[t].v[k], b = T[t].v[(k + 1) % 3];
          if (orient(pts[a], pts[b], p) <= 0.0 && t != cur) {
            mark[t] = 0;
            changed = true;
            break;
          }
          bedges.push_back({a, b, nb});
        }
        if (changed) break;
      }
    }
    for (size_t t : cav)
      if (in_cav(t)) {
        T[t].alive = false;
        mark[t] = 0;
        free_slots.push_back(t);
      }
    // re-triangulate the cavity: (a, b, p) per boundary edge
    std::unordered_map<uint32_t, size_t> by_start, by_end;
    std::vector<size_t> made;
    for (const BEdge& e : bedges) {
      size_t idx;
      const Tri nt{{e.a, e.b, (uint32_t)i}, {e.out, -1, -1}, true};
      if (!free_slots.empty()) {
        idx = free_slots.back();
        free_slots.pop_back();
        T[idx] = nt;
      } else {
        idx = T.size();
        T.push_back(nt);
      }
      made.push_back(idx);
      by_start[e.a] = idx;
      by_end[e.b] = idx;
      if (e.out >= 0) {
        Tri& o = T[(size_t)e.out];
        for (int k = 0; k < 3; ++k)
          if (o.v[k] == e.b && o.v[(k + 1) % 3] == e.a) o.nb[k] = (int64_t)idx;
      }
    }
    for (size_t idx : made) {
      Tri& t = T[idx];
      t.nb[1] = (int64_t)by_start.at(t.v[1]);  // edge b -> p is edge p -> b of the triangle starting at b
      t.nb[2] = (int64_t)by_end.at(t.v[0]);    // edge p -> a is edge a -> p of the triangle ending at a
    }
    last = made.empty() ? cur : made[0];
  }
  std::vector<Tri> out;
  std::vector<int64_t> remap(T.size(), -1);
  for (size_t t = 0; t < T.size(); ++t)
    if (T[t].alive && T[t].v[0] < n && T[t].v[1] < n && T[t].v[2] < n) {
      remap[t] = (int64_t)out.size();
      out.push_back(T[t]);
    }
  for (Tri& t : out)
    for (int k = 0; k < 3; ++k) t.nb[k] = t.nb[k] >= 0 ? remap[(size_t)t.nb[k]] : -1;
  return out;
}

// drop triangles outside the fluid: all three generators fixed and the centroid outside
std::vector<Tri> keep_fluid(const std::vector<Tri>& T, const std::vector<P>& pts, const std::vector<uint8_t>& fixed,
                            const Geometry& g) {
  std::vector<int64_t> remap(T.size(), -1);
  std::vector<Tri> out;
  for (size_t t = 0; t < T.size(); ++t) {
    const Tri& x = T[t];
    bool keep = !(fixed[x.v[0]] && fixed[x.v[1]] && fixed[x.v[2]]);
    if (!keep) {
      const P c{(pts[x.v[0]].x + pts[x.v[1]].x + pts[x.v[2]].x) / 3.0,
                (pts[x.v[0]].y + pts[x.v[1]].y + pts[x.v[2]].y) / 3.0};
      keep = inside(g, c);
    }
    if (keep) {
      remap[t] = (int64_t)out.size();
      out.push_back(x);
    }
  }
  for (Tri& t : out)
    for (int k = 0; k < 3; ++k) t.nb[k] = t.nb[k] >= 0 ? remap[(size_t)t.nb[k]] : -1;
  return out;
}

// size-weighted Laplacian step of the free generators (delaunay.rs:335-460)
void smooth_generators(std::vector<P>& pts, const std::vector<Tri>& T, const std::vector<uint8_t>& fixed,
                       const Sizing& size) {
  const size_t n = pts.size();
  std::vector<double> sx(n, 0.0), sy(n, 0.0), sw(n, 0.0);
  for (const Tri& t : T)
    for (int k = 0; k < 3; ++k)
      for (int j = 1; j < 3; ++j) {
        const uint32_t a = t.v[k], b = t.v[(k + j) % 3];
        const double w = 1.0 / std::max(size(pts[b]), 1e-6);
        sx[a] += pts[b].x * w;
        sy[a] += pts[b].y * w;
        sw[a] += w;
      }
  std::vector<P> out(pts);
  for (size_t i = 0; i < n; ++i) {
    if (fixed[i] || sw[i] == 0.0) continue;
    const P q{pts[i].x + (sx[i] / sw[i] - pts[i].x) * 0.1, pts[i].y + (sy[i] / sw[i] - pts[i].y) * 0.1};
    if (inside(size.g, q)) out[i] = q;
  }
  pts.swap(out);
}

// dual point of a triangle: the circumcentre when it lies inside (or on) it, else the centroid
P dual_point(P a, P b, P c) {
  const double d = 2.0 * (a.x * (b.y - c.y) + b.x * (c.y - a.y) + c.x * (a.y - b.y));
  const P g{(a.x + b.x + c.x) / 3.0, (a.y + b.y + c.y) / 3.0};
  if (std::fabs(d) < 1e-300) return g;
  const double a2 = a.x * a.x + a.y * a.y, b2 = b.x * b.x + b.y * b.y, c2 = c.x * c.x + c.y * c.y;
  const P cc{(a2 * (b.y - c.y) + b2 * (c.y - a.y) + c2 * (a.y - b.y)) / d,
             (a2 * (c.x - b.x) + b2 * (a.x - c.x) + c2 * (b.x - a.x)) / d};
  const double area2 = orient(a, b, c), tol = -1e-12 * std::fabs(area2);
  if (orient(a, b, cc) >= tol && orient(b, c, cc) >= tol && orient(c, a, cc) >= tol) return cc;
  return g;
}


// delaunay.rs triangulate (:125-193): generators, triangulation, smoothing
void triangulate(const Geometry& geo, double min_cell_size, double max_cell_size, double growth_rate, double domain_x,
                 double domain_y, uint64_t seed, std::vector<P>& pts, std::vector<uint8_t>& fixed,
                 std::vector<Tri>& T) {
  if (!(min_cell_size > 0.0) || !(max_cell_size >= min_cell_size) || !(domain_x > 0.0) || !(domain_y > 0.0))
    throw std::invalid_argument("voronoi mesher: bad sizes");
  const Sizing size{geo, min_cell_size, max_cell_size, growth_rate};
  pts.clear();
  fixed.clear();
  {
    std::map<std::pair<int64_t, int64_t>, size_t> seen;  // quantised de-duplication (delaunay.rs:137-149)
    for (const P& p : boundary_points(geo, min_cell_size)) {
      const auto key = std::make_pair((int64_t)std::llround(p.x * 100000.0), (int64_t)std::llround(p.y * 100000.0));
      if (seen.emplace(key, pts.size()).second) {
        pts.push_back(p);
        fixed.push_back(1);
      }
    }
  }
  Rng rng{seed};
  for (const P& p : poisson_points(pts, size, domain_x, domain_y, rng)) {
    pts.push_back(p);
    fixed.push_back(0);
  }
  {
    std::vector<size_t> ord(pts.size());
    for (size_t i = 0; i < ord.size(); ++i) ord[i] = i;
    std::vector<uint64_t> key(pts.size());
    for (size_t i = 0; i < pts.size(); ++i) key[i] = morton(pts[i].x, pts[i].y, domain_x, domain_y);
    std::stable_sort(ord.begin(), ord.end(), [&](size_t a, size_t b) { return key[a] < key[b]; });
    std::vector<P> sp(pts.size());
    std::vector<uint8_t> sf(pts.size());
    for (size_t i = 0; i < ord.size(); ++i) {
      sp[i] = pts[ord[i]];
      sf[i] = fixed[ord[i]];
    }
    pts.swap(sp);
    fixed.swap(sf);
  }
  T = keep_fluid(delaunay(pts, domain_x, domain_y), pts, fixed, geo);
  for (int it = 0; it < 20; ++it) {
    smooth_generators(pts, T, fixed, size);
    T = keep_fluid(delaunay(pts, domain_x, domain_y), pts, fixed, geo);
  }
}

}  // namespace

Mesh generate_voronoi_mesh(const Geometry& geo, double min_cell_size, double max_cell_size, double growth_rate,
                           double domain_x, double domain_y, uint64_t seed) {
  std::vector<P> pts;
  std::vector<uint8_t> fixed;
  std::vector<Tri> T;
  triangulate(geo, min_cell_size, max_cell_size, growth_rate, domain_x, domain_y, seed, pts, fixed, T);
  const size_t n = pts.size(), nt = T.size();
  // every generator must be used and every hull vertex must have exactly one fan
  std::vector<int64_t> first_tri(n, -1);
  for (size_t t = 0; t < nt; ++t)
    for (int k = 0; k < 3; ++k) first_tri[T[t].v[k]] = (int64_t)t;
  for (size_t i = 0; i < n; ++i)
    if (first_tri[i] < 0) throw std::runtime_error("voronoi mesher: a generator lies in no triangle");

  // 4. dual mesh
  Mesh m;
  for (size_t t = 0; t < nt; ++t) {
    const P d = dual_point(pts[T[t].v[0]], pts[T[t].v[1]], pts[T[t].v[2]]);
    m.vx.push_back(d.x);
    m.vy.push_back(d.y);
    m.v_fixed.push_back(0);
  }
  std::vector<int64_t> gen_vertex(n, -1);  // a boundary generator as a polygon vertex
  std::map<std::pair<uint32_t, uint32_t>, uint32_t> mid_vertex;
  auto vtx = [&](P p, uint8_t fx) {
    m.vx.push_back(p.x);
    m.vy.push_back(p.y);
    m.v_fixed.push_back(fx);
    return (uint32_t)(m.vx.size() - 1);
  };
  auto mid_of = [&](uint32_t a, uint32_t b) {
    const auto key = std::make_pair(std::min(a, b), std::max(a, b));
    auto it = mid_vertex.find(key);
    if (it != mid_vertex.end()) return it->second;
    const uint32_t v = vtx({(pts[a].x + pts[b].x) * 0.5, (pts[a].y + pts[b].y) * 0.5}, 1);
    mid_vertex.emplace(key, v);
    return v;
  };
  auto gen_of = [&](uint32_t g) {
    if (gen_vertex[g] < 0) gen_vertex[g] = vtx(pts[g], 1);
    return (uint32_t)gen_vertex[g];
  };
  // faces: one record per Delaunay edge (sorted), boundary half-faces after it
  std::map<std::pair<uint32_t, uint32_t>, std::array<int64_t, 2>> edge_tris;
  for (size_t t = 0; t < nt; ++t)
    for (int k = 0; k < 3; ++k) {
      const uint32_t a = T[t].v[k], b = T[t].v[(k + 1) % 3];
      auto& e = edge_tris.try_emplace(std::make_pair(std::min(a, b), std::max(a, b)), std::array<int64_t, 2>{-1, -1})
                    .first->second;
      (e[0] < 0 ? e[0] : e[1]) = (int64_t)t;
    }
  std::vector<std::vector<uint32_t>> cell_faces(n);
  auto face = [&](uint32_t v1, uint32_t v2, uint32_t owner, uint32_t neighbor, uint32_t bnd, double nx, double ny) {
    const double len = std::hypot(m.vx[v2] - m.vx[v1], m.vy[v2] - m.vy[v1]);
    if (!(len > 1e-12)) return;  // cocircular generators: the cells touch at a point
    const uint32_t f = (uint32_t)m.face_cx.size();
    m.face_v1.push_back(v1);
    m.face_v2.push_back(v2);
    m.face_owner.push_back(owner);
    m.face_neighbor.push_back(neighbor);
    m.face_boundary.push_back(bnd);
    m.face_nx.push_back(nx);
    m.face_ny.push_back(ny);
    m.face_area.push_back(len);
    m.face_cx.push_back(0.0);
    m.face_cy.push_back(0.0);
    cell_faces[owner].push_back(f);
    if (neighbor != kNoNeighbor) cell_faces[neighbor].push_back(f);
  };
  auto btype = [&](double x) {
    if (x < 1e-6) return (uint32_t)kInlet;
    if (std::fabs(x - domain_x) < 1e-6) return (uint32_t)kOutlet;
    return (uint32_t)kWall;
  };
  for (const auto& [e, tr] : edge_tris) {
    const uint32_t a = e.first, b = e.second;
    double ex = pts[b].x - pts[a].x, ey = pts[b].y - pts[a].y;
    const double el = std::hypot(ex, ey);
    ex /= el;
    ey /= el;
    if (tr[1] >= 0) {
      face((uint32_t)tr[0], (uint32_t)tr[1], a, b, kNone, ex, ey);
      continue;
    }
    // hull edge: interior face dual point -> midpoint, boundary half-faces midpoint -> generator
    const uint32_t mid = mid_of(a, b), t = (uint32_t)tr[0];
    face(t, mid, a, b, kNone, ex, ey);
    const Tri& x = T[t];
    const P c{(pts[x.v[0]].x + pts[x.v[1]].x + pts[x.v[2]].x) / 3.0,
              (pts[x.v[0]].y + pts[x.v[1]].y + pts[x.v[2]].y) / 3.0};
    double nx = ey, ny = -ex;  // outward: away from the triangle
    if (((pts[a].x + pts[b].x) * 0.5 - c.x) * nx + ((pts[a].y + pts[b].y) * 0.5 - c.y) * ny < 0.0) {
      nx = -nx;
      ny = -ny;
    }
    const uint32_t va = gen_of(a), vb = gen_of(b);
    face(mid, va, a, kNoNeighbor, btype(0.5 * (m.vx[mid] + m.vx[va])), nx, ny);
    face(mid, vb, b, kNoNeighbor, btype(0.5 * (m.vx[mid] + m.vx[vb])), nx, ny);
  }
  // cells: the fan of triangles around each generator, CCW
  m.cell_face_offsets.push_back(0);
  m.cell_vertex_offsets.push_back(0);
  for (uint32_t gidx = 0; gidx < (uint32_t)n; ++gidx) {
    auto pos = [&](size_t t) {
      for (int k = 0; k < 3; ++k)
        if (T[t].v[k] == gidx) return k;
      throw std::logic_error("voronoi mesher: broken fan");
    };
    // rewind clockwise to the start of an open fan (or all the way round)
    size_t start = (size_t)first_tri[gidx];
    bool open = false;
    for (size_t guard = 0; guard <= nt; ++guard) {
      const int64_t prev = T[start].nb[pos(start)];  // across edge g -> a
      if (prev < 0) {
        open = true;
        break;
      }
      if ((size_t)prev == (size_t)first_tri[gidx]) break;
      start = (size_t)prev;
    }
    std::vector<uint32_t> poly;
    if (open) {
      const Tri& s = T[start];
      poly.push_back(gen_of(gidx));
      poly.push_back(mid_of(gidx, s.v[(pos(start) + 1) % 3]));
    }
    size_t t = start, count = 0;
    for (;;) {
      poly.push_back((uint32_t)t);
      ++count;
      const int k = pos(t);
      const int64_t next = T[t].nb[(k + 2) % 3];  // across edge b -> g
      if (next < 0) {
        if (!open) throw std::logic_error("voronoi mesher: broken fan");
        poly.push_back(mid_of(gidx, T[t].v[(k + 2) % 3]));
        break;
      }
      if ((size_t)next == start) break;
      t = (size_t)next;
      if (count > nt) throw std::logic_error("voronoi mesher: broken fan");
    }
    // a hull vertex with two separate fans would be a pinched (non-manifold) boundary
    size_t deg = 0;
    for (uint32_t f : cell_faces[gidx]) deg += m.face_boundary[f] != kNone;
    if (deg > 2) throw std::runtime_error("voronoi mesher: pinched boundary at a generator");
    m.cell_vertices.insert(m.cell_vertices.end(), poly.begin(), poly.end());
    m.cell_vertex_offsets.push_back((uint32_t)m.cell_vertices.size());
    m.cell_faces.insert(m.cell_faces.end(), cell_faces[gidx].begin(), cell_faces[gidx].end());
    m.cell_face_offsets.push_back((uint32_t)m.cell_faces.size());
    m.cell_cx.push_back(pts[gidx].x);
    m.cell_cy.push_back(pts[gidx].y);
    m.cell_vol.push_back(0.0);
  }
  m.recalculate_geometry();
  return m;
}

// generate_delaunay_mesh (delaunay.rs:732-846): the triangles themselves as
// cells (centroid, area), one face per edge; a hull edge is a boundary face
// typed by position (the reference leaves an unshared edge with a free end as
// a face with neither neighbour nor boundary type; here every hull edge is a
// boundary).  Normals point out of the owner, the first cell to use the edge.
Mesh generate_delaunay_mesh(const Geometry& geo, double min_cell_size, double max_cell_size, double growth_rate,
                            double domain_x, double domain_y, uint64_t seed) {
  std::vector<P> pts;
  std::vector<uint8_t> fixed;
  std::vector<Tri> T;
  triangulate(geo, min_cell_size, max_cell_size, growth_rate, domain_x, domain_y, seed, pts, fixed, T);
  Mesh m;
  for (size_t i = 0; i < pts.size(); ++i) {
    m.vx.push_back(pts[i].x);
    m.vy.push_back(pts[i].y);
    m.v_fixed.push_back(fixed[i]);
  }
  std::map<std::pair<uint32_t, uint32_t>, uint32_t> edge_face;
  m.cell_face_offsets.push_back(0);
  m.cell_vertex_offsets.push_back(0);
  for (size_t t = 0; t < T.size(); ++t) {
    const uint32_t c = (uint32_t)t;
    const P a = pts[T[t].v[0]], b = pts[T[t].v[1]], d = pts[T[t].v[2]];
    m.cell_cx.push_back((a.x + b.x + d.x) / 3.0);
    m.cell_cy.push_back((a.y + b.y + d.y) / 3.0);
    m.cell_vol.push_back(0.5 * std::fabs((b.x - a.x) * (d.y - a.y) - (d.x - a.x) * (b.y - a.y)));
    for (int k = 0; k < 3; ++k) {
      const uint32_t u = T[t].v[k], v = T[t].v[(k + 1) % 3];
      const auto key = std::make_pair(std::min(u, v), std::max(u, v));
      auto it = edge_face.find(key);
      if (it != edge_face.end()) {
        m.face_neighbor[it->second] = c;
        m.face_boundary[it->second] = kNone;
        m.cell_faces.push_back(it->second);
        continue;
      }
      const uint32_t f = (uint32_t)m.face_cx.size();
      const P pa = pts[key.first], pb = pts[key.second];
      const double fx = (pa.x + pb.x) / 2.0, fy = (pa.y + pb.y) / 2.0, len = std::hypot(pb.x - pa.x, pb.y - pa.y);
      double nx = (pb.y - pa.y) / len, ny = (pa.x - pb.x) / len;
      if ((fx - m.cell_cx[c]) * nx + (fy - m.cell_cy[c]) * ny < 0.0) {
        nx = -nx;
        ny = -ny;
      }
      m.face_v1.push_back(key.first);
      m.face_v2.push_back(key.second);
      m.face_owner.push_back(c);
      m.face_neighbor.push_back(kNoNeighbor);
      m.face_boundary.push_back(fx < 1e-6 ? kInlet : std::fabs(fx - domain_x) < 1e-6 ? kOutlet : kWall);
      m.face_nx.push_back(nx);
      m.face_ny.push_back(ny);
      m.face_area.push_back(len);
      m.face_cx.push_back(fx);
      m.face_cy.push_back(fy);
      edge_face.emplace(key, f);
      m.cell_faces.push_back(f);
    }
    m.cell_face_offsets.push_back((uint32_t)m.cell_faces.size());
    for (int k = 0; k < 3; ++k) m.cell_vertices.push_back(T[t].v[k]);  // CCW
    m.cell_vertex_offsets.push_back((uint32_t)m.cell_vertices.size());
  }
  return m;
}

}  // namespace cfd2
