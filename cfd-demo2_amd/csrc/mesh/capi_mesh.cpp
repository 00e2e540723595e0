// C ABI for the host mesh: generation, smoothing, view, binary dump/load.
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <exception>
#include <memory>
#include <new>
#include <string>

#include "../../../include/cfd2_amd.h"
#include "../host/error.hpp"
#include "mesh.hpp"

struct cfd_mesh {
  cfd2::Mesh m;
};

using cfd2::set_error;

static bool to_geo(const cfd_geometry* g, cfd2::Geometry* out) {
  if (!g || g->kind < 0 || g->kind > 3) return false;
  out->kind = g->kind;
  std::memcpy(out->p, g->p, sizeof(out->p));
  return true;
}

// Binary format "CFDMESH1": u64 counts followed by the raw SoA arrays.
template <class T>
static bool wvec(FILE* f, const std::vector<T>& v) {
  uint64_t n = v.size();
  if (fwrite(&n, 8, 1, f) != 1) return false;
  return n == 0 || fwrite(v.data(), sizeof(T), n, f) == n;
}
// `left` = bytes of the file not read yet: a count larger than what remains
// is a truncated or corrupt file, refused before anything is allocated.
template <class T>
static bool rvec(FILE* f, std::vector<T>& v, uint64_t& left) {
  uint64_t n = 0;
  if (left < 8 || fread(&n, 8, 1, f) != 1) return false;
  left -= 8;
  if (n > left / sizeof(T)) return false;
  v.resize(n);
  if (n && fread(v.data(), sizeof(T), n, f) != n) return false;
  left -= n * sizeof(T);
  return true;
}

// Array lengths and offsets of a loaded mesh agree with each other (every
// index array is checked again by build_topology when a solver is made).
static const char* mesh_consistency(const cfd2::Mesh& m) {
  const size_t nc = m.cell_cx.size(), nf = m.face_owner.size(), nv = m.vx.size();
  if (m.cell_cy.size() != nc || m.cell_vol.size() != nc) return "cell arrays differ in length";
  if (m.face_neighbor.size() != nf || m.face_boundary.size() != nf || m.face_nx.size() != nf ||
      m.face_ny.size() != nf || m.face_area.size() != nf || m.face_cx.size() != nf || m.face_cy.size() != nf ||
      m.face_v1.size() != nf || m.face_v2.size() != nf)
    return "face arrays differ in length";
  if (m.vy.size() != nv || m.v_fixed.size() != nv) return "vertex arrays differ in length";
  if (m.cell_face_offsets.size() != nc + 1 || m.cell_vertex_offsets.size() != nc + 1)
    return "offset arrays must hold num_cells + 1 entries";
  auto monotone = [](const std::vector<uint32_t>& off, size_t total) {
    if (off.empty() || off[0] != 0 || off.back() != total) return false;
    for (size_t i = 1; i < off.size(); ++i)
      if (off[i] < off[i - 1]) return false;
    return true;
  };
  if (!monotone(m.cell_face_offsets, m.cell_faces.size())) return "cell_face_offsets not monotone / not ending at the face list";
  if (!monotone(m.cell_vertex_offsets, m.cell_vertices.size()))
    return "cell_vertex_offsets not monotone / not ending at the vertex list";
  for (uint32_t fi : m.cell_faces)
    if (fi >= nf) return "cell_faces index out of range";
  for (uint32_t vi : m.cell_vertices)
    if (vi >= nv) return "cell_vertices index out of range";
  for (size_t k = 0; k < nf; ++k) {
    if (m.face_owner[k] >= nc) return "face_owner out of range";
    if (m.face_neighbor[k] != 0xFFFFFFFFu && m.face_neighbor[k] >= nc) return "face_neighbor out of range";
    if (m.face_v1[k] >= nv || m.face_v2[k] >= nv) return "face vertex out of range";
  }
  return nullptr;
}

extern "C" {

cfd_status cfd_mesh_generate_cut_cell(const cfd_geometry* geo, double min_cell_size,
                                      double max_cell_size, double growth_rate, double domain_x,
                                      double domain_y, cfd_mesh** out) {
  if (!out) return set_error(CFD_ERR_INVALID, "out is null");
  cfd2::Geometry g;
  if (!to_geo(geo, &g)) return set_error(CFD_ERR_INVALID, "bad geometry");
  if (!(min_cell_size > 0) || !(max_cell_size > 0) || !(domain_x > 0) || !(domain_y > 0))
    return set_error(CFD_ERR_INVALID, "cell sizes and domain must be positive");
  try {
    auto* m = new cfd_mesh;
    m->m = cfd2::generate_cut_cell_mesh(g, min_cell_size, max_cell_size, growth_rate, domain_x,
                                        domain_y);
    *out = m;
    return CFD_OK;
  } catch (const std::exception& e) {
    return set_error(CFD_ERR_INTERNAL, e.what());
  }
}

cfd_status cfd_mesh_generate_voronoi(const cfd_geometry* geo, double min_cell_size, double max_cell_size,
                                     double growth_rate, double domain_x, double domain_y, uint64_t seed,
                                     cfd_mesh** out) {
  if (!out) return set_error(CFD_ERR_INVALID, "out is null");
  cfd2::Geometry g;
  if (!to_geo(geo, &g)) return set_error(CFD_ERR_INVALID, "bad geometry");
  if (!(min_cell_size > 0) || !(max_cell_size >= min_cell_size) || !(domain_x > 0) || !(domain_y > 0))
    return set_error(CFD_ERR_INVALID, "cell sizes and domain must be positive, max >= min");
  try {
    auto* m = new cfd_mesh;
    try {
      m->m = cfd2::generate_voronoi_mesh(g, min_cell_size, max_cell_size, growth_rate, domain_x, domain_y, seed);
    } catch (...) {
      delete m;
      throw;
    }
    *out = m;
    return CFD_OK;
  } catch (const std::invalid_argument& e) {
    return set_error(CFD_ERR_INVALID, e.what());
  } catch (const std::exception& e) {
    return set_error(CFD_ERR_INTERNAL, e.what());
  }
}

cfd_status cfd_mesh_generate_delaunay(const cfd_geometry* geo, double min_cell_size, double max_cell_size,
                                     double growth_rate, double domain_x, double domain_y, uint64_t seed,
                                     cfd_mesh** out) {
  if (!out) return set_error(CFD_ERR_INVALID, "out is null");
  cfd2::Geometry g;
  if (!to_geo(geo, &g)) return set_error(CFD_ERR_INVALID, "bad geometry");
  if (!(min_cell_size > 0) || !(max_cell_size >= min_cell_size) || !(domain_x > 0) || !(domain_y > 0))
    return set_error(CFD_ERR_INVALID, "cell sizes and domain must be positive, max >= min");
  try {
    auto* m = new cfd_mesh;
    try {
      m->m = cfd2::generate_delaunay_mesh(g, min_cell_size, max_cell_size, growth_rate, domain_x, domain_y, seed);
    } catch (...) {
      delete m;
      throw;
    }
    *out = m;
    return CFD_OK;
  } catch (const std::invalid_argument& e) {
    return set_error(CFD_ERR_INVALID, e.what());
  } catch (const std::exception& e) {
    return set_error(CFD_ERR_INTERNAL, e.what());
  }
}

cfd_status cfd_mesh_smooth(cfd_mesh* m, const cfd_geometry* geo, double target_skew,
                           int32_t max_iterations, int32_t* iters) {
  cfd2::Geometry g;
  if (!m || !to_geo(geo, &g)) return set_error(CFD_ERR_INVALID, "bad mesh/geometry");
  try {
    int it = m->m.smooth(g, target_skew, max_iterations);
    if (iters) *iters = it;
    return CFD_OK;
  } catch (const std::exception& e) {
    return set_error(CFD_ERR_INTERNAL, e.what());
  }
}

double cfd_mesh_max_skewness(const cfd_mesh* m) { return m ? m->m.calculate_max_skewness() : -1.0; }

cfd_status cfd_mesh_get_view(const cfd_mesh* m, cfd_mesh_view* v) {
  if (!m || !v) return set_error(CFD_ERR_INVALID, "null");
  const cfd2::Mesh& x = m->m;
  v->num_cells = x.num_cells();
  v->num_faces = x.num_faces();
  v->face_owner = x.face_owner.data();
  v->face_neighbor = x.face_neighbor.data();
  v->face_boundary = x.face_boundary.data();
  v->face_area = x.face_area.data();
  v->face_nx = x.face_nx.data();
  v->face_ny = x.face_ny.data();
  v->face_cx = x.face_cx.data();
  v->face_cy = x.face_cy.data();
  v->cell_cx = x.cell_cx.data();
  v->cell_cy = x.cell_cy.data();
  v->cell_vol = x.cell_vol.data();
  v->cell_face_offsets = x.cell_face_offsets.data();
  v->cell_faces = x.cell_faces.data();
  return CFD_OK;
}

cfd_status cfd_mesh_get_vertices(const cfd_mesh* m, uint32_t* nv, const double** vx,
                                 const double** vy, const uint8_t** vf) {
  if (!m) return set_error(CFD_ERR_INVALID, "null");
  if (nv) *nv = (uint32_t)m->m.vx.size();
  if (vx) *vx = m->m.vx.data();
  if (vy) *vy = m->m.vy.data();
  if (vf) *vf = m->m.v_fixed.data();
  return CFD_OK;
}

cfd_status cfd_mesh_get_topology(const cfd_mesh* m, const uint32_t** face_v1, const uint32_t** face_v2,
                                 const uint32_t** cell_vertex_offsets, const uint32_t** cell_vertices) {
  if (!m) return set_error(CFD_ERR_INVALID, "null");
  if (face_v1) *face_v1 = m->m.face_v1.data();
  if (face_v2) *face_v2 = m->m.face_v2.data();
  if (cell_vertex_offsets) *cell_vertex_offsets = m->m.cell_vertex_offsets.data();
  if (cell_vertices) *cell_vertices = m->m.cell_vertices.data();
  return CFD_OK;
}

#define MESH_FIELDS(X)                                                                          \
  X(vx) X(vy) X(v_fixed) X(face_v1) X(face_v2) X(face_owner) X(face_neighbor) X(face_boundary) \
      X(face_nx) X(face_ny) X(face_area) X(face_cx) X(face_cy) X(cell_cx) X(cell_cy) X(cell_vol) \
          X(cell_faces) X(cell_face_offsets) X(cell_vertices) X(cell_vertex_offsets)

cfd_status cfd_mesh_save(const cfd_mesh* m, const char* path) {
  if (!m || !path) return set_error(CFD_ERR_INVALID, "null");
  FILE* f = fopen(path, "wb");
  if (!f) return set_error(CFD_ERR_INVALID, std::string("cannot open ") + path);
  bool ok = fwrite("CFDMESH1", 1, 8, f) == 8;
#define W(name) ok = ok && wvec(f, m->m.name);
  MESH_FIELDS(W)
#undef W
  fclose(f);
  return ok ? CFD_OK : set_error(CFD_ERR_INTERNAL, "write failed");
}

cfd_status cfd_mesh_load(const char* path, cfd_mesh** out) {
  if (!out || !path) return set_error(CFD_ERR_INVALID, "null");
  try {
    std::unique_ptr<FILE, int (*)(FILE*)> fh(fopen(path, "rb"), fclose);
    FILE* f = fh.get();
    if (!f) return set_error(CFD_ERR_INVALID, std::string("cannot open ") + path);
    uint64_t left = 0;
    if (fseek(f, 0, SEEK_END) == 0) {
      const long end = ftell(f);
      left = end > 0 ? (uint64_t)end : 0;
    }
    rewind(f);
    char magic[8];
    bool ok = left >= 8 && fread(magic, 1, 8, f) == 8 && std::memcmp(magic, "CFDMESH1", 8) == 0;
    left = left >= 8 ? left - 8 : 0;
    std::unique_ptr<cfd_mesh> m(new cfd_mesh);
#define R(name) ok = ok && rvec(f, m->m.name, left);
    MESH_FIELDS(R)
#undef R
    fh.reset();
    if (!ok) return set_error(CFD_ERR_INVALID, std::string("bad mesh file (truncated or corrupt): ") + path);
    if (const char* why = mesh_consistency(m->m))
      return set_error(CFD_ERR_INVALID, std::string("inconsistent mesh file ") + path + ": " + why);
    *out = m.release();
    return CFD_OK;
  } catch (const std::bad_alloc&) {
    return set_error(CFD_ERR_INVALID, std::string("mesh file too large for host memory: ") + path);
  } catch (const std::exception& e) {
    return set_error(CFD_ERR_INTERNAL, e.what());
  }
}

void cfd_mesh_destroy(cfd_mesh* m) { delete m; }

}  // extern "C"
