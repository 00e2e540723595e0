// Host sanitizer run (SURVEY §5 "Run oracle checks under
// -fsanitize=address,undefined") -- TEST INFRASTRUCTURE ONLY.
//
// Builds, with AddressSanitizer + UBSan (tests/test_sanitize.py compiles it
// with g++ straight from the sources: this file, oracle/oracle.cpp and the
// product's host mesh code cut_cell.cpp / voronoi.cpp, which need no GPU):
//   - a cut-cell backwards-step mesh (smoothed) and a seeded Voronoi and
//     Delaunay channel-with-obstacle mesh,
//   - the oracle on each, one rank and three ranks (partition-aware AMG,
//     rank-segmented reductions), Jacobi and AMG, SOU + BDF2,
// and exits 0 when every field stays finite.  Any out-of-bounds access,
// use-after-free, overflow or other UB aborts the run with a report.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../cfd-demo2_amd/csrc/mesh/mesh.hpp"
#include "oracle.h"

namespace {

cfd_mesh_view view_of(const cfd2::Mesh& x) {
  cfd_mesh_view v{};
  v.num_cells = x.num_cells();
  v.num_faces = x.num_faces();
  v.face_owner = x.face_owner.data();
  v.face_neighbor = x.face_neighbor.data();
  v.face_boundary = x.face_boundary.data();
  v.face_area = x.face_area.data();
  v.face_nx = x.face_nx.data();
  v.face_ny = x.face_ny.data();
  v.face_cx = x.face_cx.data();
  v.face_cy = x.face_cy.data();
  v.cell_cx = x.cell_cx.data();
  v.cell_cy = x.cell_cy.data();
  v.cell_vol = x.cell_vol.data();
  v.cell_face_offsets = x.cell_face_offsets.data();
  v.cell_faces = x.cell_faces.data();
  return v;
}

int run(const char* name, const cfd2::Mesh& m, int nranks, uint32_t precond, uint32_t scheme, int local = 0) {
  cfd_config cfg{};
  cfg.n_outer_correctors = 20;
  cfg.convergence_lag = 1;
  cfg.fixed_outer = 3;
  cfg.fixed_inner = 10;
  cfg.max_restart = 50;
  cfg.max_outer_restarts = 20;
  cfg.fgmres_rtol = 1e-5f;
  cfg.fgmres_atol = 1e-7f;
  cfg.amg_rebuild_interval = 2;
  cfg.amg_local_aggregation = local;
  const cfd_mesh_view v = view_of(m);
  oracle_solver* s = oracle_create_dist(&v, &cfg, nranks);
  if (!s) {
    std::fprintf(stderr, "%s: oracle_create failed: %s\n", name, oracle_last_error());
    return 1;
  }
  const uint32_t n = m.num_cells();
  std::vector<double> uv(2 * (size_t)n, 0.0);
  for (uint32_t i = 0; i < n; ++i) uv[2 * i] = m.cell_cx[i] < 0.1 ? 1.0 : 0.1;
  oracle_set_u(s, uv.data());
  oracle_initialize_history(s);
  cfd_constants c;
  oracle_get_constants(s, &c);
  c.dt = 0.005f;
  c.viscosity = 0.01f;
  c.scheme = scheme;
  c.time_scheme = 1;
  c.precond_type = precond;
  oracle_set_constants(s, &c);
  int rc = 0;
  for (int k = 0; k < 4 && rc == 0; ++k)
    if (oracle_step(s) != 0) {
      std::fprintf(stderr, "%s: step failed: %s\n", name, oracle_last_error());
      rc = 1;
    }
  oracle_get_u(s, uv.data());
  for (double x : uv)
    if (!std::isfinite(x)) rc = 1;
  oracle_destroy(s);
  std::printf("%s: %u cells, %d rank(s)%s, precond %u, scheme %u: %s\n", name, n, nranks,
              local ? " (partition-aware AMG)" : "", precond, scheme, rc ? "FAILED" : "ok");
  return rc;
}

}  // namespace

int main() {
  oracle_set_threads(2);
  cfd2::Geometry step{cfd2::kBackwardsStep, {2.0, 0.5, 1.0, 0.5}};
  cfd2::Mesh a = cfd2::generate_cut_cell_mesh(step, 0.08, 0.08, 1.2, 2.0, 1.0);
  a.smooth(step, 0.3, 10);
  cfd2::Geometry chan{cfd2::kChannelWithObstacle, {3.0, 1.0, 1.0, 0.5, 0.2}};
  cfd2::Mesh b = cfd2::generate_voronoi_mesh(chan, 0.06, 0.15, 1.2, 3.0, 1.0, 11);
  cfd2::Mesh c = cfd2::generate_delaunay_mesh(chan, 0.06, 0.15, 1.2, 3.0, 1.0, 12);
  int rc = 0;
  for (int nr : {1, 3}) {
    rc |= run("cut-cell step", a, nr, 1, 1);
    rc |= run("voronoi channel", b, nr, 1, 0);
    rc |= run("delaunay channel", c, nr, 0, 2);
  }
  setenv("CFD_AMG_REPLICATE_ROWS", "40", 1);  // distributed coarse levels on these small meshes
  rc |= run("cut-cell step", a, 3, 1, 1, 1);
  rc |= run("voronoi channel", b, 2, 1, 0, 1);
  return rc;
}
