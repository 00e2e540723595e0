// Host-side mesh model: the `Mesh` SoA input of the hot path.
//
// Restates the reference's mesh data model and its deterministic cut-cell
// generator (the input both reference solver tests use):
//   Mesh struct            src/solver/mesh/structs.rs:12-42
//   Geometry SDFs          src/solver/mesh/geometry.rs:24-260
//   quadtree refinement    src/solver/mesh/quadtree.rs:39-103
//   cut-cell generator     src/solver/mesh/cut_cell.rs:10-510
//   smooth / recalc / skew structs.rs:61-320
// All geometry is f64 exactly as in the reference; indices are u32 (the
// reference's usize never exceeds 2^32 at the sizes we run).  Compile with
// -ffp-contract=off: Rust never contracts a*b+c into an FMA.
#pragma once
#include <cstdint>
#include <vector>

namespace cfd2 {

enum BoundaryCode : uint32_t { kNone = 0, kInlet = 1, kOutlet = 2, kWall = 3 };

// Geometry kinds of the reference (geometry.rs) plus the CircleObstacle used by
// src/solver/mesh/tests.rs:4-61.
enum GeometryKind : int32_t {
  kBackwardsStep = 0,        // length, height_inlet, height_outlet, step_x
  kChannelWithObstacle = 1,  // length, height, cx, cy, radius
  kRectangularChannel = 2,   // length, height
  kCircleObstacle = 3,       // cx, cy, radius, xmin, ymin, xmax, ymax
};

struct Geometry {
  int32_t kind;
  double p[8];
  double sdf(double x, double y) const;
};

struct Mesh {
  std::vector<double> vx, vy;
  std::vector<uint8_t> v_fixed;
  std::vector<uint32_t> face_v1, face_v2, face_owner, face_neighbor, face_boundary;
  std::vector<double> face_nx, face_ny, face_area, face_cx, face_cy;
  std::vector<double> cell_cx, cell_cy, cell_vol;
  std::vector<uint32_t> cell_faces, cell_face_offsets;
  std::vector<uint32_t> cell_vertices, cell_vertex_offsets;

  uint32_t num_cells() const { return (uint32_t)cell_cx.size(); }
  uint32_t num_faces() const { return (uint32_t)face_cx.size(); }

  void recalculate_geometry();
  double calculate_max_skewness() const;
  // Returns the number of smoothing iterations performed.
  int smooth(const Geometry& geo, double target_skew, int max_iterations);
};

static constexpr uint32_t kNoNeighbor = 0xFFFFFFFFu;

Mesh generate_cut_cell_mesh(const Geometry& geo, double min_cell_size, double max_cell_size,
                            double growth_rate, double domain_x, double domain_y);
// seeded restatement of generate_voronoi_mesh (voronoi.rs:23; voronoi.cpp)
Mesh generate_voronoi_mesh(const Geometry& geo, double min_cell_size, double max_cell_size, double growth_rate,
                           double domain_x, double domain_y, uint64_t seed);
// seeded restatement of generate_delaunay_mesh (delaunay.rs:732; triangle cells)
Mesh generate_delaunay_mesh(const Geometry& geo, double min_cell_size, double max_cell_size, double growth_rate,
                            double domain_x, double domain_y, uint64_t seed);

}  // namespace cfd2
