// Host sanitizer driver for the product's host-side setup code (no GPU):
// slab topology + halo plans for 1-4 ranks, and the host AMG hierarchy
// (greedy aggregation, R = P^T, Galerkin products) with partition-aware
// aggregation, on a cut-cell, a Voronoi and a Delaunay mesh.  Built with
// ASan + UBSan by tests/test_sanitize.py; consistency checks on the way.
#include <cstdio>
#include <stdexcept>
#include <vector>

#include "../../cfd-demo2_amd/csrc/host/solver_impl.hpp"
#include "../../cfd-demo2_amd/csrc/mesh/mesh.hpp"

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

void check(bool ok, const char* what) {
  if (!ok) throw std::runtime_error(what);
}

void run(const char* name, const cfd2::Mesh& m) {
  const cfd_mesh_view v = view_of(m);
  const uint32_t n = m.num_cells();
  for (int R = 1; R <= 4 && (uint32_t)R <= cfd2::red_geom(n).nseg; ++R) {
    const auto starts = cfd2::partition_starts(n, R);
    uint64_t rows = 0, nnz = 0, sends = 0, recvs = 0, reg_rows = 0;
    for (int r = 0; r < R; ++r) {
      cfd2::Topology t;
      cfd2::build_topology(v, t, (uint32_t)starts[r], (uint32_t)starts[r + 1]);
      const cfd2::HaloPlan p =
          cfd2::build_halo_plan(starts, r, t.srow.data(), t.N, t.scol.data(), t.ghost, t.glo, t.npad);
      rows += t.N;
      nnz += t.scol.size();
      // aligned-slot coupled ELL: every CSR entry in its own, increasing slot,
      // with its column there; slots in use and gaps as the mask says
      for (uint32_t i = 0; i < t.N; ++i) {
        const uint32_t a = t.srow[i], len = t.srow[i + 1] - a;
        uint32_t on = 0;
        int prev = -1;
        for (uint32_t q = 0; q < len; ++q) {
          const int s = t.tslot[a + q];
          check(s > prev && s < t.ws, "aligned slots must increase inside the ELL width");
          check(t.tcol[(size_t)s * t.ld + i] == t.rel(t.scol[a + q]), "aligned slot holds its column");
          on |= 1u << s;
          prev = s;
        }
        const uint32_t used = t.tlg[i] & 0x7Fu, gap = t.tlg[i] >> 8;
        check(used == (uint32_t)prev + 1 && (gap | on) == (1u << used) - 1u && !(gap & on), "slot mask");
        check(t.tslot[a + t.ell_drank[i]] == t.tdrank8[i], "diagonal slot");
        bool all_modal = true;
        for (int r = 0; r < t.ws; ++r) {
          const int32_t c = t.tcol[(size_t)r * t.ld + i];
          check(c >= -(int32_t)t.glo && c < (int32_t)(t.npad + t.ghi), "virtual columns inside the vectors");
          if (r >= (int)t.tmode.size() || c != (int32_t)i + t.tmode[r]) all_modal = false;
        }
        // regular row (the kernels derive its columns): flagged iff every slot
        // holds row + tmode[slot] (aligned-slot layout only)
        const bool typed = t.ws <= 8;
        check(((t.tlg[i] & 0x80u) != 0) == (typed && all_modal), "regular-row flag");
        if (t.tlg[i] & 0x80u) reg_rows++;
      }
      for (const auto& h : p.peers) {
        sends += h.send_cnt;
        recvs += h.recv_cnt;
      }
    }
    check(rows == n, "rows do not add up");
    check(sends == recvs, "halo sends != receives");
    // host AMG hierarchy of a synthetic SPD-like matrix on the global pattern
    cfd2::Topology g;
    cfd2::build_topology(v, g);
    cfd2::HostCsr A;
    A.rows = A.cols = n;
    A.row = g.srow;
    A.col = g.scol;
    A.val.resize(g.scol.size());
    for (uint32_t i = 0; i < n; ++i)
      for (uint32_t k = g.srow[i]; k < g.srow[i + 1]; ++k)
        A.val[k] = g.scol[k] == i ? (float)(g.srow[i + 1] - g.srow[i]) : -1.0f;
    const auto H = cfd2::build_amg_hierarchy(A, 20, starts);
    check(!H.empty() && H[0].A.rows == n, "empty hierarchy");
    {  // partition-aware mode: no aggregate of a partitioned level straddles two parts
      const auto HL = cfd2::build_amg_hierarchy(A, 20, starts, true, 40);
      for (size_t l = 0; l + 1 < HL.size() && HL[l].A.rows > 40; ++l)
        for (int q = 0; q < R; ++q)
          for (uint64_t i = HL[l].part[q]; i < HL[l].part[q + 1]; ++i)
            check(HL[l].agg[i] >= HL[l + 1].part[q] && HL[l].agg[i] < HL[l + 1].part[q + 1],
                  "partition-aware aggregate straddles ranks");
    }
    for (size_t l = 0; l + 1 < H.size(); ++l)
      check(H[l].has_op && H[l + 1].A.rows == H[l].nc, "level sizes");
    // down-leg pair partitions (k_amg_resrestrict_pair) of every level pair
    // with a coarser level, at the kernel's capacity and at a small one
    for (size_t l = 0; l + 2 < H.size(); ++l)
      for (uint32_t cap : {1024u, 96u}) {
        const cfd2::HostCsr& M = H[l + 1].A;
        const uint32_t nm = (uint32_t)M.rows;
        std::vector<uint32_t> mrow(nm + 1, 0), mcol;
        for (uint32_t g = 0; g < nm; ++g) {
          for (uint32_t k = M.row[g]; k < M.row[g + 1]; ++k)
            if (M.col[k] != g) mcol.push_back(M.col[k]);
          mrow[g + 1] = (uint32_t)mcol.size();
        }
        cfd2::PairPartition pp;
        if (!cfd2::build_pair_partition(H[l].r_row, H[l].r_col, H[l + 1].r_row, H[l + 1].r_col, mrow, mcol, cap, pp))
          continue;  // an aggregate alone over the capacity: no pair here
        std::vector<int> owner(nm, -1);
        const uint32_t nb = (uint32_t)pp.jb.size() - 1;
        check(pp.jb.back() == H[l + 1].nc && pp.sb.size() == nb + 1, "pair partition blocks");
        for (uint32_t b = 0; b < nb; ++b) {
          const uint32_t m0 = H[l + 1].r_row[pp.jb[b]], m1 = H[l + 1].r_row[pp.jb[b + 1]];
          const uint32_t s0 = pp.sb[b], s1 = pp.sb[b + 1];
          check(s1 - s0 <= cap && pp.fo[s1] - pp.fo[s0] <= cap && m1 - m0 <= s1 - s0, "pair block capacity");
          std::vector<int> in_s(nm, -1);
          for (uint32_t q = s0; q < s1; ++q) {
            check(in_s[pp.s[q]] < 0, "pair S row twice");
            in_s[pp.s[q]] = (int)(q - s0);
            const uint32_t g = pp.s[q];
            check(pp.fo[q + 1] - pp.fo[q] == H[l].r_row[g + 1] - H[l].r_row[g], "pair member count");
            for (uint32_t e = 0; e < pp.fo[q + 1] - pp.fo[q]; ++e)
              check(pp.f[pp.fo[q] + e] == H[l].r_col[H[l].r_row[g] + e], "pair members in R order");
          }
          for (uint32_t q = 0; q < m1 - m0; ++q) {
            const uint32_t g = pp.s[s0 + q];
            check(g == H[l + 1].r_col[m0 + q], "pair owned rows in R order");
            check(owner[g] < 0, "pair row owned twice");
            owner[g] = (int)b;
            for (uint32_t e = mrow[g]; e < mrow[g + 1]; ++e)
              check(in_s[mcol[e]] >= 0 && pp.lc[e] == (uint16_t)in_s[mcol[e]], "pair local column");
          }
          for (uint32_t q = m1 - m0; q < s1 - s0; ++q) {  // ring rows: columns of owned rows
            bool used = false;
            const uint32_t c = pp.s[s0 + q];
            for (uint32_t r = 0; r < m1 - m0 && !used; ++r) {
              const uint32_t g = pp.s[s0 + r];
              for (uint32_t e = mrow[g]; e < mrow[g + 1]; ++e) used = used || mcol[e] == c;
            }
            check(used, "pair ring row not a column of an owned row");
          }
        }
        for (uint32_t g = 0; g < nm; ++g) check(owner[g] >= 0, "pair row not owned");
      }
    // up-leg pair partitions (k_amg_prolong_smooth_pair): fine level l, coarse l + 1
    for (size_t l = 0; l + 1 < H.size(); ++l)
      for (uint32_t rows : {256u, 64u}) {
        const cfd2::HostCsr& Fm = H[l].A;
        const uint32_t nf = (uint32_t)Fm.rows, nc = H[l].nc;
        std::vector<uint32_t> frow(nf + 1, 0), fcol;
        for (uint32_t g = 0; g < nf; ++g) {
          for (uint32_t k = Fm.row[g]; k < Fm.row[g + 1]; ++k)
            if (Fm.col[k] != g) fcol.push_back(Fm.col[k]);
          frow[g + 1] = (uint32_t)fcol.size();
        }
        cfd2::UpPairPartition up;
        if (!cfd2::build_up_pair_partition(frow, fcol, H[l].agg, nc, rows, 1024, up)) continue;
        const uint32_t nb = (nf + rows - 1) / rows;
        check(up.tb.size() == nb + 1, "up pair blocks");
        for (uint32_t b = 0; b < nb; ++b) {
          const uint32_t t0 = up.tb[b], t1 = up.tb[b + 1];
          for (uint32_t q = t0 + 1; q < t1; ++q) check(up.t[q - 1] < up.t[q], "up pair T ascending");
          for (uint32_t f = b * rows; f < std::min(nf, (b + 1) * rows); ++f) {
            check(up.t[t0 + up.lto[f]] == H[l].agg[f], "up pair own aggregate");
            for (uint32_t e = frow[f]; e < frow[f + 1]; ++e)
              check(up.t[t0 + up.lt[e]] == H[l].agg[fcol[e]], "up pair column aggregate");
          }
        }
      }
    for (size_t l = 0; l < H.size(); ++l) {  // coarse rows follow their seeds: a partition in rank order
      check(H[l].part.size() == (size_t)R + 1 && H[l].part[0] == 0 && H[l].part[R] == H[l].A.rows, "level partition");
      for (int q = 0; q < R; ++q) check(H[l].part[q] <= H[l].part[q + 1], "level partition order");
    }
    std::printf("%s: %u cells, %d rank(s): nnz %llu, halo %llu, regular coupled rows %llu, %zu AMG levels: ok\n",
                name, n, R, (unsigned long long)nnz, (unsigned long long)sends, (unsigned long long)reg_rows,
                H.size());
  }
}

}  // namespace

int main() {
  try {
    cfd2::Geometry step{cfd2::kBackwardsStep, {2.0, 0.5, 1.0, 0.5}};
    cfd2::Mesh a = cfd2::generate_cut_cell_mesh(step, 0.05, 0.05, 1.2, 2.0, 1.0);
    a.smooth(step, 0.3, 10);
    cfd2::Geometry chan{cfd2::kChannelWithObstacle, {3.0, 1.0, 1.0, 0.5, 0.2}};
    cfd2::Mesh b = cfd2::generate_voronoi_mesh(chan, 0.04, 0.12, 1.2, 3.0, 1.0, 21);
    cfd2::Mesh c = cfd2::generate_delaunay_mesh(chan, 0.04, 0.12, 1.2, 3.0, 1.0, 22);
    run("cut-cell step", a);
    run("voronoi channel", b);
    run("delaunay channel", c);
  } catch (const std::exception& e) {
    std::fprintf(stderr, "FAILED: %s\n", e.what());
    return 1;
  }
  return 0;
}
