"""Redundant-work ratios of a two-level fused AMG kernel.

Host only.  Builds the pattern hierarchy of the fixed-schedule bench meshes
(greedy index-order aggregation without strength test, amg.rs:84-116, and the
Galerkin pattern P^T A P, amg.rs:187-235) and, for each adjacent level pair
(l, l+1) and row-block size B, the extra rows a block must compute to do both
levels' work in one launch:

- down-leg (k_amg_resrestrict of l, then of l+1): a block owning a range of
  level-(l+2) aggregates with level-(l+1) members M needs b_{l+1} (and the
  zero-x pre-smoothed x_{l+1}) on M and its 1-ring N_{l+1}(M), i.e. the
  level-l residuals of every fine member of M u N(M):
  ratio_down = |F(M u N(M))| / |F(M)| (fine rows computed / fine rows owned);
- up-leg (fused prolongation + post-smoother of l+1, then of l): a block of
  level-l rows R needs the final x_{l+1} on agg(R u N_l(R)):
  ratio_up = |agg(R u N_l(R))| / |agg(R)| (level-(l+1) rows computed / owned).

Usage: python tools/amg_fusion_ratio.py c1 [c2]   (C1 ~10 s of mesh, C2 ~2 min)
"""
import os
import sys
import time

import numpy as np
import scipy.sparse as sp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cfd-demo2_amd"))

H = {"c0": None, "c1": 0.001723, "c2": 0.0005449}


def scalar_pattern(mesh):
    a = mesh.arrays()
    n = mesh.num_cells()
    own, nb, bd = a["face_owner"].astype(np.int64), a["face_neighbor"].astype(np.int64), a["face_boundary"]
    inner = nb < n  # interior faces (boundary faces carry no neighbour cell)
    inner &= nb != own
    r = np.concatenate([np.arange(n), own[inner], nb[inner]])
    c = np.concatenate([np.arange(n), nb[inner], own[inner]])
    A = sp.csr_matrix((np.ones(len(r), np.int8), (r, c)), shape=(n, n))
    A.sum_duplicates()
    A.sort_indices()
    return A


def aggregate(A):
    """amg.rs:84-116: greedy, index order (row entries in column order)."""
    n = A.shape[0]
    ip, ix = A.indptr, A.indices
    agg = np.full(n, -1, np.int64)
    k = 0
    for i in range(n):
        if agg[i] >= 0:
            continue
        agg[i] = k
        for j in ix[ip[i]:ip[i + 1]]:
            if agg[j] < 0:
                agg[j] = k
        k += 1
    return agg, k


def hierarchy(A0, min_rows=64):
    levels = [A0]
    aggs = []
    while levels[-1].shape[0] > min_rows and len(levels) < 12:
        A = levels[-1]
        agg, nc = aggregate(A)
        if nc == A.shape[0]:
            break
        P = sp.csr_matrix((np.ones(A.shape[0], np.int8), (np.arange(A.shape[0]), agg)), shape=(A.shape[0], nc))
        Ac = (P.T @ A @ P).tocsr()
        Ac.data[:] = 1
        Ac.sort_indices()
        aggs.append(agg)
        levels.append(Ac)
    return levels, aggs


def ring(A, rows):
    """rows u their neighbours in A (1-ring), as unique indices."""
    return np.unique(np.concatenate([rows, A[rows].indices]))


def ratios(levels, aggs, l, B):
    """Mean redundant-work ratios over contiguous blocks for pair (l, l+1)."""
    A0, A1 = levels[l], levels[l + 1]
    n0, n1 = A0.shape[0], A1.shape[0]
    out = {}
    # fine rows per level-(l+1) row
    cnt0 = np.bincount(aggs[l], minlength=n1)
    if l + 2 < len(levels):
        a1 = aggs[l + 1]  # level-(l+1) row -> level-(l+2) aggregate
        n2 = levels[l + 2].shape[0]
        # R of l+1 in aggregate order: block = consecutive l+2 aggregates with ~B level-(l+1) members
        order = np.argsort(a1, kind="stable")
        tot_c = tot_o = 0
        for s in range(0, n1, B):
            sel = order[s:s + B]
            tot_c += cnt0[ring(A1, sel)].sum()
            tot_o += cnt0[sel].sum()
        out["down"] = tot_c / tot_o
    # up-leg: blocks of B consecutive level-l rows
    tot_c = tot_o = 0
    for s in range(0, n0, B):
        R = np.arange(s, min(s + B, n0))
        tot_c += len(np.unique(aggs[l][ring(A0, R)]))
        tot_o += len(np.unique(aggs[l][R]))
    out["up"] = tot_c / tot_o
    return out


def main():
    from cfd2_amd.mesh import bench_channel
    for cfg in sys.argv[1:] or ["c1"]:
        t = time.time()
        mesh = bench_channel(H[cfg], 100)
        A0 = scalar_pattern(mesh)
        levels, aggs = hierarchy(A0)
        print(f"{cfg}: {A0.shape[0]} cells, levels {[L.shape[0] for L in levels]} ({time.time() - t:.0f} s)")
        print(f"{'pair':>10s} {'rows l':>9s} {'rows l+1':>9s} {'B':>6s} {'down':>6s} {'up':>6s}")
        for l in range(len(levels) - 1):
            if levels[l].shape[0] > 600_000 or levels[l].shape[0] < 2_000:
                continue  # the pairs a fused kernel could take (below the big levels, above the LDS tail)
            for B in (256, 1024, 4096):
                r = ratios(levels, aggs, l, B)
                print(f"{l:>4d},{l + 1:<5d} {levels[l].shape[0]:9d} {levels[l + 1].shape[0]:9d} {B:6d} "
                      f"{r.get('down', float('nan')):6.2f} {r['up']:6.2f}")


if __name__ == "__main__":
    main()
