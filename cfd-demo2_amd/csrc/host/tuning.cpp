// Environment knobs (tuning.hpp): the table, the one getenv of the library,
// and the warning for removed knobs.
#include "tuning.hpp"

#include <cstdio>
#include <cstdlib>
#include <mutex>

namespace cfd2 {

namespace {

struct KnobInfo {
  Knob k;
  const char* name;
  const char* meaning;  // default, then what it selects (same bits either way)
};

// Keep in the order of the enum; INTEGRATION.md lists the same table.
constexpr KnobInfo kKnobs[] = {
    {Knob::AmgReplicateRows, "CFD_AMG_REPLICATE_ROWS",
     "2^20: distributed AMG levels of at most this many rows are replicated on every rank"},
    {Knob::AmgSetup, "CFD_AMG_SETUP",
     "device: AMG setup on the GPU (amg_rebuild_interval re-setups refresh the values over the kept "
     "structure); host: the host setup; rebuild: device setup, every re-setup a full one (same hierarchy)"},
    {Knob::OverlapMinRows, "CFD_OVERLAP_MIN_ROWS",
     "2^20: halo'd launches of at least this many rows split interior / boundary around the exchange"},
    {Knob::Nt, "CFD_NT", "47: nontemporal-load mask per kernel (Solver::nt_mask)"},
    {Knob::AmgFull, "CFD_AMG_FULL",
     "unset: unconditional slot loads on level 0, regular and <= 2^19-row levels; 1 every level; 0 none"},
    {Knob::AmgTailRows, "CFD_AMG_TAIL_ROWS", "4096: levels of at most this many rows run in the one-workgroup tail"},
    {Knob::AmgTail, "CFD_AMG_TAIL",
     "blob2: tail form -- blobK LDS image of matrices + vectors, starting up to K levels lower to fit; "
     "lds: vectors in LDS only; global: no LDS"},
    {Knob::AmgFusedProlongRows, "CFD_AMG_FUSED_PROLONG_ROWS",
     "2^20: post-smoother reads x + P x_c on single-GPU / replicated levels of at most this many rows; 0 off"},
    {Knob::AmgFusedRrRows, "CFD_AMG_FUSED_RR_ROWS",
     "2^18: residual + restriction in one launch on single-GPU / replicated levels up to this size; 0 off"},
    {Knob::AmgWideLimit, "CFD_AMG_WIDE_LIMIT", "255: rows with more off-diagonals use the 16-bit-length layout"},
    {Knob::SmallMeshForms, "CFD_SMALL_MESH_FORMS",
     "1: small-mesh kernel forms (CGS latency forms <= 2^17 cells, in-kernel CGS reduction <= 256 units, "
     "single-launch Jacobi relaxation <= 8191 cells); 0: the large-mesh forms everywhere"},
    {Knob::AmgFusedPair, "CFD_AMG_FUSED_PAIR",
     "1: two adjacent k_amg_resrestrict levels of the down-leg in one launch (k_amg_resrestrict_pair) where "
     "the ring's redundant rows stay within 50 %; 2: every candidate pair; 0 off"},
};
static_assert(sizeof(kKnobs) / sizeof(kKnobs[0]) == (size_t)Knob::Count, "one table entry per knob");

// knobs of settled experiments (removed in round 6; outcomes in DESIGN.md /
// profiles/*/ab_log.md): a run that still sets one is told so
constexpr const char* kRemoved[] = {
    "CFD_RELAX4",         "CFD_COUPLED_REG",      "CFD_TYPED_ELL",           "CFD_AMG_FUSE_PRESMOOTH",
    "CFD_CGS_KEEP_MB",    "CFD_CGS_UPDATE_NT",    "CFD_AMG_HALO_OVERLAP",    "CFD_HALO_PACK",
    "CFD_GRAPH",          "CFD_PROF_STRIDE",      "CFD_CHECK_SYNC",          "CFD_AMG_SETUP_TIMING",
    "CFD_AMG_TAIL_LDS",   "CFD_AMG_TAIL_BLOB",    "CFD_AMG_BLOB_SHIFT",      "CFD_AMG_FUSED_PROLONG",
    "CFD_AMG_FUSED_RR",   "CFD_CGS_LAT",          "CFD_CGS_FUSE_REDUCE",     "CFD_RELAX_FUSED",
    "CFD_AMG_REFRESH",
};

void warn_removed_once() {
  static std::once_flag once;
  std::call_once(once, [] {
    for (const char* n : kRemoved)
      if (std::getenv(n))
        std::fprintf(stderr,
                     "cfd2_amd: %s is no longer read (removed in round 6, see INTEGRATION.md \"Environment knobs\")\n",
                     n);
  });
}

}  // namespace

const char* knob(Knob k) {
  warn_removed_once();
  return std::getenv(kKnobs[(int)k].name);
}

uint64_t knob_u64(Knob k, uint64_t def) {
  const char* v = knob(k);
  if (!v) return def;
  const bool hex = v[0] == '0' && (v[1] == 'x' || v[1] == 'X');
  return std::strtoull(v, nullptr, hex ? 16 : 10);
}

bool knob_on(Knob k, bool def) {
  const char* v = knob(k);
  return v ? v[0] != '0' : def;
}

}  // namespace cfd2
