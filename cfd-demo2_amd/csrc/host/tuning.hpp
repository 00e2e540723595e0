// Environment knobs of the library: the one place that reads CFD_* variables.
//
// Every knob is declared in kKnobs (tuning.cpp) with its default and meaning,
// listed in INTEGRATION.md ("Environment knobs") and exercised by a parity
// variant in the GPU tests (tests/test_gpu_parity.py
// test_amg_kernel_variants_parity and the tests named in the table).  None
// changes a result bit: they pick thresholds and kernel forms that give the
// same bits, so tests can reach on small meshes the paths large meshes take,
// and A/B runs can compare forms on one box.  Knobs of settled experiments are
// removed (round 6); setting one of those prints a one-time warning instead of
// being silently ignored.
#pragma once
#include <cstdint>

namespace cfd2 {

enum class Knob : int {
  AmgReplicateRows,    // CFD_AMG_REPLICATE_ROWS
  AmgSetup,            // CFD_AMG_SETUP
  OverlapMinRows,      // CFD_OVERLAP_MIN_ROWS
  Nt,                  // CFD_NT
  AmgFull,             // CFD_AMG_FULL
  AmgTailRows,         // CFD_AMG_TAIL_ROWS
  AmgTail,             // CFD_AMG_TAIL
  AmgFusedProlongRows, // CFD_AMG_FUSED_PROLONG_ROWS
  AmgFusedRrRows,      // CFD_AMG_FUSED_RR_ROWS
  AmgWideLimit,        // CFD_AMG_WIDE_LIMIT
  SmallMeshForms,      // CFD_SMALL_MESH_FORMS
  AmgFusedPair,        // CFD_AMG_FUSED_PAIR
  Count
};

// the variable's value, or nullptr when unset (first call: warns about any
// removed knob that is set)
const char* knob(Knob k);
// unsigned integer value, or `def` when unset
uint64_t knob_u64(Knob k, uint64_t def);
// false when the variable is set to a value starting with '0'
bool knob_on(Knob k, bool def = true);

}  // namespace cfd2
