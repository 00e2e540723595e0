/* C99 consumer of include/cfd2_amd.h: the header is plain C and the library
 * links and runs from C (what a cgo / bindgen binding sees).  Built by
 * tests/test_capi_c.py (compile + link on CPU; run on a GPU box). */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include "../../include/cfd2_amd.h"

#define CHECK(call)                                                          \
  do {                                                                       \
    cfd_status st_ = (call);                                                 \
    if (st_ != CFD_OK) {                                                     \
      fprintf(stderr, "%s failed (%d): %s\n", #call, (int)st_, cfd_last_error()); \
      return 1;                                                              \
    }                                                                        \
  } while (0)

int main(int argc, char** argv) {
  const char* state_path = argc > 1 ? argv[1] : "abi_smoke.state";
  cfd_geometry geo = {1, {3.0, 1.0, 1.0, 0.5, 0.2, 0.0, 0.0, 0.0}}; /* ChannelWithObstacle */
  cfd_mesh* mesh = NULL;
  CHECK(cfd_mesh_generate_cut_cell(&geo, 0.05, 0.05, 1.2, 3.0, 1.0, &mesh));
  int32_t iters = 0;
  CHECK(cfd_mesh_smooth(mesh, &geo, 0.3, 50, &iters));
  cfd_mesh_view view;
  CHECK(cfd_mesh_get_view(mesh, &view));
  cfd_config cfg;
  cfd_config_default(&cfg);
  cfg.fixed_outer = 2;
  cfg.fixed_inner = 8;
  cfd_solver* s = NULL;
  CHECK(cfd_solver_create(&view, &cfg, 0, &s));
  CHECK(cfd_set_dt(s, 0.01f));
  CHECK(cfd_set_viscosity(s, 0.01f));
  CHECK(cfd_set_precond_type(s, 1));
  CHECK(cfd_initialize_history(s));
  for (int k = 0; k < 3; ++k) CHECK(cfd_step(s));
  const uint32_t n = cfd_num_cells(s);
  double* uv = (double*)malloc(2 * (size_t)n * sizeof(double));
  CHECK(cfd_get_u(s, uv));
  double umax = 0.0;
  for (uint32_t i = 0; i < 2 * n; ++i) {
    if (!isfinite(uv[i])) {
      fprintf(stderr, "non-finite u\n");
      return 1;
    }
    if (fabs(uv[i]) > umax) umax = fabs(uv[i]);
  }
  cfd_step_info info;
  CHECK(cfd_get_step_info(s, &info));
  /* LinearSolverStats.time (coupled_solver_fgmres.rs:2446): the last solve's wall time */
  if (!(info.stats_p.time_s > 0.0) || !(info.stats_p.time_s < 60.0)) {
    fprintf(stderr, "stats_p.time_s not filled: %g\n", info.stats_p.time_s);
    return 1;
  }
  /* the public stop fields are caller-writable (structs.rs:244-247; the GUI
   * clears should_stop before it resumes, src/ui/app.rs:852-857) */
  CHECK(cfd_set_stop_state(s, 1, 0, 7));
  CHECK(cfd_get_step_info(s, &info));
  if (info.should_stop != 1 || info.degenerate_count != 0 || info.steady_state_count != 7) {
    fprintf(stderr, "cfd_set_stop_state not applied\n");
    return 1;
  }
  CHECK(cfd_set_stop_state(s, 0, 0, 0));
  /* n_outer_correctors is a public field too (structs.rs:238): 12 Picard
   * iterations at most from the next step on; a negative count is refused */
  CHECK(cfd_set_n_outer_correctors(s, 12));
  if (cfd_set_n_outer_correctors(s, -1) != CFD_ERR_INVALID) {
    fprintf(stderr, "negative n_outer_correctors accepted\n");
    return 1;
  }
  CHECK(cfd_step(s));
  CHECK(cfd_get_step_info(s, &info));
  if (info.outer_iterations > 12) {
    fprintf(stderr, "n_outer_correctors = 12 not applied: %u outer iterations\n", info.outer_iterations);
    return 1;
  }
  if (info.should_stop != 0) { /* the flow still evolves: no stop */
    fprintf(stderr, "should_stop set again on an evolving flow\n");
    return 1;
  }
  CHECK(cfd_state_save(s, state_path));
  /* a bad call reports a status and a message instead of aborting */
  if (cfd_set_u(NULL, uv) != CFD_ERR_INVALID || cfd_last_error()[0] == '\0') {
    fprintf(stderr, "null handle not rejected\n");
    return 1;
  }
  printf("abi_smoke: %u cells, max|u| = %.6f, outer iterations %u, linear %u, last solve %.3f ms: ok\n", n, umax,
         info.outer_iterations, info.total_linear_iterations, 1e3 * info.stats_p.time_s);
  free(uv);
  cfd_solver_destroy(s);
  cfd_mesh_destroy(mesh);
  return 0;
}
