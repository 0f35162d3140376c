/*
 * macroc_amd — C host driver of the MI355X MacroC Newton inner loop (single rank).
 *
 * Mirrors the reference driver src/main.c:25-125: same flags (mcx_parse_args accepts the
 * options-DB names of src/init.c:66-83, -da_* and -ksp_*), same time loop and Newton loop
 * (:49-82), same log lines ("|RES| = ", "KSP : |Ax - b|/|Ax| = ... Its = ..."), the history
 * commit of :83, the per-time-step post-processing of :86-97 (non-linear GP count, reaction
 * force, f_trial_max; info.dat row; gauss_evolution.dat row of src/util.c:77-84) and the final
 * "Elapsed time".  Multi-GPU runs go through bench.py (one process per GPU over RCCL); this
 * driver is the single-rank drop-in.
 */
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

#include "macroc_amd.h"

static double wtime(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + 1e-9 * t.tv_nsec;
}

#define CHK(x)                                                          \
  do {                                                                  \
    int e_ = (x);                                                       \
    if (e_) {                                                           \
      fprintf(stderr, "%s failed (%d): %s\n", #x, e_, mcx_last_error()); \
      return e_;                                                        \
    }                                                                   \
  } while (0)

int main(int argc, char** argv) {
  mcx_opts o;
  mcx_default_opts(&o);
  CHK(mcx_parse_args(&o, argc - 1, (const char* const*)argv + 1));
  FILE* file_out = fopen("info.dat", "w");
  FILE* file_gps = fopen("gauss_evolution.dat", "w");  // src/init.c:135
  printf("\nMacroC : A HPC for FE2 Multi-scale Simulations\n\n");
  void* ctx = NULL;
  CHK(mcx_init(&o, 0, 1, NULL, &ctx));
  mcx_info in;
  CHK(mcx_get_info(ctx, &in));
  printf("Boundary Condition : %s\n", o.bc_type == MCX_BC_BENDING ? "BC_BENDING" : "BC_CIRCLE");
  printf("Number of CPUs     : %d\n", in.nranks);
  printf("Number of Elements : %ld\n", (long)((in.NX - 1) * (in.NY - 1) * (in.NZ - 1)));
  printf("Number of Nodes    : %ld\n", (long)(in.NX * in.NY * in.NZ));
  printf("Number of DOFs     : %ld\n\n", (long)(in.NX * in.NY * in.NZ * 3));
  printf("NP_X : %d\tNP_Y : %d\tNP_Z : %d\n", in.px, in.py, in.pz);
  printf("NX   : %ld\tNY   : %ld\tNZ   : %ld\n\n", (long)in.NX, (long)in.NY, (long)in.NZ);
  printf("KSP Info: type = cg\trtol = %e\tabstol = %e\tdtol = %e\tmaxits = %d\n\n", o.ksp_rtol, o.ksp_abstol,
         o.ksp_dtol, o.ksp_max_it);
  printf("------------------------------------------------------------\n"
         "STARTING CALCULATION...\n"
         "------------------------------------------------------------\n");
  double t1 = wtime();
  for (int time_s = 0; time_s < o.ts; ++time_s) {
    printf("\n\nTime Step = %d\n", time_s);
    double U = mcx_get_displacement(ctx, time_s);
    CHK(mcx_apply_bc_u(ctx, U));
    int newton_it = 0;
    double norm = 0., norm_0 = 0.;
    while (newton_it < o.newton_max_its) {
      printf("\nNewton Iteration = %d\n", newton_it);
      printf("Homogenizing MicroPP\n");
      CHK(mcx_set_strains(ctx));
      CHK(mcx_homogenize(ctx));
      printf("Assemblying RHS\n");
      CHK(mcx_assembly_res(ctx, &norm));
      printf("|RES| = %e\n", norm);
      if (newton_it == 0) norm_0 = norm;
      if (norm < o.newton_min_tol || norm < norm_0 * o.newton_rel_tol) break;
      CHK(mcx_assembly_jac(ctx));
      int its = 0, reason = 0;
      double rnorm = 0.;
      CHK(mcx_solve(ctx, &its, &rnorm, &reason));
      printf("KSP : |Ax - b|/|Ax| = %e\tIts = %d\n", rnorm, its);
      CHK(mcx_update_u(ctx));
      newton_it++;
    }
    CHK(mcx_update_vars(ctx));  // micropp_C_update_vars(), src/main.c:83
    int64_t nl_local = 0, nl = 0;
    double f_trial_max = 0., force = 0.;
    CHK(mcx_reduce_nonlinear(ctx, &nl_local, &nl, &f_trial_max));
    if (file_gps) fprintf(file_gps, "%d\t%ld\t\n", time_s, (long)nl_local);
    printf("Non-Linear Gauss points : %ld\n", (long)nl);
    CHK(mcx_calc_force(ctx, &force));
    printf("F_trial_max             : %e\n", f_trial_max);
    if (file_out)
      fprintf(file_out, "%d\t%e\t%e\t%e\t%e\t%d\n", time_s, time_s * o.dt, U, force, f_trial_max, (int)nl);
    if (o.vtu_freq > 0 && time_s % o.vtu_freq == 0) {  // src/main.c:100-108
      char file_prefix[256];
      snprintf(file_prefix, sizeof(file_prefix), "solution_%d", time_s);
      CHK(mcx_write_vtu(ctx, file_prefix));
    }
  }
  CHK(mcx_synchronize(ctx));
  double t2 = wtime();
  printf("\n\n"
         "------------------------------------------------------------\n"
         "FINISHING CALCULATION...\n"
         "------------------------------------------------------------\n");
  printf("Elapsed time : %f\n", t2 - t1);
  if (file_out) fclose(file_out);
  if (file_gps) fclose(file_gps);
  return mcx_finalize(ctx);
}
