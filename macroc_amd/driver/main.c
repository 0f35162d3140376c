/*
 * macroc_amd — C host driver of the MI355X MacroC Newton inner loop.
 *
 * Mirrors the reference driver src/main.c:25-125: same flags (mcx_parse_args accepts the
 * options-DB names of src/init.c:66-83, -da_* and -ksp_*), same time loop and Newton loop
 * (:49-82), same log lines ("|RES| = ", "KSP : |Ax - b|/|Ax| = ... Its = ..."), the history
 * commit of :83, the per-time-step post-processing of :86-97 (non-linear GP count, reaction
 * force, f_trial_max; info.dat row; gauss_evolution.dat row of src/util.c:77-84) and the final
 * "Elapsed time".
 *
 * Builds (Makefile):
 *   driver         single rank (one GPU)
 *   driver-mpi     -DMCX_WITH_MPI with mpicc: one MPI rank per GPU like `mpirun -np N macroc`
 *                  (tests/CMakeLists.txt:21-32); rank 0 creates the RCCL id and MPI_Bcast's it,
 *                  the GPU is the node-local rank, -da_processors_x/y/z pick the rank grid.
 *   -DMCX_WITH_MICROPP: links a MicroPP C wrapper (micropp_C_*) and, with -mat_law external,
 *                  creates it as src/init.c:196-216 does and registers it as the Gauss-point
 *                  callback (mcx_set_micropp).
 * -plan_only (driver option, no GPU touched): print every rank's DMDA corners, DOF offset and
 * forward-halo plan (mcx_plan / mcx_plan_halo) and exit.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "macroc_amd.h"

#ifdef MCX_WITH_MPI
#include <mpi.h>
#endif

#ifdef MCX_WITH_MICROPP
/* micropp_c_wrapper.h call shapes (src/init.c:196-216, src/assembly.c:59,92,149, src/main.c:62,83,
   src/util.c:71,96) */
void micropp_C_material_set(int id, double E, double nu, double Sy, double Ka, int type);
void micropp_C_material_print(int id);
void micropp_C_create3(int ngp, int size[3], int micro_type, double params[4]);
void micropp_C_print_info(void);
void micropp_C_set_strain3(int gp, double strain[6]);
void micropp_C_homogenize(void);
void micropp_C_get_stress3(int gp, double stress[6]);
void micropp_C_get_ctan3(int gp, double ctan[36]);
void micropp_C_update_vars(void);
int micropp_C_get_non_linear_gps(void);
double micropp_C_get_f_trial_max(void);
#endif

static int g_rank = 0, g_size = 1;

static double wtime(void) {
#ifdef MCX_WITH_MPI
  return MPI_Wtime();
#else
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + 1e-9 * t.tv_nsec;
#endif
}

/* PetscPrintf(PETSC_COMM_WORLD, ...): rank 0 prints */
#define PRINTF(...)                  \
  do {                               \
    if (!g_rank) printf(__VA_ARGS__); \
  } while (0)

#define CHK(x)                                                                            \
  do {                                                                                    \
    int e_ = (x);                                                                         \
    if (e_) {                                                                             \
      fprintf(stderr, "[%d] %s failed (%d): %s\n", g_rank, #x, e_, mcx_last_error());      \
      return e_;                                                                          \
    }                                                                                     \
  } while (0)

/* -plan_only: the decomposition and halo plan of this rank (or of every rank without MPI) */
static int plan_only(const mcx_opts* o, int nranks) {
  int r0 = g_size > 1 ? g_rank : 0, r1 = g_size > 1 ? g_rank + 1 : nranks;
  for (int r = r0; r < r1; r++) {
    mcx_info in;
    CHK(mcx_plan(o, r, nranks, &in));
    int nnbr = 0, nbr[26];
    int64_t sc[26], rc[26], ns = 0, nr = 0;
    CHK(mcx_plan_halo(o, r, nranks, &nnbr, nbr, sc, rc, NULL, NULL, &ns, &nr));
    /* one write per line (ranks share stdout; a pipe write of < 4 KiB is not interleaved) */
    char line[2048];
    int len = snprintf(line, sizeof(line),
                       "PLAN rank %d of %d grid %d %d %d corners %ld %ld %ld %ld %ld %ld dof_offset %ld ndofs %ld nnz %ld"
                       " nelem %ld halo %d",
                       r, nranks, in.px, in.py, in.pz, (long)in.xs, (long)in.ys, (long)in.zs, (long)in.nx, (long)in.ny,
                       (long)in.nz, (long)in.dof_offset, (long)in.ndofs_local, (long)in.nnz_local, (long)in.nelem_local,
                       nnbr);
    for (int q = 0; q < nnbr; q++)
      len += snprintf(line + len, sizeof(line) - len, " %d:%ld:%ld", nbr[q], (long)sc[q], (long)rc[q]);
    snprintf(line + len, sizeof(line) - len, "\n");
    fputs(line, stdout);
    fflush(stdout);
  }
  return 0;
}

static int run(int argc, char** argv) {
  mcx_opts o;
  mcx_default_opts(&o);
  /* driver-only options are taken out before the options-DB parse */
  int plan = 0, nargs = 0;
  const char** args = malloc(sizeof(char*) * (argc + 1));
  for (int a = 1; a < argc; a++) {
    if (!strcmp(argv[a], "-plan_only")) plan = 1;
    else args[nargs++] = argv[a];
  }
  int rc = mcx_parse_args(&o, nargs, args);
  free(args);
  CHK(rc);
  int want = (o.px > 0 ? o.px : 1) * (o.py > 0 ? o.py : 1) * (o.pz > 0 ? o.pz : 1);
  if (plan) return plan_only(&o, g_size > 1 ? g_size : want);
  if (g_size == 1 && want > 1) {
    fprintf(stderr, "-da_processors_x/y/z ask for %d ranks: run the MPI build (make driver-mpi) under mpirun\n", want);
    return 2;
  }
  unsigned char id[MCX_COMM_ID_BYTES];
  memset(id, 0, sizeof(id));
#ifdef MCX_WITH_MPI
  if (g_size > 1) {
    if (!g_rank) CHK(mcx_comm_unique_id(id));
    MPI_Bcast(id, MCX_COMM_ID_BYTES, MPI_BYTE, 0, MPI_COMM_WORLD);
    if (o.device < 0) { /* the node-local rank picks the GPU */
      MPI_Comm node;
      int local = 0;
      MPI_Comm_split_type(MPI_COMM_WORLD, MPI_COMM_TYPE_SHARED, g_rank, MPI_INFO_NULL, &node);
      MPI_Comm_rank(node, &local);
      MPI_Comm_free(&node);
      o.device = local;
    }
  }
#endif
  FILE* file_out = g_rank ? NULL : fopen("info.dat", "w");
  FILE* file_gps = g_rank ? NULL : fopen("gauss_evolution.dat", "w"); /* src/init.c:135 */
  PRINTF("\nMacroC : A HPC for FE2 Multi-scale Simulations\n\n");
  void* ctx = NULL;
  CHK(mcx_init(&o, g_rank, g_size, g_size > 1 ? id : NULL, &ctx));
  mcx_info in;
  CHK(mcx_get_info(ctx, &in));
#ifdef MCX_WITH_MICROPP
  if (o.mat_law == MCX_LAW_EXTERNAL) { /* src/init.c:196-216 */
    micropp_C_material_set(0, o.micro_mat_1[0], o.micro_mat_1[1], o.micro_mat_1[2], o.micro_mat_1[3], 1);
    micropp_C_material_set(1, o.micro_mat_2[0], o.micro_mat_2[1], o.micro_mat_2[2], o.micro_mat_2[3], 1);
    PRINTF("Material Values : \n");
    if (!g_rank) {
      micropp_C_material_print(0);
      micropp_C_material_print(1);
    }
    int size[3] = {o.micro_n, o.micro_n, o.micro_n};
    double params[4] = {1., 1., 1., .5};
    micropp_C_create3((int)(in.nelem_ext * 8), size, o.micro_type, params);
    if (!g_rank) micropp_C_print_info();
    mcx_micropp_api api = {micropp_C_set_strain3, micropp_C_homogenize, micropp_C_get_stress3, micropp_C_get_ctan3,
                           micropp_C_update_vars, micropp_C_get_non_linear_gps, micropp_C_get_f_trial_max};
    CHK(mcx_set_micropp(ctx, &api));
  }
#else
  if (o.mat_law == MCX_LAW_EXTERNAL) {
    fprintf(stderr, "-mat_law external: this driver was built without a MicroPP (-DMCX_WITH_MICROPP)\n");
    return 2;
  }
#endif
  PRINTF("Boundary Condition : %s\n", o.bc_type == MCX_BC_BENDING ? "BC_BENDING" : "BC_CIRCLE");
  PRINTF("Number of CPUs     : %d\n", in.nranks);
  PRINTF("Number of Elements : %ld\n", (long)((in.NX - 1) * (in.NY - 1) * (in.NZ - 1)));
  PRINTF("Number of Nodes    : %ld\n", (long)(in.NX * in.NY * in.NZ));
  PRINTF("Number of DOFs     : %ld\n\n", (long)(in.NX * in.NY * in.NZ * 3));
  PRINTF("NP_X : %d\tNP_Y : %d\tNP_Z : %d\n", in.px, in.py, in.pz);
  PRINTF("NX   : %ld\tNY   : %ld\tNZ   : %ld\n\n", (long)in.NX, (long)in.NY, (long)in.NZ);
  PRINTF("KSP Info: type = cg\trtol = %e\tabstol = %e\tdtol = %e\tmaxits = %d\n\n", o.ksp_rtol, o.ksp_abstol,
         o.ksp_dtol, o.ksp_max_it);
  PRINTF("------------------------------------------------------------\n"
         "STARTING CALCULATION...\n"
         "------------------------------------------------------------\n");
  double t1 = wtime();
  for (int time_s = 0; time_s < o.ts; ++time_s) {
    PRINTF("\n\nTime Step = %d\n", time_s);
    double U = mcx_get_displacement(ctx, time_s);
    CHK(mcx_apply_bc_u(ctx, U));
    int newton_it = 0;
    double norm = 0., norm_0 = 0.;
    while (newton_it < o.newton_max_its) {
      PRINTF("\nNewton Iteration = %d\n", newton_it);
      PRINTF("Homogenizing MicroPP\n");
      CHK(mcx_set_strains(ctx));
      CHK(mcx_homogenize(ctx));
      PRINTF("Assemblying RHS\n");
      CHK(mcx_assembly_res(ctx, &norm));
      PRINTF("|RES| = %e\n", norm);
      if (newton_it == 0) norm_0 = norm;
      if (norm < o.newton_min_tol || norm < norm_0 * o.newton_rel_tol) break;
      CHK(mcx_assembly_jac(ctx));
      int its = 0, reason = 0;
      double rnorm = 0.;
      CHK(mcx_solve(ctx, &its, &rnorm, &reason));
      PRINTF("KSP : |Ax - b|/|Ax| = %e\tIts = %d\n", rnorm, its);
      CHK(mcx_update_u(ctx));
      newton_it++;
    }
    CHK(mcx_update_vars(ctx)); /* micropp_C_update_vars(), src/main.c:83 */
    int64_t nl_local = 0, nl = 0;
    double f_trial_max = 0., force = 0.;
    CHK(mcx_reduce_nonlinear(ctx, &nl_local, &nl, &f_trial_max));
    /* gauss_evolution.dat row (src/util.c:77-84): time step, then every rank's count */
    long* counts = malloc(sizeof(long) * g_size);
    counts[0] = (long)nl_local;
#ifdef MCX_WITH_MPI
    long mine = (long)nl_local;
    MPI_Gather(&mine, 1, MPI_LONG, counts, 1, MPI_LONG, 0, MPI_COMM_WORLD);
#endif
    if (file_gps) {
      fprintf(file_gps, "%d\t", time_s);
      for (int r = 0; r < g_size; r++) fprintf(file_gps, "%ld\t", counts[r]);
      fprintf(file_gps, "\n");
    }
    free(counts);
    PRINTF("Non-Linear Gauss points : %ld\n", (long)nl);
    CHK(mcx_calc_force(ctx, &force));
    PRINTF("F_trial_max             : %e\n", f_trial_max);
    if (file_out)
      fprintf(file_out, "%d\t%e\t%e\t%e\t%e\t%d\n", time_s, time_s * o.dt, U, force, f_trial_max, (int)nl);
    if (o.vtu_freq > 0 && time_s % o.vtu_freq == 0) { /* src/main.c:100-108 */
      char file_prefix[256];
      snprintf(file_prefix, sizeof(file_prefix), "solution_%d", time_s);
      CHK(mcx_write_vtu(ctx, file_prefix));
    }
  }
  CHK(mcx_synchronize(ctx));
  double t2 = wtime();
  PRINTF("\n\n"
         "------------------------------------------------------------\n"
         "FINISHING CALCULATION...\n"
         "------------------------------------------------------------\n");
  PRINTF("Elapsed time : %f\n", t2 - t1);
  if (file_out) fclose(file_out);
  if (file_gps) fclose(file_gps);
  return mcx_finalize(ctx);
}

int main(int argc, char** argv) {
#ifdef MCX_WITH_MPI
  MPI_Init(&argc, &argv);
  MPI_Comm_rank(MPI_COMM_WORLD, &g_rank);
  MPI_Comm_size(MPI_COMM_WORLD, &g_size);
#endif
  int rc = run(argc, argv);
#ifdef MCX_WITH_MPI
  if (rc) MPI_Abort(MPI_COMM_WORLD, rc);
  MPI_Finalize();
#endif
  return rc;
}
