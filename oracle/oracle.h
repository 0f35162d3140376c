/*
 * oracle.h — CPU restatement of MacroC's Newton inner loop (TEST INFRASTRUCTURE ONLY).
 *
 * This is the parity checker for the MI355X path in macroc_amd/.  It is NOT part of
 * the product: only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load it, and only as the checker / the timed CPU baseline, never as a fallback.
 *
 * What it restates (all paths relative to the reference checkout, GG1991/macroc):
 *   calc_B .................... src/assembly.c:195-254, xg include/macroc.h:61-69
 *   set_strains ............... src/assembly.c:25-66
 *   assembly_jac .............. src/assembly.c:69-117 (+ apply_bc_on_jac src/bcs.c:341-347)
 *   assembly_res .............. src/assembly.c:120-176 (+ apply_bc_on_res src/bcs.c:350-362)
 *   BC index sets / apply ..... src/bcs.c:29-146, 154-338
 *   get_displacement .......... src/bcs.c:52-58 (intended `return`, see Appendix A.3)
 *   Newton / time loop ........ src/main.c:49-109
 *   wg, dx, KSP defaults ...... src/init.c:137-164, include/macroc.h:32-52
 * plus PETSc semantics the reference relies on ([ext], PETSc not vendored, version
 * unpinned — restated from PETSc's public source):
 *   DMDA 3-D partition (PETSC_DECIDE heuristic, ownership split, rank-contiguous
 *   global ordering), DMDAGetElements Q1 connectivity, DMDA box-stencil AIJ pattern,
 *   MatZeroRowsColumns, MatMult_SeqAIJ_Inode/MPIAIJ row-sum order, PCJacobi, KSPSolve_CG with
 *   KSP_NORM_PRECONDITIONED and KSPConvergedDefault.
 * MicroPP (the Gauss-point callback, not vendored) is replaced by an isotropic
 * linear-elastic material (both reference materials are E=1e7, nu=0.25, src/init.c:31-32).
 *
 * Parity pinning: the DMDA ordering is pinned by the only known answer the reference
 * holds (tests/test_dm_1.c:5-19); every numeric result is cross-checked against an
 * independent numpy/scipy restatement (tests/golden/make_golden.py).  No reference test
 * pins a numeric result of the hot path.
 *
 * The oracle works on the GLOBAL problem in one process and emulates the MPI rank grid
 * only where it changes integers or summation order (DOF numbering, element ownership,
 * Dirichlet lists, off-rank stash order, per-rank partial dot products).
 */
#ifndef MACROC_ORACLE_H
#define MACROC_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { ORC_BC_BENDING = 0, ORC_BC_CIRCLE = 1 };

/* KSPConvergedReason values (PETSc include/petscksp.h) */
enum {
  ORC_KSP_CONVERGED_RTOL = 2,
  ORC_KSP_CONVERGED_ATOL = 3,
  ORC_KSP_CONVERGED_ITERATING = 0,
  ORC_KSP_DIVERGED_ITS = -3,
  ORC_KSP_DIVERGED_DTOL = -4,
  ORC_KSP_DIVERGED_INDEFINITE_PC = -8,
  ORC_KSP_DIVERGED_NANORINF = -9,
  ORC_KSP_DIVERGED_INDEFINITE_MAT = -10
};

typedef struct {
  int64_t NX, NY, NZ;      /* -da_grid_x/y/z (src/init.c:179-181, DMSetFromOptions) */
  int m, n, p;             /* -da_processors_x/y/z, 0 = PETSC_DECIDE */
  int nranks;              /* MPI size emulated */
  double lx, ly, lz;       /* -lx -ly -lz */
  double dt, final_time;   /* -dt, FINAL_TIME */
  int ts;                  /* -ts */
  int bc_type;             /* -bc_type */
  double rad;              /* src/init.c:141 */
  int newton_max_its;      /* -newton_max_its */
  double newton_min_tol;   /* -newton_min_tol */
  double newton_rel_tol;   /* -newton_rel_tol */
  double rtol, abstol, dtol; /* -ksp_rtol ... (src/init.c:147-156) */
  int maxits;              /* -ksp_max_it */
  double E, nu;            /* material (src/init.c:31-32) */
  double Sy, Ka;           /* yield stress, hardening modulus (micro_mat_1[2..3]) */
  int law;                 /* 0 = isotropic elastic, 1 = J2 plasticity (MicroPP material type 1) */
} orc_opts;

typedef struct orc_problem orc_problem;

/* defaults of src/init.c:47-64 + include/macroc.h:36-52 */
void orc_default_opts(orc_opts* o);

/* PETSc da3.c PETSC_DECIDE partition; returns 0 on success */
int orc_dmda_decide(int64_t M, int64_t N, int64_t P, int size, int* m, int* n, int* p);

orc_problem* orc_create(const orc_opts* o);   /* NULL on error (bad partition) */
void orc_destroy(orc_problem* P);

/* sizes */
int64_t orc_ndofs(const orc_problem* P);
int64_t orc_nnz(const orc_problem* P);
void orc_get_decomp(const orc_problem* P, int* mnp /*3*/);
/* corners of rank r: xs,ys,zs,nx,ny,nz (owned) and Xs,Ys,Zs,Nx,Ny,Nz (ghost) */
void orc_rank_corners(const orc_problem* P, int r, int64_t* c12);
int64_t orc_rank_nelem(const orc_problem* P, int r);
int64_t orc_rank_dof_offset(const orc_problem* P, int r);
double orc_wg(const orc_problem* P);

/* integer artefacts */
void orc_dof_map(const orc_problem* P, int64_t* natural_to_petsc); /* len ndofs */
void orc_rank_elements(const orc_problem* P, int r, int32_t* conn); /* nelem*8 ghosted-local ids */
/* Dirichlet list of rank r exactly as bc_init builds it (incl. -1 padding); returns nbcs */
int64_t orc_rank_dirichlet(const orc_problem* P, int r, int64_t* ix, int64_t cap);
/* sorted unique union of all ranks' non-negative Dirichlet DOFs; returns count */
int64_t orc_dirichlet_set(const orc_problem* P, int64_t* out, int64_t cap);
void orc_csr_pattern(const orc_problem* P, int64_t* rowptr, int32_t* colidx);
int orc_petsc_numbering(int64_t M, int64_t N, int64_t P, int size, int m, int n, int p, int64_t* out);

/* element kinematics */
void orc_calc_B(int gp, double B[6][24]);

/* state access (vectors in PETSc global ordering) */
double* orc_u(orc_problem* P);
double* orc_b(orc_problem* P);
double* orc_du(orc_problem* P);
double* orc_A_values(orc_problem* P);         /* CSR values, pattern of orc_csr_pattern */
double* orc_strain(orc_problem* P);           /* [ngp][6] rank-major, ie*8+gp */
double* orc_stress(orc_problem* P);
int64_t orc_ngp(const orc_problem* P);

/* hot-path steps (mirror src/main.c:53-79) */
double orc_get_displacement(const orc_problem* P, int time_s);
void orc_apply_bc_u(orc_problem* P, double U);
void orc_set_strains(orc_problem* P);
void orc_homogenize(orc_problem* P);
void orc_assembly_res(orc_problem* P);
double orc_norm2(const orc_problem* P, const double* v);
void orc_assembly_jac(orc_problem* P);
void orc_sbaij_mirror(orc_problem* P);
/* MatMult row-sum orders: the MATAIJ inode kernel (default) or MatMult_SeqAIJ's plain loop */
enum { ORC_SPMV_INODE = 0, ORC_SPMV_SEQAIJ = 1 };
void orc_spmv(const orc_problem* P, const double* x, double* y);  /* the problem's order */
void orc_spmv_order(const orc_problem* P, const double* x, double* y, int order);
/* KSPSolve(CG, Jacobi) of A du = b; hist (len maxits+1, may be NULL) = residual history */
int orc_solve(orc_problem* P, int* its, double* rnorm, int* reason, double* hist);
void orc_update_u(orc_problem* P);
/* micropp_C_update_vars (src/main.c:83): commit the Gauss-point history */
void orc_update_vars(orc_problem* P);
/* non-linear Gauss points of the last homogenize and max f_trial (src/util.c:69-102) */
int64_t orc_nonlinear_gps(const orc_problem* P, double* f_trial_max);
double* orc_ctan(orc_problem* P);  /* [ngp][36] */

/* full run of src/main.c:49-109; writes log lines to `log` (may be NULL).
   newton_out: per (time step, newton it) records: |RES|, ksp its, ksp rnorm (cap entries) */
int orc_run(orc_problem* P, const char* log_path, double* t_newton_solve_s);
int orc_run_files(orc_problem* P, const char* log_path, const char* info_path, const char* gauss_path,
                  double* t_newton_solve_s);
/* post-processing of src/main.c:86-97 */
double orc_calc_force(const orc_problem* P);                 /* src/forces.c:25-166 */
int orc_write_vtu(const orc_problem* P, const char* prefix); /* src/output.c:25-267 */
int64_t orc_rank_nonlinear_gps(const orc_problem* P, int r); /* src/util.c:69-87, one rank */
int orc_set_threads(int n);

#ifdef __cplusplus
}
#endif
#endif
