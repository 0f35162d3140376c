/*
 * macroc_amd.h — C-ABI of the MI355X-native MacroC Newton inner loop.
 *
 * One context = one MPI-style rank = one GPU subdomain of the DMDA box decomposition.
 * Every entry point returns 0 on success and a non-zero code on failure, mirroring the
 * reference's PetscErrorCode convention (src/assembly.c:37-42 ... CHKERRQ); the message of
 * the last failure (per calling thread) is available from mcx_last_error().  No C++ exception
 * crosses this interface: an internal one (e.g. a failed host allocation) returns 90 with its
 * message.  Multi-rank host waits (CG polls, all-reduced norms, the in-process group's barrier
 * inside collective entries) are bounded: after the context's "comm_timeout" option (default
 * MCX_COMM_TIMEOUT seconds at mcx_init, else 300), or on an RCCL asynchronous
 * error, the communicator is aborted and the call returns 24 / 25 naming the rank and the
 * operation; later collectives of that context fail at once.  Host buffers are caller-owned;
 * the context owns all device memory.  A context is not thread-safe; different contexts
 * may be driven from different threads.  No torch / HIP types appear in this interface.
 *
 * Reference interface each entry replaces (paths relative to GG1991/macroc):
 *   mcx_default_opts / mcx_parse_args  <- init() defaults + PetscOptionsGet, DMSetFromOptions,
 *                                         KSPSetFromOptions   src/init.c:47-83,93,156
 *   mcx_init                          <- init() grid/Mat/Vec/KSP part  src/init.c:85-171,
 *                                         bc_init src/bcs.c:154-195
 *   mcx_finalize                      <- finish()  src/init.c:222-237
 *   mcx_get_displacement              <- get_displacement  src/bcs.c:52-58
 *   mcx_apply_bc_u                    <- apply_bc_on_u  src/bcs.c:29-45 (-> :61-146)
 *   mcx_set_strains                   <- set_strains  src/assembly.c:25-66
 *   mcx_homogenize                    <- micropp_C_homogenize  src/main.c:62 (device-batched
 *                                         constitutive callback, see mcx_material_set)
 *   mcx_assembly_res                  <- assembly_res + VecNorm  src/assembly.c:120-176,
 *                                         src/main.c:67
 *   mcx_assembly_jac                  <- assembly_jac + apply_bc_on_jac  src/assembly.c:69-117,
 *                                         src/bcs.c:341-347
 *   mcx_solve                         <- solve_Ax -> KSPSolve(CG, Jacobi)  src/assembly.c:179-192
 *   mcx_update_u                      <- VecAXPY(u, 1., du)  src/main.c:79
 *   mcx_material_set                  <- micropp_C_material_set  src/init.c:196-201
 *   mcx_set_micropp / mcx_set_device_law / mcx_set_gp_stress / mcx_set_gp_ctan
 *                                     <- the MicroPP C-wrapper boundary itself: micropp_C_set_strain3
 *                                        src/assembly.c:59, micropp_C_homogenize src/main.c:62,
 *                                        micropp_C_get_stress3 src/assembly.c:149,
 *                                        micropp_C_get_ctan3 src/assembly.c:92,
 *                                        micropp_C_update_vars src/main.c:83,
 *                                        micropp_C_get_non_linear_gps / _get_f_trial_max
 *                                        src/util.c:71,96 (-mat_law external)
 */
#ifndef MACROC_AMD_H
#define MACROC_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MCX_COMM_ID_BYTES 128 /* size of an ncclUniqueId */

/* ABI revision of this header.  Revision 3 (round 6) adds mcx_abi_version and mcx_comm_info;
   revision 2 (round 5) grew the structs mcx_info by st_listed and mcx_timing by cg_vec_bytes_per_iter, so a
   caller built against an older header passes smaller structs: check
   mcx_abi_version() == MCX_ABI_VERSION before calling mcx_get_info / mcx_get_timing / mcx_plan. */
#define MCX_ABI_VERSION 3

enum { MCX_BC_BENDING = 0, MCX_BC_CIRCLE = 1 }; /* include/macroc.h:58 */

/* KSPConvergedReason (PETSc) */
enum {
  MCX_KSP_CONVERGED_ITERATING = 0,
  MCX_KSP_CONVERGED_RTOL = 2,
  MCX_KSP_CONVERGED_ATOL = 3,
  MCX_KSP_DIVERGED_ITS = -3,
  MCX_KSP_DIVERGED_DTOL = -4,
  MCX_KSP_DIVERGED_INDEFINITE_PC = -8,
  MCX_KSP_DIVERGED_NANORINF = -9,
  MCX_KSP_DIVERGED_INDEFINITE_MAT = -10
};

/* matrix storage: -dm_mat_type aij (default, the reference's MATAIJ, src/init.c:92) or
   sbaij (PETSc MATSBAIJ semantics with -mat_ignore_lower_triangular: upper triangle kept,
   lower triangle mirrored from it) */
enum { MCX_MAT_AIJ = 0, MCX_MAT_SBAIJ = 1 };

/* constitutive laws behind the Gauss-point callback (-mat_law elastic|plastic|external):
   device isotropic elastic, device J2 plasticity (MicroPP material type 1), or an external law
   registered through mcx_set_micropp / mcx_set_device_law / mcx_set_gp_stress+ctan */
enum { MCX_LAW_ELASTIC = 0, MCX_LAW_PLASTIC = 1, MCX_LAW_EXTERNAL = 2 };

typedef struct {
  int64_t NX, NY, NZ;          /* -da_grid_x/y/z          (default 40 3 40, include/macroc.h:44-46) */
  int px, py, pz;              /* -da_processors_x/y/z    (0 = PETSC_DECIDE) */
  double lx, ly, lz;           /* -lx -ly -lz             (50 1 50) */
  double dt, final_time;       /* -dt                     (0.001, FINAL_TIME 1.0) */
  int ts;                      /* -ts                     (1) */
  int vtu_freq;                /* -vtu_freq               (-1: no VTU output; mcx_write_vtu) */
  int bc_type;                 /* -bc_type                (BC_CIRCLE) */
  double rad;                  /* load-circle radius      (1.0, src/init.c:141) */
  int newton_max_its;          /* -newton_max_its         (5) */
  double newton_min_tol;       /* -newton_min_tol         (0.1) */
  double newton_rel_tol;       /* -newton_rel_tol         (1e-4) */
  double ksp_rtol, ksp_abstol, ksp_dtol; /* -ksp_rtol -ksp_atol -ksp_divtol (1e-5 1e-50 1e4) */
  int ksp_max_it;              /* -ksp_max_it             (10000) */
  int micro_n, micro_type;     /* -micro_n -micro_type    (2, 1) */
  double micro_mat_1[4];       /* -micro_mat_1 E,nu,Sy,Ka (1e7,.25,1e4,1e7) */
  double micro_mat_2[4];       /* -micro_mat_2 */
  int device;                  /* HIP device of this rank (-1: rank % device count) */
  int ksp_monitor;             /* -ksp_monitor: keep the residual history */
  int mat_type;                /* -dm_mat_type aij|sbaij  (MCX_MAT_AIJ) */
  int mat_law;                 /* -mat_law elastic|plastic (MCX_LAW_ELASTIC; plastic = J2 with
                                  micro_mat_1's Sy, Ka: MicroPP material type 1) */
  int mat_aij_split;           /* -mat_aij_split 0|1 (1): hold the AIJ matrix exactly as upper blocks +
                                  bf16 lower corrections when all are exact (else plain AIJ blocks);
                                  0: AIJ blocks, rows summed in the reference's MatMult order (inode column pairs) (bit-exact SpMV) */
  int mat_aij_vi;              /* -mat_aij_vi 0|1 (1): hold the AIJ matrix exactly as one index byte per
                                  value into a dictionary of its distinct values when there are at most
                                  256 (value-indexed AIJ; rows summed in the reference's MatMult order (inode column pairs), bit-exact
                                  SpMV); otherwise -mat_aij_split decides */
  int mat_vi_fma;              /* -mat_vi_fma 0|1 (1): the value-indexed SpMV's z-marching kernel sums
                                  each row with fused multiply-adds (one rounding per term, what a
                                  PETSc built with -march=native does in MatMult), rows within
                                  1e-14 sum|a_ij x_j| of the reference's MatMult order (inode column pairs); 0: separate multiply and
                                  add in the reference's MatMult order (inode column pairs) (bit-exact SpMV) */
} mcx_opts;

typedef struct {
  int64_t NX, NY, NZ;
  int px, py, pz;              /* rank grid actually used */
  int rank, nranks;
  int64_t xs, ys, zs, nx, ny, nz;   /* owned node corners (DMDAGetCorners) */
  int64_t Xs, Ys, Zs, Nx, Ny, Nz;   /* ghost corners (DMDAGetGhostCorners) */
  int64_t ndofs_global;
  int64_t ndofs_local;          /* 3*nx*ny*nz, PETSc-global rows owned */
  int64_t dof_offset;           /* first global PETSc row of this rank */
  int64_t nnz_local;            /* AIJ nonzeros of the owned rows (pattern of DMCreateMatrix) */
  int64_t nnz_global;
  int64_t nelem_local;          /* DMDAGetElementsSizes product (PETSc-owned elements) */
  int64_t nelem_ext;            /* elements evaluated on this device (owned + upper ghost layer) */
  double dx, dy, dz, wg;        /* src/init.c:137-140 */
  int64_t device_bytes;         /* device memory held by the context */
  int device;
  int storage;                  /* matrix as last assembled: 0 AIJ blocks, 1 SBAIJ upper blocks,
                                   2 AIJ-split (upper blocks + bf16 lower corrections),
                                   3 AIJ value-indexed (index bytes + dictionary) */
  int split_slots;              /* AIJ-split: correction slots stored per node (of 117) */
  int split_bits;               /* AIJ-split: bits per correction (16 = bf16, 32 = f32) */
  /* Gauss-point box of the constitutive callback: the elements this context evaluates, x
     fastest from element (ex0, ey0, ez0) (global element = lower-left node), nelem_ext =
     nex*ney*nez; Gauss point gpi = ie*8 + gp.  One rank: DMDAGetElements' own order.  Several
     ranks: the rank's PETSc elements plus the upper ghost layer (owner computes). */
  int64_t ex0, ey0, ez0, nex, ney, nez;
  int vi_values;                /* value-indexed AIJ: distinct matrix values */
  int vi_bits;                  /* value-indexed AIJ: 4 = a nibble per value into its slot's dictionary
                                   (every slot takes <= 16 values), 8 = a byte into one dictionary */
  int vi_blocks;                /* value-indexed AIJ, block mode: distinct 3x3 blocks (one index byte per
                                   block into a dictionary of them), 0 when values are indexed one by one */
  int spmv_tx, spmv_ty, spmv_kc; /* SpMV of the last assembled storage when it is a z-marching tile kernel:
                                   tile width (x nodes), height (y rows) and planes per z-chunk; 0 for the
                                   gathered (one-node-per-thread) kernels */
  int64_t vi_exc_nodes;         /* value-indexed AIJ, block mode: owned nodes whose 27 blocks are stored as
                                   plain values (a per-GP-tangent law: the nodes touching an element whose
                                   tangent differs from the law's reference tangent) */
  int64_t split_escapes;        /* AIJ-split with dense bf16 corrections: corrections not exact in bf16, kept as
                                   their bf16 hi plus an exact double residual (0 otherwise) */
  int64_t st_listed;            /* value-indexed AIJ through the default-stencil SpMV: owned nodes whose 27 blocks
                                   differ from the default (interior) stencil's, computed from their own index
                                   bytes or exception blocks; -1 when the SpMV does not take that path */
} mcx_info;

typedef struct {
  /* wall milliseconds of the last call of each phase (HIP events on the compute stream) */
  double strains_ms, homogenize_ms, residual_ms, jacobian_ms, solve_ms, update_ms;
  /* SpMV kernel inside the last mcx_solve: HIP event pairs around every 8th launch (at most
     512), their count and summed device time */
  int64_t spmv_launches;
  double spmv_ms_total;
  int64_t spmv_bytes_per_launch; /* algorithmic bytes of one SpMV (values + x once + y once) */
  /* algorithmic bytes of the CG vector kernels per iteration of the last solve, averaged over the
     iterations (VecAXPY(r) + PCApply_Jacobi + the two dots, VecAYPX(p), the deferred VecAXPY(x)
     amortised over the iterations that apply it): with spmv_bytes_per_launch the bytes of one
     whole CG iteration */
  int64_t cg_vec_bytes_per_iter;
} mcx_timing;

const char* mcx_last_error(void);
const char* mcx_version(void);
int mcx_abi_version(void); /* MCX_ABI_VERSION of the library's build */

void mcx_default_opts(mcx_opts* o);
/* parse the reference's command-line surface (PETSc options-DB names); unknown flags are
   warned about on stderr and ignored, like the reference's options DB */
int mcx_parse_args(mcx_opts* o, int argc, const char* const* argv);

/* rank 0 creates the communicator id, the host transports it to every rank (MPI_Bcast,
   torch.distributed, a file ...).  Only needed when nranks > 1. */
int mcx_comm_unique_id(void* id /* MCX_COMM_ID_BYTES */);

/* Host-only planning (no GPU needed): the DMDA decomposition a rank would get, and its
   forward-halo plan — neighbour ranks and, per neighbour, the natural node ids
   (i + j*NX + k*NX*NY) sent and received, in message order.  Pass NULL arrays to query
   counts (*nnbr <= 26; *nsend / *nrecv = total nodes). */
int mcx_plan(const mcx_opts* o, int rank, int nranks, mcx_info* info);
int mcx_plan_halo(const mcx_opts* o, int rank, int nranks, int* nnbr, int* nbr_rank, int64_t* send_cnt,
                  int64_t* recv_cnt, int64_t* send_nat, int64_t* recv_nat, int64_t* nsend, int64_t* nrecv);

/* comm_id: rank 0's mcx_comm_unique_id, required when nranks > 1; with nranks == 1 a non-NULL id
   makes a one-rank RCCL communicator, so the reductions take the multi-rank (RCCL) path */
int mcx_init(const mcx_opts* o, int rank, int nranks, const void* comm_id, void** ctx);
/* In-process transport: `nranks` contexts on one device, each driven by its own host thread,
   exchanging halos / partial sums by device copies (multi-rank path without RCCL; every
   collective entry point must then be called by all members). */
int mcx_local_group_create(int nranks, int device, void** group);
int mcx_local_group_destroy(void* group);
/* MPI_Barrier(PETSC_COMM_WORLD) of the in-process transport (host only).  Every crossing of the
   group's barrier — this one and those inside the collective entry points — is tagged with its
   collective: a member reaching a different collective than the others, or a member missing for
   MCX_COMM_TIMEOUT seconds (environment at group creation, default 300), fails the crossing with
   a non-zero code naming the ranks and collectives, and every later crossing of that group fails
   at once (instead of pairing unrelated collectives or hanging). */
int mcx_local_group_barrier(void* group, int rank);
int mcx_init_local(const mcx_opts* o, int rank, void* group, void** ctx);
int mcx_finalize(void* ctx);
int mcx_get_info(void* ctx, mcx_info* info);
/* the ranks that actually joined this context's communicator (MPI_Comm_size / MPI_Comm_rank of
   PETSC_COMM_WORLD): ncclCommCount, ncclCommUserRank and ncclCommCuDevice of the RCCL
   communicator; the group size and member rank of the in-process transport; 1, 0 and the
   context's device without a communicator.  Any pointer may be NULL. */
int mcx_comm_info(void* ctx, int* comm_ranks, int* comm_rank, int* device);

/* Gauss-point constitutive model (micropp_C_material_set(id,E,nu,Sy,Ka,type)) */
int mcx_material_set(void* ctx, int id, double E, double nu, double Sy, double Ka, int type);

/* ---- the MicroPP Gauss-point callback boundary (-mat_law external) ----
 * The reference hands every Gauss point's strain to MicroPP's C wrapper and reads stress and
 * tangent back per Gauss point (src/assembly.c:59,92,149, src/main.c:62,83).  With -mat_law
 * external the device laws are replaced by one of:
 *  (1) host callbacks with the wrapper's call shapes (a real MicroPP links straight in:
 *      api.set_strain3 = micropp_C_set_strain3, ...).  mcx_homogenize then copies the strains to
 *      the host, calls set_strain3(gpi, strain) for every Gauss point (gpi = ie*8 + gp over
 *      mcx_info's Gauss-point box, ascending), homogenize() once, get_stress3(gpi, stress) and
 *      get_ctan3(gpi, ctan) for every Gauss point, and copies stress and tangent back.
 *      mcx_update_vars calls update_vars(); the non-linear statistics come from
 *      get_non_linear_gps / get_f_trial_max when given.
 *  (2) a device law: law->homogenize(law->user, &batch) runs on the context's stream with
 *      device pointers to strain, stress and tangent (the same contract as the built-in laws).
 *  (3) batched injection: mcx_set_gp_stress / mcx_set_gp_ctan copy caller-computed values
 *      (host, [ngp][6] / [ngp][36], gpi order) into the device arrays; mcx_get_gp_strain reads
 *      the strains of the same box.
 * Stress and tangent are Voigt (xx, yy, zz, xy, xz, yz; engineering shear), the tangent row
 * major (ctan[k*6+l], src/assembly.c:99).  Pass NULL to unregister. */
typedef struct {
  void (*set_strain3)(int gpi, double* strain);  /* micropp_C_set_strain3   src/assembly.c:59 */
  void (*homogenize)(void);                      /* micropp_C_homogenize    src/main.c:62 */
  void (*get_stress3)(int gpi, double* stress);  /* micropp_C_get_stress3   src/assembly.c:149 */
  void (*get_ctan3)(int gpi, double* ctan);      /* micropp_C_get_ctan3     src/assembly.c:92 */
  void (*update_vars)(void);                     /* micropp_C_update_vars   src/main.c:83 (may be NULL) */
  int (*get_non_linear_gps)(void);               /* src/util.c:71 (may be NULL) */
  double (*get_f_trial_max)(void);               /* src/util.c:96 (may be NULL) */
} mcx_micropp_api;

typedef struct {
  int64_t nelem;      /* elements of the Gauss-point box (mcx_info.nelem_ext) */
  int64_t ngp;        /* 8 * nelem */
  const double* eps;  /* device [6][8][nelem]: component k of GP gp of element e at k*ngp + gp*nelem + e */
  double* sig;        /* device, same layout */
  double* ctan;       /* device [36][8][nelem]: ctan[k*6+l] of GP gp of element e at (k*6+l)*ngp + gp*nelem + e */
  void* stream;       /* the context's HIP stream: launch on it, or finish before returning */
} mcx_gp_batch;

typedef struct {
  int (*homogenize)(void* user, const mcx_gp_batch* batch);            /* required; 0 = OK */
  int (*update_vars)(void* user);                                      /* may be NULL */
  int (*nonlinear_stats)(void* user, int64_t* n_nonlinear, double* f_trial_max); /* may be NULL */
  void* user;
} mcx_device_law;

int mcx_set_micropp(void* ctx, const mcx_micropp_api* api);
int mcx_set_device_law(void* ctx, const mcx_device_law* law);
int mcx_set_gp_stress(void* ctx, const double* host /* [ngp][6] */);
int mcx_set_gp_ctan(void* ctx, const double* host /* [ngp][36] */);
int mcx_get_gp_strain(void* ctx, double* host /* [ngp][6] */);

double mcx_get_displacement(void* ctx, int time_s);
int mcx_zero_u(void* ctx);                 /* VecZeroEntries(u)  src/init.c:103 */
int mcx_apply_bc_u(void* ctx, double U);
int mcx_set_strains(void* ctx);
int mcx_homogenize(void* ctx);
int mcx_assembly_res(void* ctx, double* norm2);
int mcx_assembly_jac(void* ctx);
int mcx_solve(void* ctx, int* its, double* rnorm, int* reason);
int mcx_update_u(void* ctx);
/* micropp_C_update_vars (src/main.c:83): commit the Gauss-point history of the time step */
int mcx_update_vars(void* ctx);
/* get_non_linear_gps / get_f_trial_max (src/util.c:69-102) over this rank's PETSc-owned
   elements: GPs with f_trial > 0 in the last homogenize, and the max f_trial */
int mcx_get_nonlinear_stats(void* ctx, int64_t* n_nonlinear, double* f_trial_max);

/* get_non_linear_gps + get_f_trial_max (src/util.c:69-102, called at src/main.c:88,93):
 * collective.  n_local = this rank's count (its gauss_evolution.dat column), n_total = the sum
 * over ranks (MPI_Gather + sum), f_trial_max = the max over ranks (MPI_Reduce MAX). */
int mcx_reduce_nonlinear(void* ctx, int64_t* n_local, int64_t* n_total, double* f_trial_max);

/* calc_force (src/forces.c:25-166, called at src/main.c:91): reaction force of the load case
 * from the Gauss-point stresses of the last homogenize — BC_CIRCLE: sum over the top element
 * layer inside the load circle of (sum over 8 GPs of sigma_yy) * dx * dz; BC_BENDING: last x
 * layer, sigma_xy * dy * dz; per rank in the reference's loop order and element set, then
 * summed over ranks.  Collective; every rank receives the total. */
int mcx_calc_force(void* ctx, double* force);

/* write_pvtu (src/output.c:25-267, called at src/main.c:100-108 every -vtu_freq time steps):
 * "<prefix>.pvtu" (rank 0) + "<prefix>-subdo-<rank>.vtu" with the ghosted box points, the
 * rank's elements, the ghosted displacement and cell data (part, cost = 0: no micro solver,
 * non-linear GP count, wg-weighted GP sums of strain and stress).  Collective (u halo). */
int mcx_write_vtu(void* ctx, const char* file_prefix);

/* src/main.c:57-82 for one time step; returns Newton iterations done, per-iteration
   |RES|, KSP its and KSP rnorm in caller arrays of length >= newton_max_its (may be NULL) */
int mcx_time_step(void* ctx, int time_s, int* newton_its, double* res, int* ksp_its, double* ksp_rnorm);

/* ---- data access (owned rows, PETSc-local order, host buffers) ---- */
int mcx_get_u(void* ctx, double* host);      /* ndofs_local */
int mcx_set_u(void* ctx, const double* host);
int mcx_get_b(void* ctx, double* host);
int mcx_get_du(void* ctx, double* host);
/* strains / stresses of the PETSc-owned elements, [ie*8+gp][6] (micropp gp index) */
int mcx_get_strain(void* ctx, double* host);
int mcx_get_stress(void* ctx, double* host);
/* global PETSc DOF of every owned local DOF, and its natural (i + j*NX + k*NX*NY)*3+d index */
int mcx_owned_dofs(void* ctx, int64_t* petsc, int64_t* natural);
/* owned rows of A in AIJ form: rowptr (ndofs_local+1, local offsets), global column ids
   sorted ascending, values (any pointer may be NULL) */
int mcx_dump_csr(void* ctx, int64_t* rowptr, int64_t* colidx, double* vals);
/* sorted global PETSc ids of the owned Dirichlet DOFs; *n in: capacity, out: count */
int mcx_dump_dirichlet(void* ctx, int64_t* idx, int64_t* n);
/* y = A x on owned rows (collective when nranks > 1) */
int mcx_spmv(void* ctx, const double* x_host, double* y_host);
/* KSP residual history of the last solve (ksp_monitor); *n in: capacity, out: count */
int mcx_get_ksp_history(void* ctx, double* hist, int64_t* n);

int mcx_set_timing(void* ctx, int on);
int mcx_get_timing(void* ctx, mcx_timing* t);
int mcx_synchronize(void* ctx);
/* tuning knobs ("spmv_subl": lines per sub-slab of the SpMV sweep, 0 = whole XCD slab) and a
   device-only SpMV timer (iters launches on the current search direction, HIP events) */
int mcx_set_option(void* ctx, const char* name, double value);
int mcx_time_spmv(void* ctx, int iters, double* avg_ms);

#ifdef __cplusplus
}
#endif
#endif
