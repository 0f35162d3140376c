/*
 * oracle.c — CPU restatement of MacroC's Newton inner loop.  TEST INFRASTRUCTURE ONLY
 * (see oracle.h for scope, citations and the pinning status).  Compiled with
 * -ffp-contract=off so that every product/sum is rounded in the order written, as the
 * reference's x86-64 build (no FMA) does.
 */
#include "oracle.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define NGP 8
#define NPE 8
#define NVOI 6
#define DIM 3
#define CONSTXG 0.577350269189626 /* include/macroc.h:52 (truncated 1/sqrt(3), kept) */
#define U_MAX (-1.0)              /* include/macroc.h:51 */

/* include/macroc.h:61-69 */
static const double xg[8][3] = {{-CONSTXG, -CONSTXG, -CONSTXG}, {+CONSTXG, -CONSTXG, -CONSTXG},
                                {+CONSTXG, +CONSTXG, -CONSTXG}, {-CONSTXG, +CONSTXG, -CONSTXG},
                                {-CONSTXG, -CONSTXG, +CONSTXG}, {+CONSTXG, -CONSTXG, +CONSTXG},
                                {+CONSTXG, +CONSTXG, +CONSTXG}, {-CONSTXG, +CONSTXG, +CONSTXG}};

typedef struct {
  int64_t row, col;
  double v;
} stash_entry;

struct orc_problem {
  orc_opts o;
  int m, n, p, nranks;
  int64_t *lxw, *lyw, *lzw;  /* ownership widths per processor column */
  int64_t *xs0, *ys0, *zs0;  /* ownership starts */
  int *ipx, *ipy, *ipz;      /* processor coordinate of each node index */
  int64_t *node_off;         /* first global node of each rank (nranks+1) */
  int64_t ndofs;
  double dx, dy, dz, wg;
  int64_t *ne, *gp_off, ngp;
  int64_t *rowptr;
  int32_t *colidx;
  double *val;
  int64_t nnz;
  double *u, *b, *du;
  double *eps, *sig, *ctan;
  double *hist_old, *hist_new;  /* [ngp][7]: plastic strain (tensor components) + alpha */
  double *ftrial;
  double C[36];
  double Btab[NGP][NVOI][NPE * DIM];
  int64_t *dir;
  int64_t ndir;
  double *r, *z, *pp, *w, *dinv; /* CG work vectors */
  int spmv_order;                /* ORC_SPMV_INODE (MATAIJ default) | ORC_SPMV_SEQAIJ (plain; SBAIJ mirror) */
};

/* ------------------------------------------------------------------------------------
 * calc_B — src/assembly.c:195-254.  Unit reference cube (local dx=dy=dz=1, :198),
 * expressions evaluated in the order written (:202-231), Voigt rows :234-253.
 * ---------------------------------------------------------------------------------- */
void orc_calc_B(int gp, double B[6][24]) {
  int i;
  double dx = 1., dy = 1., dz = 1.;
  const double dsh[NPE][DIM] = {
      {-(1 - xg[gp][1]) * (1 - xg[gp][2]) / 8. * 2. / dx, -(1 - xg[gp][0]) * (1 - xg[gp][2]) / 8. * 2. / dy,
       -(1 - xg[gp][0]) * (1 - xg[gp][1]) / 8. * 2. / dz},
      {+(1 - xg[gp][1]) * (1 - xg[gp][2]) / 8. * 2. / dx, -(1 + xg[gp][0]) * (1 - xg[gp][2]) / 8. * 2. / dy,
       -(1 + xg[gp][0]) * (1 - xg[gp][1]) / 8. * 2. / dz},
      {+(1 + xg[gp][1]) * (1 - xg[gp][2]) / 8. * 2. / dx, +(1 + xg[gp][0]) * (1 - xg[gp][2]) / 8. * 2. / dy,
       -(1 + xg[gp][0]) * (1 + xg[gp][1]) / 8. * 2. / dz},
      {-(1 + xg[gp][1]) * (1 - xg[gp][2]) / 8. * 2. / dx, +(1 - xg[gp][0]) * (1 - xg[gp][2]) / 8. * 2. / dy,
       -(1 - xg[gp][0]) * (1 + xg[gp][1]) / 8. * 2. / dz},
      {-(1 - xg[gp][1]) * (1 + xg[gp][2]) / 8. * 2. / dx, -(1 - xg[gp][0]) * (1 + xg[gp][2]) / 8. * 2. / dy,
       +(1 - xg[gp][0]) * (1 - xg[gp][1]) / 8. * 2. / dz},
      {+(1 - xg[gp][1]) * (1 + xg[gp][2]) / 8. * 2. / dx, -(1 + xg[gp][0]) * (1 + xg[gp][2]) / 8. * 2. / dy,
       +(1 + xg[gp][0]) * (1 - xg[gp][1]) / 8. * 2. / dz},
      {+(1 + xg[gp][1]) * (1 + xg[gp][2]) / 8. * 2. / dx, +(1 + xg[gp][0]) * (1 + xg[gp][2]) / 8. * 2. / dy,
       +(1 + xg[gp][0]) * (1 + xg[gp][1]) / 8. * 2. / dz},
      {-(1 + xg[gp][1]) * (1 + xg[gp][2]) / 8. * 2. / dx, +(1 - xg[gp][0]) * (1 + xg[gp][2]) / 8. * 2. / dy,
       +(1 - xg[gp][0]) * (1 + xg[gp][1]) / 8. * 2. / dz}};
  for (i = 0; i < NPE; ++i) {
    B[0][i * DIM] = dsh[i][0];
    B[0][i * DIM + 1] = 0;
    B[0][i * DIM + 2] = 0;
    B[1][i * DIM] = 0;
    B[1][i * DIM + 1] = dsh[i][1];
    B[1][i * DIM + 2] = 0;
    B[2][i * DIM] = 0;
    B[2][i * DIM + 1] = 0;
    B[2][i * DIM + 2] = dsh[i][2];
    B[3][i * DIM] = dsh[i][1];
    B[3][i * DIM + 1] = dsh[i][0];
    B[3][i * DIM + 2] = 0;
    B[4][i * DIM] = dsh[i][2];
    B[4][i * DIM + 1] = 0;
    B[4][i * DIM + 2] = dsh[i][0];
    B[5][i * DIM] = 0;
    B[5][i * DIM + 1] = dsh[i][2];
    B[5][i * DIM + 2] = dsh[i][1];
  }
}

/* defaults: src/init.c:47-64, include/macroc.h:36-52, KSP src/init.c:146-148 */
void orc_default_opts(orc_opts* o) {
  memset(o, 0, sizeof(*o));
  o->NX = 40;
  o->NY = 3;
  o->NZ = 40;
  o->nranks = 1;
  o->lx = 50.0;
  o->ly = 1.0;
  o->lz = 50.0;
  o->dt = 0.001;
  o->final_time = 1.0;
  o->ts = 1;
  o->bc_type = ORC_BC_CIRCLE;
  o->rad = 1.0;
  o->newton_max_its = 5;
  o->newton_min_tol = 1.0e-1;
  o->newton_rel_tol = 1.0e-4;
  o->rtol = 1.0e-5;
  o->abstol = 1.0e-50;
  o->dtol = 1.0e4;
  o->maxits = 10000;
  o->E = 1.0e7;
  o->nu = 0.25;
  o->Sy = 1.0e4;
  o->Ka = 1.0e7;
  o->law = 0;
}

/* ------------------------------------------------------------------------------------
 * PETSc DMSetUp_DA_3D partition (src/dm/impls/da/da3.c) [ext, restated, unpinned
 * except through the 2-rank known answer of tests/test_dm_1.c:5-19].
 * ---------------------------------------------------------------------------------- */
int orc_dmda_decide(int64_t M, int64_t N, int64_t P, int size, int* pm_, int* pn_, int* pp_) {
  int64_t m = *pm_ > 0 ? *pm_ : -1, n = *pn_ > 0 ? *pn_ : -1, p = *pp_ > 0 ? *pp_ : -1, pm;
  const int64_t D = -1;
  if (m != D && (m < 1 || m > size)) return 1;
  if (n != D && (n < 1 || n > size)) return 1;
  if (p != D && (p < 1 || p > size)) return 1;
  if (m > 0 && n > 0 && p > 0 && m * n * p != size) return 2;
  if (m == D && n != D && p != D) {
    m = size / (n * p);
  } else if (m != D && n == D && p != D) {
    n = size / (m * p);
  } else if (m != D && n != D && p == D) {
    p = size / (m * n);
  } else if (m == D && n == D && p != D) {
    m = (int64_t)(0.5 + sqrt(((double)M) * ((double)size) / ((double)N * p)));
    if (!m) m = 1;
    while (m > 0) {
      n = size / (m * p);
      if (m * n * p == size) break;
      m--;
    }
    if (!m) return 3;
    if (M > N && m < n) { int64_t t = m; m = n; n = t; }
  } else if (m == D && n != D && p == D) {
    m = (int64_t)(0.5 + sqrt(((double)M) * ((double)size) / ((double)P * n)));
    if (!m) m = 1;
    while (m > 0) {
      p = size / (m * n);
      if (m * n * p == size) break;
      m--;
    }
    if (!m) return 3;
    if (M > P && m < p) { int64_t t = m; m = p; p = t; }
  } else if (m != D && n == D && p == D) {
    n = (int64_t)(0.5 + sqrt(((double)N) * ((double)size) / ((double)P * m)));
    if (!n) n = 1;
    while (n > 0) {
      p = size / (m * n);
      if (m * n * p == size) break;
      n--;
    }
    if (!n) return 3;
    if (N > P && n < p) { int64_t t = n; n = p; p = t; }
  } else if (m == D && n == D && p == D) {
    n = (int64_t)(0.5 + pow(((double)N * N) * ((double)size) / ((double)P * M), 1. / 3.));
    if (!n) n = 1;
    while (n > 0) {
      pm = size / n;
      if (n * pm == size) break;
      n--;
    }
    if (!n) n = 1;
    m = (int64_t)(0.5 + sqrt(((double)M) * ((double)size) / ((double)P * n)));
    if (!m) m = 1;
    while (m > 0) {
      p = size / (m * n);
      if (m * n * p == size) break;
      m--;
    }
    if (M > P && m < p) { int64_t t = m; m = p; p = t; }
  }
  if (m * n * p != size) return 2;
  if (M < m || N < n || P < p) return 4; /* "Partition in x direction is too fine!" */
  *pm_ = (int)m;
  *pn_ = (int)n;
  *pp_ = (int)p;
  return 0;
}

/* ---------------------------------------------------------------- DMDA numbering */
static int64_t petsc_node(const orc_problem* P, int64_t i, int64_t j, int64_t k) {
  int pi = P->ipx[i], pj = P->ipy[j], pk = P->ipz[k];
  int r = pi + pj * P->m + pk * P->m * P->n;
  int64_t nx = P->lxw[pi], ny = P->lyw[pj];
  return P->node_off[r] + (i - P->xs0[pi]) + (j - P->ys0[pj]) * nx + (k - P->zs0[pk]) * nx * ny;
}

static void rank_coords(const orc_problem* P, int r, int* pi, int* pj, int* pk) {
  *pi = r % P->m;
  *pj = (r % (P->m * P->n)) / P->m;
  *pk = r / (P->m * P->n);
}

/* owned corners + ghost corners (DMDAGetCorners / DMDAGetGhostCorners, stencil width 1,
   DM_BOUNDARY_NONE) */
void orc_rank_corners(const orc_problem* P, int r, int64_t* c) {
  int pi, pj, pk;
  rank_coords(P, r, &pi, &pj, &pk);
  int64_t xs = P->xs0[pi], ys = P->ys0[pj], zs = P->zs0[pk];
  int64_t nx = P->lxw[pi], ny = P->lyw[pj], nz = P->lzw[pk];
  int64_t Xs = xs > 0 ? xs - 1 : 0, Ys = ys > 0 ? ys - 1 : 0, Zs = zs > 0 ? zs - 1 : 0;
  int64_t Xe = xs + nx < P->o.NX ? xs + nx + 1 : P->o.NX;
  int64_t Ye = ys + ny < P->o.NY ? ys + ny + 1 : P->o.NY;
  int64_t Ze = zs + nz < P->o.NZ ? zs + nz + 1 : P->o.NZ;
  c[0] = xs; c[1] = ys; c[2] = zs; c[3] = nx; c[4] = ny; c[5] = nz;
  c[6] = Xs; c[7] = Ys; c[8] = Zs; c[9] = Xe - Xs; c[10] = Ye - Ys; c[11] = Ze - Zs;
}

/* ghosted-local node id -> global PETSc node (ISLocalToGlobalMapping of the DMDA, /3) */
static int64_t ltog_node(const orc_problem* P, const int64_t* c, int64_t l) {
  int64_t Nx = c[9], Ny = c[10];
  int64_t gi = c[6] + l % Nx, gj = c[7] + (l / Nx) % Ny, gk = c[8] + l / (Nx * Ny);
  return petsc_node(P, gi, gj, gk);
}

/* DMDAGetElements (3-D, Q1) element ranges: i in [xs - (xs!=Xs), xe-1) per dim */
static void rank_elem_range(const orc_problem* P, int r, int64_t* lo, int64_t* cnt) {
  int64_t c[12];
  orc_rank_corners(P, r, c);
  for (int d = 0; d < 3; d++) {
    int64_t xs = c[d], xe = c[d] + c[3 + d], Xs = c[6 + d];
    int64_t s = (xs != Xs) ? xs - 1 : xs;
    lo[d] = s;
    cnt[d] = xe - 1 - s;
    if (cnt[d] < 0) cnt[d] = 0;
  }
}

int64_t orc_rank_nelem(const orc_problem* P, int r) { return P->ne[r]; }
int64_t orc_rank_dof_offset(const orc_problem* P, int r) { return 3 * P->node_off[r]; }
double orc_wg(const orc_problem* P) { return P->wg; }

void orc_rank_elements(const orc_problem* P, int r, int32_t* conn) {
  int64_t c[12], lo[3], cnt[3];
  orc_rank_corners(P, r, c);
  rank_elem_range(P, r, lo, cnt);
  int64_t Xs = c[6], Ys = c[7], Zs = c[8], Nx = c[9], Ny = c[10];
  int64_t e = 0;
  for (int64_t l = lo[2]; l < lo[2] + cnt[2]; l++)
    for (int64_t j = lo[1]; j < lo[1] + cnt[1]; j++)
      for (int64_t i = lo[0]; i < lo[0] + cnt[0]; i++) {
        int32_t* cell = conn + 8 * e++;
        cell[0] = (int32_t)((i - Xs) + (j - Ys) * Nx + (l - Zs) * Nx * Ny);
        cell[1] = (int32_t)((i - Xs + 1) + (j - Ys) * Nx + (l - Zs) * Nx * Ny);
        cell[2] = (int32_t)((i - Xs + 1) + (j - Ys + 1) * Nx + (l - Zs) * Nx * Ny);
        cell[3] = (int32_t)((i - Xs) + (j - Ys + 1) * Nx + (l - Zs) * Nx * Ny);
        cell[4] = (int32_t)((i - Xs) + (j - Ys) * Nx + (l - Zs + 1) * Nx * Ny);
        cell[5] = (int32_t)((i - Xs + 1) + (j - Ys) * Nx + (l - Zs + 1) * Nx * Ny);
        cell[6] = (int32_t)((i - Xs + 1) + (j - Ys + 1) * Nx + (l - Zs + 1) * Nx * Ny);
        cell[7] = (int32_t)((i - Xs) + (j - Ys + 1) * Nx + (l - Zs + 1) * Nx * Ny);
      }
}

static int rank_of_dof(const orc_problem* P, int64_t g) {
  int64_t node = g / 3;
  int lo = 0, hi = P->nranks - 1;
  while (lo < hi) {
    int mid = (lo + hi + 1) / 2;
    if (P->node_off[mid] <= node) lo = mid; else hi = mid - 1;
  }
  return lo;
}

void orc_dof_map(const orc_problem* P, int64_t* map) {
  const orc_opts* o = &P->o;
  for (int64_t k = 0; k < o->NZ; k++)
    for (int64_t j = 0; j < o->NY; j++)
      for (int64_t i = 0; i < o->NX; i++) {
        int64_t nat = i + j * o->NX + k * o->NX * o->NY;
        int64_t g = petsc_node(P, i, j, k);
        for (int d = 0; d < 3; d++) map[3 * nat + d] = 3 * g + d;
      }
}

/* ------------------------------------------------------------------------------------
 * Dirichlet index lists — bc_init_circle src/bcs.c:254-338, bc_init_bending :198-251.
 * Enumerated over the rank's GHOST corners exactly as the reference (Appendix A.8).
 * ---------------------------------------------------------------------------------- */
int64_t orc_rank_dirichlet(const orc_problem* P, int r, int64_t* ix, int64_t cap) {
  int64_t c[12];
  orc_rank_corners(P, r, c);
  int64_t si = c[6], sj = c[7], sk = c[8], nxg = c[9], nyg = c[10], nzg = c[11];
  const orc_opts* o = &P->o;
  int64_t nbcs, index = 0, i, j, k;
  int d;
  if (o->bc_type == ORC_BC_BENDING) nbcs = 2 * nyg * nzg * DIM;
  else nbcs = (2 * nxg + 2 * nzg) * DIM + nxg * nzg;
  if (!ix) return nbcs;
  if (cap < nbcs) return -1;
  for (i = 0; i < nbcs; i++) ix[i] = -1;
#define LID(i_, j_, k_) ((i_) + (j_) * nxg + (k_) * nxg * nyg)
  if (o->bc_type == ORC_BC_BENDING) {
    if (si == 0) {
      i = 0;
      for (k = 0; k < nzg; ++k)
        for (j = 0; j < nyg; ++j)
          for (d = 0; d < DIM; ++d) ix[index++] = 3 * ltog_node(P, c, LID(i, j, k)) + d;
    }
    if (si + nxg == o->NX) {
      i = nxg - 1;
      for (k = 0; k < nzg; ++k)
        for (j = 0; j < nyg; ++j)
          for (d = 0; d < DIM; ++d) ix[index++] = 3 * ltog_node(P, c, LID(i, j, k)) + d;
    }
    return nbcs;
  }
  if (si == 0 && sj == 0) {
    i = 0; j = 0;
    for (k = 0; k < nzg; ++k)
      for (d = 0; d < DIM; ++d) ix[index++] = 3 * ltog_node(P, c, LID(i, j, k)) + d;
  }
  if (si + nxg == o->NX && sj == 0) {
    i = nxg - 1; j = 0;
    for (k = 0; k < nzg; ++k)
      for (d = 0; d < DIM; ++d) ix[index++] = 3 * ltog_node(P, c, LID(i, j, k)) + d;
  }
  if (sk == 0 && sj == 0) {
    k = 0; j = 0;
    for (i = 1; i < nxg - 1; ++i)
      for (d = 0; d < DIM; ++d) ix[index++] = 3 * ltog_node(P, c, LID(i, j, k)) + d;
  }
  if (sk + nzg == o->NZ && sj == 0) {
    k = nzg - 1; j = 0;
    for (i = 1; i < nxg - 1; ++i)
      for (d = 0; d < DIM; ++d) ix[index++] = 3 * ltog_node(P, c, LID(i, j, k)) + d;
  }
  if (sj + nyg == o->NY) {
    j = nyg - 1;
    for (i = 0; i < nxg; ++i)
      for (k = 0; k < nzg; ++k) {
        double x = o->lx / 2. - ((si + i) * P->dx + P->dx / 2.);
        double z = o->lz / 2. - ((sk + k) * P->dz + P->dz / 2.);
        const int dd = 1;
        if ((x * x + z * z) < (o->rad * o->rad)) ix[index++] = 3 * ltog_node(P, c, LID(i, j, k)) + dd;
      }
  }
#undef LID
  return nbcs;
}

/* values list matching orc_rank_dirichlet order: bc_apply_on_u_circle src/bcs.c:94-146,
   bc_apply_on_u_bending :61-91 */
static int64_t rank_dirichlet_values(const orc_problem* P, int r, double U, double* vals) {
  int64_t c[12];
  orc_rank_corners(P, r, c);
  int64_t si = c[6], sj = c[7], sk = c[8], nxg = c[9], nyg = c[10], nzg = c[11];
  const orc_opts* o = &P->o;
  int64_t index = 0, i, j, k;
  int d;
  if (o->bc_type == ORC_BC_BENDING) {
    if (si == 0)
      for (k = 0; k < nzg; ++k)
        for (j = 0; j < nyg; ++j)
          for (d = 0; d < DIM; ++d) vals[index++] = 0.;
    if (si + nxg == o->NX)
      for (k = 0; k < nzg; ++k)
        for (j = 0; j < nyg; ++j)
          for (d = 0; d < DIM; ++d) vals[index++] = (d == 1) ? U : 0.;
    return index;
  }
  if (si == 0 && sj == 0)
    for (k = 0; k < nzg; ++k)
      for (d = 0; d < DIM; ++d) vals[index++] = 0.;
  if (si + nxg == o->NX && sj == 0)
    for (k = 0; k < nzg; ++k)
      for (d = 0; d < DIM; ++d) vals[index++] = 0.;
  if (sk == 0 && sj == 0)
    for (i = 1; i < nxg - 1; ++i)
      for (d = 0; d < DIM; ++d) vals[index++] = 0.;
  if (sk + nzg == o->NZ && sj == 0)
    for (i = 1; i < nxg - 1; ++i)
      for (d = 0; d < DIM; ++d) vals[index++] = 0.;
  if (sj + nyg == o->NY)
    for (i = 0; i < nxg; ++i)
      for (k = 0; k < nzg; ++k) {
        double x = o->lx / 2. - ((si + i) * P->dx + P->dx / 2.);
        double z = o->lz / 2. - ((sk + k) * P->dz + P->dz / 2.);
        if ((x * x + z * z) < (o->rad * o->rad)) vals[index++] = U;
      }
  return index;
}

static int cmp_i64(const void* a, const void* b) {
  int64_t x = *(const int64_t*)a, y = *(const int64_t*)b;
  return (x > y) - (x < y);
}

int64_t orc_dirichlet_set(const orc_problem* P, int64_t* out, int64_t cap) {
  if (!out) return P->ndir;
  if (cap < P->ndir) return -1;
  memcpy(out, P->dir, P->ndir * sizeof(int64_t));
  return P->ndir;
}

static void build_dirichlet_set(orc_problem* P) {
  int64_t tot = 0;
  for (int r = 0; r < P->nranks; r++) tot += orc_rank_dirichlet(P, r, NULL, 0);
  int64_t* all = malloc((tot + 1) * sizeof(int64_t));
  int64_t na = 0;
  for (int r = 0; r < P->nranks; r++) {
    int64_t nb = orc_rank_dirichlet(P, r, NULL, 0);
    int64_t* ix = malloc((nb + 1) * sizeof(int64_t));
    orc_rank_dirichlet(P, r, ix, nb);
    for (int64_t q = 0; q < nb; q++)
      if (ix[q] >= 0) all[na++] = ix[q];
    free(ix);
  }
  qsort(all, na, sizeof(int64_t), cmp_i64);
  int64_t nu = 0;
  for (int64_t q = 0; q < na; q++)
    if (nu == 0 || all[q] != all[nu - 1]) all[nu++] = all[q];
  P->dir = all;
  P->ndir = nu;
}

static int is_dirichlet(const orc_problem* P, int64_t g) {
  int64_t lo = 0, hi = P->ndir - 1;
  while (lo <= hi) {
    int64_t mid = (lo + hi) / 2;
    if (P->dir[mid] == g) return 1;
    if (P->dir[mid] < g) lo = mid + 1; else hi = mid - 1;
  }
  return 0;
}

/* ------------------------------------------------------------------------------------
 * AIJ pattern that DMCreateMatrix gives a DMDA with DMDA_STENCIL_BOX, s=1, dof=3
 * [ext]: full 27-node box x 3x3 coupling, clipped at the domain, columns sorted.
 * ---------------------------------------------------------------------------------- */
static int cmp_i32(const void* a, const void* b) {
  int32_t x = *(const int32_t*)a, y = *(const int32_t*)b;
  return (x > y) - (x < y);
}

static void build_csr(orc_problem* P) {
  const orc_opts* o = &P->o;
  int64_t nrows = P->ndofs;
  P->rowptr = malloc((nrows + 1) * sizeof(int64_t));
  /* first pass: counts (rows enumerated in PETSc order = rank, local node, dof) */
  int64_t nnz = 0;
  P->rowptr[0] = 0;
  int64_t row = 0;
  for (int r = 0; r < P->nranks; r++) {
    int64_t c[12];
    orc_rank_corners(P, r, c);
    for (int64_t k = c[2]; k < c[2] + c[5]; k++)
      for (int64_t j = c[1]; j < c[1] + c[4]; j++)
        for (int64_t i = c[0]; i < c[0] + c[3]; i++) {
          int64_t cx = (i > 0) + 1 + (i < o->NX - 1), cy = (j > 0) + 1 + (j < o->NY - 1),
                  cz = (k > 0) + 1 + (k < o->NZ - 1);
          int64_t cnt = 3 * cx * cy * cz;
          for (int d = 0; d < 3; d++) {
            nnz += cnt;
            P->rowptr[++row] = nnz;
          }
        }
  }
  P->nnz = nnz;
  P->colidx = malloc(nnz * sizeof(int32_t));
  P->val = calloc(nnz, sizeof(double));
  row = 0;
  for (int r = 0; r < P->nranks; r++) {
    int64_t c[12];
    orc_rank_corners(P, r, c);
    for (int64_t k = c[2]; k < c[2] + c[5]; k++)
      for (int64_t j = c[1]; j < c[1] + c[4]; j++)
        for (int64_t i = c[0]; i < c[0] + c[3]; i++) {
          int32_t cols[81];
          int nc = 0;
          for (int64_t kk = k - 1; kk <= k + 1; kk++)
            for (int64_t jj = j - 1; jj <= j + 1; jj++)
              for (int64_t ii = i - 1; ii <= i + 1; ii++) {
                if (ii < 0 || jj < 0 || kk < 0 || ii >= o->NX || jj >= o->NY || kk >= o->NZ) continue;
                int64_t g = petsc_node(P, ii, jj, kk);
                for (int d = 0; d < 3; d++) cols[nc++] = (int32_t)(3 * g + d);
              }
          qsort(cols, nc, sizeof(int32_t), cmp_i32);
          for (int d = 0; d < 3; d++) {
            memcpy(P->colidx + P->rowptr[row], cols, nc * sizeof(int32_t));
            row++;
          }
        }
  }
}

void orc_csr_pattern(const orc_problem* P, int64_t* rowptr, int32_t* colidx) {
  if (rowptr) memcpy(rowptr, P->rowptr, (P->ndofs + 1) * sizeof(int64_t));
  if (colidx) memcpy(colidx, P->colidx, P->nnz * sizeof(int32_t));
}

static int64_t csr_find(const orc_problem* P, int64_t row, int64_t col) {
  int64_t lo = P->rowptr[row], hi = P->rowptr[row + 1] - 1;
  while (lo <= hi) {
    int64_t mid = (lo + hi) / 2;
    if (P->colidx[mid] == col) return mid;
    if (P->colidx[mid] < col) lo = mid + 1; else hi = mid - 1;
  }
  return -1;
}

/* isotropic linear-elastic tangent in Voigt order xx,yy,zz,xy,xz,yz with engineering
   shear — the MicroPP surrogate (A6).  Row-major ctan[k*6+l] as used at
   src/assembly.c:99. */
static void elastic_C(double E, double nu, double C[36]) {
  double lam = E * nu / ((1. + nu) * (1. - 2. * nu));
  double mu = E / (2. * (1. + nu));
  memset(C, 0, 36 * sizeof(double));
  for (int a = 0; a < 3; a++)
    for (int b = 0; b < 3; b++) C[a * 6 + b] = lam + (a == b ? 2. * mu : 0.);
  for (int a = 3; a < 6; a++) C[a * 6 + a] = mu;
}

orc_problem* orc_create(const orc_opts* o) {
  int m = o->m, n = o->n, p = o->p;
  if (o->NX < 2 || o->NY < 2 || o->NZ < 2) return NULL;
  if (orc_dmda_decide(o->NX, o->NY, o->NZ, o->nranks, &m, &n, &p)) return NULL;
  orc_problem* P = calloc(1, sizeof(*P));
  P->o = *o;
  P->m = m; P->n = n; P->p = p; P->nranks = o->nranks;
  int64_t dims[3] = {o->NX, o->NY, o->NZ};
  int procs[3] = {m, n, p};
  int64_t** wid[3] = {&P->lxw, &P->lyw, &P->lzw};
  int64_t** st[3] = {&P->xs0, &P->ys0, &P->zs0};
  int** ip[3] = {&P->ipx, &P->ipy, &P->ipz};
  for (int d = 0; d < 3; d++) {
    *wid[d] = malloc(procs[d] * sizeof(int64_t));
    *st[d] = malloc(procs[d] * sizeof(int64_t));
    *ip[d] = malloc(dims[d] * sizeof(int));
    int64_t s = 0;
    for (int q = 0; q < procs[d]; q++) {
      /* lx[i] = M/m + ((M % m) > i) */
      (*wid[d])[q] = dims[d] / procs[d] + ((dims[d] % procs[d]) > q);
      (*st[d])[q] = s;
      for (int64_t t = s; t < s + (*wid[d])[q]; t++) (*ip[d])[t] = q;
      s += (*wid[d])[q];
    }
  }
  P->node_off = malloc((P->nranks + 1) * sizeof(int64_t));
  P->node_off[0] = 0;
  for (int r = 0; r < P->nranks; r++) {
    int pi, pj, pk;
    rank_coords(P, r, &pi, &pj, &pk);
    P->node_off[r + 1] = P->node_off[r] + P->lxw[pi] * P->lyw[pj] * P->lzw[pk];
  }
  P->ndofs = 3 * P->node_off[P->nranks];
  /* src/init.c:137-141 */
  P->dx = o->lx / (o->NX - 1);
  P->dy = o->ly / (o->NY - 1);
  P->dz = o->lz / (o->NZ - 1);
  P->wg = P->dx * P->dy * P->dz / NPE;
  P->ne = malloc(P->nranks * sizeof(int64_t));
  P->gp_off = malloc((P->nranks + 1) * sizeof(int64_t));
  P->gp_off[0] = 0;
  for (int r = 0; r < P->nranks; r++) {
    int64_t lo[3], cnt[3];
    rank_elem_range(P, r, lo, cnt);
    P->ne[r] = cnt[0] * cnt[1] * cnt[2];
    P->gp_off[r + 1] = P->gp_off[r] + P->ne[r] * NGP;
  }
  P->ngp = P->gp_off[P->nranks];
  for (int g = 0; g < NGP; g++) orc_calc_B(g, P->Btab[g]);
  elastic_C(o->E, o->nu, P->C);
  build_dirichlet_set(P);
  build_csr(P);
  int64_t N = P->ndofs;
  P->u = calloc(N, sizeof(double));
  P->b = calloc(N, sizeof(double));
  P->du = calloc(N, sizeof(double));
  P->r = calloc(N, sizeof(double));
  P->z = calloc(N, sizeof(double));
  P->pp = calloc(N, sizeof(double));
  P->w = calloc(N, sizeof(double));
  P->dinv = calloc(N, sizeof(double));
  P->eps = calloc(P->ngp * NVOI, sizeof(double));
  P->sig = calloc(P->ngp * NVOI, sizeof(double));
  P->ctan = calloc(P->ngp * 36, sizeof(double));
  P->hist_old = calloc(P->ngp * 7, sizeof(double));
  P->hist_new = calloc(P->ngp * 7, sizeof(double));
  P->ftrial = calloc(P->ngp, sizeof(double));
  return P;
}

void orc_destroy(orc_problem* P) {
  if (!P) return;
  free(P->lxw); free(P->lyw); free(P->lzw);
  free(P->xs0); free(P->ys0); free(P->zs0);
  free(P->ipx); free(P->ipy); free(P->ipz);
  free(P->node_off); free(P->ne); free(P->gp_off);
  free(P->rowptr); free(P->colidx); free(P->val);
  free(P->u); free(P->b); free(P->du); free(P->r); free(P->z); free(P->pp); free(P->w);
  free(P->dinv); free(P->eps); free(P->sig); free(P->dir);
  free(P->ctan); free(P->hist_old); free(P->hist_new); free(P->ftrial);
  free(P);
}

int64_t orc_ndofs(const orc_problem* P) { return P->ndofs; }
int64_t orc_nnz(const orc_problem* P) { return P->nnz; }
int64_t orc_ngp(const orc_problem* P) { return P->ngp; }
void orc_get_decomp(const orc_problem* P, int* mnp) { mnp[0] = P->m; mnp[1] = P->n; mnp[2] = P->p; }
double* orc_u(orc_problem* P) { return P->u; }
double* orc_b(orc_problem* P) { return P->b; }
double* orc_du(orc_problem* P) { return P->du; }
double* orc_A_values(orc_problem* P) { return P->val; }
double* orc_strain(orc_problem* P) { return P->eps; }
double* orc_stress(orc_problem* P) { return P->sig; }

/* get_displacement src/bcs.c:52-58, with the missing `return` restored (Appendix A.3) */
double orc_get_displacement(const orc_problem* P, int time_s) {
  double time = time_s * P->o.dt;
  return U_MAX * (time / P->o.final_time);
}

/* apply_bc_on_u -> VecSetValues(INSERT) of every rank's list (src/bcs.c:29-146) */
void orc_apply_bc_u(orc_problem* P, double U) {
  for (int r = 0; r < P->nranks; r++) {
    int64_t nb = orc_rank_dirichlet(P, r, NULL, 0);
    int64_t* ix = malloc((nb + 1) * sizeof(int64_t));
    double* v = malloc((nb + 1) * sizeof(double));
    orc_rank_dirichlet(P, r, ix, nb);
    int64_t nv = rank_dirichlet_values(P, r, U, v);
    for (int64_t q = 0; q < nv; q++)
      if (ix[q] >= 0) P->u[ix[q]] = v[q];
    free(ix);
    free(v);
  }
}

/* set_strains src/assembly.c:25-66 (per rank, elements in DMDAGetElements order) */
void orc_set_strains(orc_problem* P) {
#pragma omp parallel for schedule(dynamic, 1)
  for (int r = 0; r < P->nranks; r++) {
    int64_t c[12];
    orc_rank_corners(P, r, c);
    int64_t ne = P->ne[r];
    int32_t* conn = malloc((ne * 8 + 1) * sizeof(int32_t));
    orc_rank_elements(P, r, conn);
    for (int64_t ie = 0; ie < ne; ++ie) {
      double u_e[NPE * DIM];
      for (int nn = 0; nn < NPE; ++nn) {
        int64_t g = ltog_node(P, c, conn[ie * NPE + nn]);
        for (int d = 0; d < DIM; ++d) u_e[nn * DIM + d] = P->u[3 * g + d];
      }
      for (int gp = 0; gp < NGP; ++gp) {
        double strain[NVOI];
        memset(strain, 0, sizeof(strain));
        for (int i = 0; i < NVOI; ++i)
          for (int j = 0; j < NPE * DIM; ++j) strain[i] += P->Btab[gp][i][j] * u_e[j];
        int64_t gpi = P->gp_off[r] + ie * NGP + gp;
        memcpy(P->eps + gpi * NVOI, strain, sizeof(strain));
      }
    }
    free(conn);
  }
}

/* Gauss-point constitutive law behind micropp_C_homogenize (src/main.c:62).
   law 0: isotropic elastic, sigma = C eps, ctan = C.
   law 1: small-strain J2 plasticity with linear isotropic hardening (MicroPP material type 1
   with parameters E, nu, Sy, Ka; src/init.c:196-201), radial return + consistent tangent.
   Voigt xx,yy,zz,xy,xz,yz; strains engineering shear; history = plastic strain (tensor
   components) + accumulated plastic strain alpha.  Shared by the GPU kernel (same order of
   operations) — MicroPP itself is not available: parity vs MicroPP is unpinned. */
void orc_j2_point(double E, double nu, double Sy, double Ka, const double* e, const double* hold,
                  double* s, double* C, double* hnew, double* ftrial) {
  const double G = E / (2. * (1. + nu));
  const double K = E / (3. * (1. - 2. * nu));
  const double tr = e[0] + e[1] + e[2];
  double dev[6];
  for (int i = 0; i < 3; i++) dev[i] = e[i] - tr / 3.;
  for (int i = 3; i < 6; i++) dev[i] = e[i] / 2.;
  double st[6];
  for (int i = 0; i < 6; i++) st[i] = 2. * G * (dev[i] - hold[i]);
  double nrm2 = st[0] * st[0] + st[1] * st[1] + st[2] * st[2];
  nrm2 = nrm2 + 2. * (st[3] * st[3] + st[4] * st[4] + st[5] * st[5]);
  const double snorm = sqrt(nrm2);
  const double alpha = hold[6];
  const double f = snorm - sqrt(2. / 3.) * (Sy + Ka * alpha);
  *ftrial = f;
  const double lam = K - 2. * G / 3.;
  for (int k = 0; k < 36; k++) C[k] = 0.;
  for (int a = 0; a < 3; a++)
    for (int b = 0; b < 3; b++) C[a * 6 + b] = lam + (a == b ? 2. * G : 0.);
  for (int a = 3; a < 6; a++) C[a * 6 + a] = G;
  if (f <= 0.) {
    for (int i = 0; i < 3; i++) s[i] = K * tr + st[i];
    for (int i = 3; i < 6; i++) s[i] = st[i];
    for (int i = 0; i < 7; i++) hnew[i] = hold[i];
    return;
  }
  const double dg = f / (2. * G + 2. / 3. * Ka);
  double n[6];
  for (int i = 0; i < 6; i++) n[i] = st[i] / snorm;
  for (int i = 0; i < 3; i++) s[i] = K * tr + (st[i] - 2. * G * dg * n[i]);
  for (int i = 3; i < 6; i++) s[i] = st[i] - 2. * G * dg * n[i];
  for (int i = 0; i < 6; i++) hnew[i] = hold[i] + dg * n[i];
  hnew[6] = alpha + sqrt(2. / 3.) * dg;
  const double theta = 1. - 2. * G * dg / snorm;
  const double thetab = 1. / (1. + Ka / (3. * G)) - (1. - theta);
  for (int a = 0; a < 3; a++)
    for (int b = 0; b < 3; b++) C[a * 6 + b] = K + 2. * G * theta * ((a == b ? 1. : 0.) - 1. / 3.);
  for (int a = 3; a < 6; a++) C[a * 6 + a] = G * theta;
  for (int a = 0; a < 6; a++)
    for (int b = 0; b < 6; b++) C[a * 6 + b] = C[a * 6 + b] - 2. * G * thetab * n[a] * n[b];
}

void orc_homogenize(orc_problem* P) {
#pragma omp parallel for schedule(static)
  for (int64_t g = 0; g < P->ngp; g++) {
    const double* e = P->eps + g * NVOI;
    double* s = P->sig + g * NVOI;
    if (P->o.law == 1) {
      orc_j2_point(P->o.E, P->o.nu, P->o.Sy, P->o.Ka, e, P->hist_old + 7 * g, s, P->ctan + 36 * g,
                   P->hist_new + 7 * g, P->ftrial + g);
      continue;
    }
    for (int k = 0; k < NVOI; k++) {
      double acc = 0.;
      for (int l = 0; l < NVOI; l++) acc += P->C[k * NVOI + l] * e[l];
      s[k] = acc;
    }
    memcpy(P->ctan + 36 * g, P->C, 36 * sizeof(double));
    P->ftrial[g] = 0.;
  }
}

void orc_update_vars(orc_problem* P) {
  memcpy(P->hist_old, P->hist_new, P->ngp * 7 * sizeof(double));
}

int64_t orc_nonlinear_gps(const orc_problem* P, double* fmax) {
  int64_t n = 0;
  double m = -1e300;
  for (int64_t g = 0; g < P->ngp; g++) {
    if (P->ftrial[g] > 0.) n++;
    if (P->ftrial[g] > m) m = P->ftrial[g];
  }
  if (fmax) *fmax = m;
  return n;
}

double* orc_ctan(orc_problem* P) { return P->ctan; }

/* micropp_C_get_non_linear_gps() of one emulated rank (its GP range), the per-rank column
   of gauss_evolution.dat (src/util.c:69-87) */
int64_t orc_rank_nonlinear_gps(const orc_problem* P, int r) {
  int64_t n = 0;
  for (int64_t g = P->gp_off[r]; g < P->gp_off[r] + P->ne[r] * NGP; g++) n += P->ftrial[g] > 0.;
  return n;
}

/* calc_force src/forces.c:25-50: per rank calc_force_circle (:115-166) or calc_force_bending
   (:58-106) over the rank's own elements and GP stresses, then MPI_Reduce(SUM) — emulated in
   rank order.  Quirks kept: the circle test uses the GHOST corners si, sk, sj and the owned
   ny (:130-133), so only ranks with no lower y ghost (ys == 0) that also reach NY contribute
   (with more than one rank in y the force is 0); stress_ave is the plain sum over the 8 GPs
   (:145-154). */
double orc_calc_force(const orc_problem* P) {
  double force = 0.0;
  for (int r = 0; r < P->nranks; r++) {
    int64_t c[12], lo[3], cnt[3];
    orc_rank_corners(P, r, c);
    rank_elem_range(P, r, lo, cnt);
    const int64_t nex = cnt[0], ney = cnt[1], nez = cnt[2];
    const double* sig = P->sig + P->gp_off[r] * NVOI;
    double mpi_force = 0.0;
    double stress_ave[NVOI];
    if (P->o.bc_type == 0) { /* BC_BENDING */
      if (c[0] + c[3] == P->o.NX) {
        for (int64_t ey = 0; ey < ney; ++ey)
          for (int64_t ez = 0; ez < nez; ++ez) {
            const int64_t e = (nex - 1) + ey * nex + ez * (nex * ney);
            memset(stress_ave, 0, sizeof(stress_ave));
            for (int gp = 0; gp < NGP; ++gp)
              for (int i = 0; i < NVOI; ++i) stress_ave[i] += sig[(e * NGP + gp) * NVOI + i];
            mpi_force += stress_ave[3] * P->dy * P->dz;
          }
      }
    } else { /* BC_CIRCLE */
      const int64_t si = c[6], sj = c[7], sk = c[8];
      if (sj + c[4] == P->o.NY) {
        for (int64_t ex = 0; ex < nex; ++ex)
          for (int64_t ez = 0; ez < nez; ++ez) {
            const double x = P->o.lx / 2. - ((si + ex) * P->dx + P->dx / 2.);
            const double z = P->o.lz / 2. - ((sk + ez) * P->dz + P->dz / 2.);
            if ((x * x + z * z) < 1 * (P->o.rad * P->o.rad)) {
              const int64_t e = ex + (ney - 1) * nex + ez * (nex * ney);
              memset(stress_ave, 0, sizeof(stress_ave));
              for (int gp = 0; gp < NGP; ++gp)
                for (int i = 0; i < NVOI; ++i) stress_ave[i] += sig[(e * NGP + gp) * NVOI + i];
              mpi_force += stress_ave[1] * P->dx * P->dz;
            }
          }
      }
    }
    force += mpi_force;
  }
  return force;
}

/* assembly_res src/assembly.c:120-176 with DMLocalToGlobal(ADD) emulated as
   owned part first, then remote ghost contributions by source rank */
void orc_assembly_res(orc_problem* P) {
  memset(P->b, 0, P->ndofs * sizeof(double));
  double** bloc = malloc(P->nranks * sizeof(double*));
#pragma omp parallel for schedule(dynamic, 1)
  for (int r = 0; r < P->nranks; r++) {
    int64_t c[12];
    orc_rank_corners(P, r, c);
    int64_t nl = c[9] * c[10] * c[11];
    bloc[r] = calloc(nl * 3, sizeof(double));
    int64_t ne = P->ne[r];
    int32_t* conn = malloc((ne * 8 + 1) * sizeof(int32_t));
    orc_rank_elements(P, r, conn);
    for (int64_t ie = 0; ie < ne; ++ie) {
      double be[NPE * DIM];
      memset(be, 0, sizeof(be));
      for (int gp = 0; gp < NGP; ++gp) {
        const double* stress = P->sig + (P->gp_off[r] + ie * NGP + gp) * NVOI;
        for (int i = 0; i < NPE * DIM; ++i)
          for (int j = 0; j < NVOI; ++j) be[i] += P->Btab[gp][j][i] * stress[j] * P->wg;
      }
      for (int nn = 0; nn < NPE; ++nn)
        for (int d = 0; d < DIM; ++d) bloc[r][conn[ie * NPE + nn] * DIM + d] += be[nn * DIM + d];
    }
    free(conn);
  }
  /* owned entries */
#pragma omp parallel for schedule(dynamic, 1)
  for (int r = 0; r < P->nranks; r++) {
    int64_t c[12];
    orc_rank_corners(P, r, c);
    int64_t nl = c[9] * c[10] * c[11];
    for (int64_t l = 0; l < nl; l++) {
      int64_t g = ltog_node(P, c, l);
      if (rank_of_dof(P, 3 * g) != r) continue;
      for (int d = 0; d < 3; d++) P->b[3 * g + d] += bloc[r][3 * l + d];
    }
  }
  /* ghost entries, by destination then source rank */
#pragma omp parallel for schedule(dynamic, 1)
  for (int dst = 0; dst < P->nranks; dst++)
    for (int r = 0; r < P->nranks; r++) {
      if (r == dst) continue;
      int64_t c[12];
      orc_rank_corners(P, r, c);
      int64_t nl = c[9] * c[10] * c[11];
      for (int64_t l = 0; l < nl; l++) {
        int64_t g = ltog_node(P, c, l);
        if (rank_of_dof(P, 3 * g) != dst) continue;
        for (int d = 0; d < 3; d++) P->b[3 * g + d] += bloc[r][3 * l + d];
      }
    }
  for (int r = 0; r < P->nranks; r++) free(bloc[r]);
  free(bloc);
  /* apply_bc_on_res src/bcs.c:350-362, then VecScale(b,-1) src/assembly.c:173 */
  for (int64_t q = 0; q < P->ndir; q++) P->b[P->dir[q]] = 0.;
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < P->ndofs; i++) P->b[i] = P->b[i] * -1.;
}

/* VecNorm(NORM_2) — per-rank partial sums, summed in rank order [ext] */
double orc_norm2(const orc_problem* P, const double* v) {
  double* part = malloc(P->nranks * sizeof(double));
#pragma omp parallel for schedule(static)
  for (int r = 0; r < P->nranks; r++) {
    double s = 0.;
    for (int64_t i = 3 * P->node_off[r]; i < 3 * P->node_off[r + 1]; i++) s += v[i] * v[i];
    part[r] = s;
  }
  double tot = 0.;
  for (int r = 0; r < P->nranks; r++) tot += part[r];
  free(part);
  return sqrt(tot);
}

static double dot(const orc_problem* P, const double* x, const double* y) {
  double* part = malloc(P->nranks * sizeof(double));
#pragma omp parallel for schedule(static)
  for (int r = 0; r < P->nranks; r++) {
    double s = 0.;
    for (int64_t i = 3 * P->node_off[r]; i < 3 * P->node_off[r + 1]; i++) s += x[i] * y[i];
    part[r] = s;
  }
  double tot = 0.;
  for (int r = 0; r < P->nranks; r++) tot += part[r];
  free(part);
  return tot;
}

/* assembly_jac src/assembly.c:69-117: naive 4-nest per element (:94-99), MatSetValuesLocal
   ADD (:106-107) with off-rank rows stashed and added at MatAssemblyEnd [ext], then
   apply_bc_on_jac = MatZeroRowsColumns(diag = 1) src/bcs.c:341-347 */
void orc_assembly_jac(orc_problem* P) {
  memset(P->val, 0, P->nnz * sizeof(double));
  int64_t* ns = calloc(P->nranks * P->nranks, sizeof(int64_t));
  int64_t* cap = calloc(P->nranks * P->nranks, sizeof(int64_t));
  stash_entry** st = calloc(P->nranks * P->nranks, sizeof(stash_entry*));
#pragma omp parallel for schedule(dynamic, 1)
  for (int r = 0; r < P->nranks; r++) {
    double Ae[NPE * DIM * NPE * DIM];
    int64_t c[12];
    orc_rank_corners(P, r, c);
    int64_t ne = P->ne[r];
    int32_t* conn = malloc((ne * 8 + 1) * sizeof(int32_t));
    orc_rank_elements(P, r, conn);
    for (int64_t ie = 0; ie < ne; ++ie) {
      memset(Ae, 0, sizeof(Ae));
      for (int gp = 0; gp < NGP; ++gp) {
        const double* ctan = P->ctan + 36 * (P->gp_off[r] + ie * NGP + gp); /* micropp_C_get_ctan3 */
        double(*B)[NPE * DIM] = P->Btab[gp];
        for (int i = 0; i < NPE * DIM; ++i)
          for (int j = 0; j < NPE * DIM; ++j)
            for (int k = 0; k < NVOI; ++k)
              for (int l = 0; l < NVOI; ++l) Ae[NPE * DIM * i + j] += B[k][i] * ctan[k * NVOI + l] * B[l][j] * P->wg;
      }
      int64_t ix[NPE * DIM];
      for (int nn = 0; nn < NPE; ++nn)
        for (int d = 0; d < DIM; ++d) ix[nn * DIM + d] = 3 * ltog_node(P, c, conn[ie * NPE + nn]) + d;
      for (int i = 0; i < NPE * DIM; i++) {
        int owner = rank_of_dof(P, ix[i]);
        for (int j = 0; j < NPE * DIM; j++) {
          if (owner == r) {
            P->val[csr_find(P, ix[i], ix[j])] += Ae[NPE * DIM * i + j];
          } else {
            int q = owner * P->nranks + r;
            if (ns[q] == cap[q]) {
              cap[q] = cap[q] ? 2 * cap[q] : 1024;
              st[q] = realloc(st[q], cap[q] * sizeof(stash_entry));
            }
            st[q][ns[q]++] = (stash_entry){ix[i], ix[j], Ae[NPE * DIM * i + j]};
          }
        }
      }
    }
    free(conn);
  }
#pragma omp parallel for schedule(dynamic, 1)
  for (int dst = 0; dst < P->nranks; dst++)
    for (int src = 0; src < P->nranks; src++) {
      int q = dst * P->nranks + src;
      for (int64_t e = 0; e < ns[q]; e++) P->val[csr_find(P, st[q][e].row, st[q][e].col)] += st[q][e].v;
      free(st[q]);
    }
  free(st); free(ns); free(cap);
  /* MatZeroRowsColumns(A, n, rows, 1.0, NULL, NULL) over the union of rank lists */
#pragma omp parallel for schedule(static)
  for (int64_t row = 0; row < P->ndofs; row++) {
    int rowD = is_dirichlet(P, row);
    for (int64_t q = P->rowptr[row]; q < P->rowptr[row + 1]; q++) {
      int64_t col = P->colidx[q];
      if (rowD) P->val[q] = (col == row) ? 1.0 : 0.0;
      else if (is_dirichlet(P, col)) P->val[q] = 0.0;
    }
  }
}

/* One row's part of MatMult, sum0 + the terms of its columns col in [lo, hi) or outside it
   (own = 0), in ascending column order.
   ORC_SPMV_INODE — MatMult_SeqAIJ_Inode / MatMultAdd_SeqAIJ_Inode [ext] (PETSc
   src/mat/impls/aij/seq/inode.c, the kernel a MATAIJ with identical consecutive row patterns
   runs: MatSeqAIJCheckInode groups the 3 rows of a DMDA node, dof 3, into one inode, and
   KSPSolve's MatMult dispatches to it).  Its unrolled loop adds the row's terms in column
   pairs, `sum += v[0]*x[i1] + v[1]*x[i2]`, then an odd last term, `sum += v[0]*x[i1]`; the x86
   build has no FMA, so every product and sum is rounded as written:
     sum = sum0 + (t0 + t1) + (t2 + t3) + ... [+ t_last],   t = a * x.
   The pairs run over the row's stored columns, so a column clipped by the DMDA stencil at the
   domain boundary shifts the pairing of the columns after it, and the zeroed (MatZeroRowsColumns)
   entries, which stay in the pattern, take part.
   ORC_SPMV_SEQAIJ — MatMult_SeqAIJ's plain loop, sum += a * x term by term. */
static double row_part(const orc_problem* P, int64_t row, int64_t lo, int64_t hi, int own, double sum0,
                       const double* x, int order) {
  double sum = sum0, pend = 0.;
  int have = 0;
  for (int64_t q = P->rowptr[row]; q < P->rowptr[row + 1]; q++) {
    const int64_t col = P->colidx[q];
    if ((col >= lo && col < hi) != own) continue;
    const double t = P->val[q] * x[col];
    if (order == ORC_SPMV_SEQAIJ) {
      sum += t;
    } else if (!have) {
      pend = t;
      have = 1;
    } else {
      sum += pend + t;
      have = 0;
    }
  }
  if (have) sum += pend;
  return sum;
}

/* MatMult (KSPSolve's, src/assembly.c:185): one rank = the SeqAIJ kernel above over the row;
   several ranks = MatMult_MPIAIJ, the diagonal (owned-column) block A first, then MatMultAdd of
   the off-diagonal block B (its columns, the compressed ghosts, in ascending global order)
   starting from that sum [ext].  MatAssemblyEnd_MPIAIJ turns inodes off for B
   (MatSetOption(aij->B, MAT_USE_INODES, PETSC_FALSE) before B's assembly [ext]), so B's part
   always runs MatMultAdd_SeqAIJ's plain loop, sum += a * x term by term; A keeps
   the order asked for. */
void orc_spmv_order(const orc_problem* P, const double* x, double* y, int order) {
#pragma omp parallel for schedule(static)
  for (int r = 0; r < P->nranks; r++) {
    int64_t c0 = 3 * P->node_off[r], c1 = 3 * P->node_off[r + 1];
    for (int64_t row = c0; row < c1; row++) {
      double sum = row_part(P, row, c0, c1, 1, 0., x, order);
      if (P->nranks > 1) sum = row_part(P, row, c0, c1, 0, sum, x, ORC_SPMV_SEQAIJ);
      y[row] = sum;
    }
  }
}

void orc_spmv(const orc_problem* P, const double* x, double* y) { orc_spmv_order(P, x, y, P->spmv_order); }

/* KSPConvergedDefault [ext] */
static int converged_default(double rnorm, double ttol, double abstol, double divtol, double rnorm0) {
  if (isnan(rnorm) || isinf(rnorm)) return ORC_KSP_DIVERGED_NANORINF;
  if (rnorm <= ttol) return rnorm < abstol ? ORC_KSP_CONVERGED_ATOL : ORC_KSP_CONVERGED_RTOL;
  if (rnorm >= divtol * rnorm0) return ORC_KSP_DIVERGED_DTOL;
  return 0;
}

/* KSPSolve_CG, KSP_NORM_PRECONDITIONED, zero initial guess, PCJacobi [ext] */
int orc_solve(orc_problem* P, int* its_out, double* rnorm_out, int* reason_out, double* hist) {
  const orc_opts* o = &P->o;
  int64_t N = P->ndofs;
  double *X = P->du, *R = P->r, *Z = P->z, *Pv = P->pp, *W = P->w;
  /* PCSetUp_Jacobi: diag, VecReciprocal (zeros untouched), then zeros -> 1 */
  #pragma omp parallel for schedule(static)
  for (int64_t row = 0; row < N; row++) {
    double d = P->val[csr_find(P, row, row)];
    if (d != 0.0) d = 1.0 / d;
    if (d == 0.0) d = 1.0;
    P->dinv[row] = d;
  }
  double dp, beta = 0., betaold = 0., dpi = 0., dpiold, a, b;
  int reason = 0, its = 0, i;
  memset(X, 0, N * sizeof(double));                       /* guess zero */
  memcpy(R, P->b, N * sizeof(double));                    /* r <- b */
  #pragma omp parallel for schedule(static)
  for (int64_t q = 0; q < N; q++) Z[q] = R[q] * P->dinv[q]; /* z <- Br */
  dp = orc_norm2(P, Z);
  if (hist) hist[0] = dp;
  double ttol = fmax(o->rtol * dp, o->abstol), rnorm0 = dp;
  reason = converged_default(dp, ttol, o->abstol, o->dtol, rnorm0);
  double rnorm = dp;
  if (reason) goto done;
  beta = dot(P, Z, R);
  i = 0;
  do {
    its = i + 1;
    if (beta == 0.0) {
      reason = ORC_KSP_CONVERGED_ATOL;
      break;
    } else if ((i > 0) && (beta * betaold < 0.0)) {
      reason = ORC_KSP_DIVERGED_INDEFINITE_PC;
      break;
    }
    if (!i) {
      memcpy(Pv, Z, N * sizeof(double));
      b = 0.0;
    } else {
      b = beta / betaold;
      #pragma omp parallel for schedule(static)
      for (int64_t q = 0; q < N; q++) Pv[q] = Z[q] + b * Pv[q]; /* VecAYPX */
    }
    dpiold = dpi;
    orc_spmv(P, Pv, W);
    dpi = dot(P, Pv, W);
    betaold = beta;
    if ((dpi == 0.0) || ((i > 0) && (dpi * dpiold <= 0.0))) {
      reason = ORC_KSP_DIVERGED_INDEFINITE_MAT;
      break;
    }
    a = beta / dpi;
    #pragma omp parallel for schedule(static)
    for (int64_t q = 0; q < N; q++) X[q] = X[q] + a * Pv[q];
    #pragma omp parallel for schedule(static)
    for (int64_t q = 0; q < N; q++) R[q] = R[q] + (-a) * W[q];
    #pragma omp parallel for schedule(static)
    for (int64_t q = 0; q < N; q++) Z[q] = R[q] * P->dinv[q];
    dp = orc_norm2(P, Z);
    rnorm = dp;
    if (hist) hist[i + 1] = dp;
    reason = converged_default(dp, ttol, o->abstol, o->dtol, rnorm0);
    if (reason) break;
    beta = dot(P, Z, R);
    i++;
  } while (i < o->maxits);
  if (!reason && i >= o->maxits) reason = ORC_KSP_DIVERGED_ITS;
done:
  if (its_out) *its_out = its;
  if (rnorm_out) *rnorm_out = rnorm;
  if (reason_out) *reason_out = reason;
  return 0;
}

/* VecAXPY(u, 1., du) src/main.c:79 */
void orc_update_u(orc_problem* P) {
  for (int64_t q = 0; q < P->ndofs; q++) P->u[q] = P->u[q] + 1. * P->du[q];
}

static double now_s(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + 1e-9 * t.tv_nsec;
}

/* write_pvtu src/output.c:25-267 for every emulated rank: "<prefix>.pvtu" + one
   "<prefix>-subdo-<r>.vtu" piece per rank (ghosted box points, the rank's DMDAGetElements
   elements, ghosted u, cell data).  micropp_C_get_sigma_cost3 (:180-187) has no counterpart
   without a micro solver: cost = 0.  micropp_C_is_non_linear = f_trial > 0. */
int orc_write_vtu(const orc_problem* P, const char* prefix) {
  char name[1024];
  snprintf(name, sizeof(name), "%s.pvtu", prefix);
  FILE* fp = fopen(name, "w");
  if (!fp) return 1;
  fprintf(fp,
          "<?xml version=\"1.0\"?>\n"
          "<VTKFile type=\"PUnstructuredGrid\" version=\"0.1\" byte_order=\"LittleEndian\">\n"
          "<PUnstructuredGrid GhostLevel=\"0\">\n"
          "<PPoints>\n"
          "  <PDataArray type=\"Float64\" Name=\"Position\"   NumberOfComponents=\"3\"/>\n"
          "</PPoints>\n"
          "<PCells>\n"
          "  <PDataArray type=\"Int32\" Name=\"connectivity\" NumberOfComponents=\"1\"/>\n"
          "  <PDataArray type=\"Int32\" Name=\"offsets\"      NumberOfComponents=\"1\"/>\n"
          "  <PDataArray type=\"UInt8\" Name=\"types\"        NumberOfComponents=\"1\"/>\n"
          "</PCells>\n"
          "<PPointData Vectors=\"displ\">\n"
          "  <PDataArray type=\"Float64\" Name=\"displ\"      NumberOfComponents=\"3\" />\n"
          "</PPointData>\n"
          "<PCellData>\n"
          "  <PDataArray type=\"Int32\"   Name=\"part\"       NumberOfComponents=\"1\"/>\n"
          "  <PDataArray type=\"Float64\" Name=\"cost\"       NumberOfComponents=\"1\"/>\n"
          "  <PDataArray type=\"Int32\"   Name=\"non-linear\" NumberOfComponents=\"1\"/>\n"
          "<PDataArray type=\"Float64\" Name=\"strain\"       NumberOfComponents=\"6\"/>\n"
          "<PDataArray type=\"Float64\" Name=\"stress\"       NumberOfComponents=\"6\"/>\n"
          "</PCellData>\n");
  for (int r = 0; r < P->nranks; ++r) fprintf(fp, "  <Piece Source=\"%s-subdo-%d.vtu\"/>\n", prefix, r);
  fprintf(fp, "</PUnstructuredGrid>\n</VTKFile>\n");
  fclose(fp);
  for (int r = 0; r < P->nranks; ++r) {
    int64_t c[12];
    orc_rank_corners(P, r, c);
    const int64_t si = c[6], sj = c[7], sk = c[8], nx = c[9], ny = c[10], nz = c[11], N = nx * ny * nz;
    const int64_t nelem = P->ne[r];
    int32_t* eix = malloc((nelem * NPE + 1) * sizeof(int32_t));
    orc_rank_elements(P, r, eix);
    double* u_arr = malloc((N * DIM + 1) * sizeof(double));
    for (int64_t l = 0; l < N; ++l)
      for (int d = 0; d < DIM; ++d) u_arr[l * DIM + d] = P->u[ltog_node(P, c, l) * DIM + d];
    snprintf(name, sizeof(name), "%s-subdo-%d.vtu", prefix, r);
    fp = fopen(name, "w");
    if (!fp) return 1;
    fprintf(fp,
            "<?xml version=\"1.0\"?>\n"
            "<VTKFile type=\"UnstructuredGrid\" version=\"0.1\" byte_order=\"LittleEndian\">\n"
            "<UnstructuredGrid>\n"
            "<Piece NumberOfPoints=\"%d\" NumberOfCells=\"%d\">\n"
            "<Points>\n",
            (int)N, (int)nelem);
    fprintf(fp, "<DataArray type=\"Float64\" Name=\"Position\" NumberOfComponents=\"3\" format=\"ascii\">\n");
    for (int64_t k = sk; k < sk + nz; ++k)
      for (int64_t j = sj; j < sj + ny; ++j)
        for (int64_t i = si; i < si + nx; ++i) fprintf(fp, "%01.6e\t%01.6e\t%01.6e\n", i * P->dx, j * P->dy, k * P->dz);
    fprintf(fp, "</DataArray>\n</Points>\n<Cells>\n");
    fprintf(fp, "<DataArray type=\"Int32\" Name=\"connectivity\" NumberOfComponents=\"1\" format=\"ascii\">\n");
    for (int64_t e = 0; e < nelem; ++e) {
      for (int n = 0; n < NPE; ++n) fprintf(fp, "%-6d\t", eix[e * NPE + n]);
      fprintf(fp, "\n");
    }
    fprintf(fp, "</DataArray>\n");
    fprintf(fp, "<DataArray type=\"Int32\" Name=\"offsets\" NumberOfComponents=\"1\" format=\"ascii\">\n");
    for (int64_t e = 1; e < nelem + 1; ++e) fprintf(fp, "%d\t", (int)(e * NPE));
    fprintf(fp, "\n</DataArray>\n");
    fprintf(fp, "<DataArray type=\"UInt8\"  Name=\"types\" NumberOfComponents=\"1\" format=\"ascii\">\n");
    for (int64_t e = 0; e < nelem; ++e) fprintf(fp, "12\t");
    fprintf(fp, "\n</DataArray>\n</Cells>\n<PointData Vectors=\"displ\">\n");
    fprintf(fp, "<DataArray type=\"Float64\" Name=\"displ\" NumberOfComponents=\"3\" format=\"ascii\" >\n");
    for (int64_t n = 0; n < N; ++n)
      fprintf(fp, "%01.6e\t%01.6e\t%01.6e\n", u_arr[n * DIM + 0], u_arr[n * DIM + 1], u_arr[n * DIM + 2]);
    fprintf(fp, "</DataArray>\n</PointData>\n<CellData>\n");
    fprintf(fp, "<DataArray type=\"Int32\" Name=\"part\" NumberOfComponents=\"1\" format=\"ascii\">\n");
    for (int64_t e = 0; e < nelem; ++e) fprintf(fp, "%d\t", r);
    fprintf(fp, "\n</DataArray>\n");
    fprintf(fp, "<DataArray type=\"Float64\" Name=\"cost\" NumberOfComponents=\"1\" format=\"ascii\">\n");
    for (int64_t e = 0; e < nelem; ++e) fprintf(fp, "%lf\t", 0. / NGP);
    fprintf(fp, "\n</DataArray>\n");
    fprintf(fp, "<DataArray type=\"Int32\" Name=\"non-linear\" NumberOfComponents=\"1\" format=\"ascii\">\n");
    const double* ft = P->ftrial + P->gp_off[r];
    for (int64_t e = 0; e < nelem; ++e) {
      int non_linear = 0;
      for (int gp = 0; gp < NGP; ++gp) non_linear += ft[e * NPE + gp] > 0.;
      fprintf(fp, "%d\t", non_linear);
    }
    fprintf(fp, "\n</DataArray>\n");
    fprintf(fp, "<DataArray type=\"Float64\" Name=\"strain\" NumberOfComponents=\"6\" format=\"ascii\">");
    for (int64_t e = 0; e < nelem; ++e) {
      double u_e[NPE * DIM], strain[NVOI] = {0.}, strain_gp[NVOI];
      for (int n = 0; n < NPE; ++n)
        for (int i = 0; i < DIM; ++i) u_e[n * DIM + i] = u_arr[eix[e * NPE + n] * DIM + i];
      for (int gp = 0; gp < NGP; ++gp) {
        memset(strain_gp, 0, sizeof(strain_gp));
        for (int i = 0; i < NVOI; ++i)
          for (int j = 0; j < NPE * DIM; ++j) strain_gp[i] += P->Btab[gp][i][j] * u_e[j];
        for (int i = 0; i < NVOI; ++i) strain[i] += strain_gp[i] * P->wg;
      }
      for (int i = 0; i < NVOI; ++i) fprintf(fp, "%e\t", strain[i]);
    }
    fprintf(fp, "\n</DataArray>\n");
    fprintf(fp, "<DataArray type=\"Float64\" Name=\"stress\" NumberOfComponents=\"6\" format=\"ascii\">");
    const double* sg = P->sig + P->gp_off[r] * NVOI;
    for (int64_t e = 0; e < nelem; ++e) {
      double stress[NVOI] = {0.};
      for (int gp = 0; gp < NGP; ++gp)
        for (int i = 0; i < NVOI; ++i) stress[i] += sg[(e * NPE + gp) * NVOI + i] * P->wg;
      for (int i = 0; i < NVOI; ++i) fprintf(fp, "%e\t", stress[i]);
    }
    fprintf(fp, "\n</DataArray>\n</CellData>\n</Piece>\n</UnstructuredGrid>\n</VTKFile>\n");
    fclose(fp);
    free(eix);
    free(u_arr);
  }
  return 0;
}

/* src/main.c:49-109 with the per-time-step post-processing of :86-97: non-linear GP counts
   (gauss_evolution.dat, src/util.c:69-87), reaction force (src/forces.c:25-50), f_trial_max
   (src/util.c:94-102) and the info.dat row (:96-97; the int64 count is printed with %d). */
int orc_run_files(orc_problem* P, const char* log_path, const char* info_path, const char* gauss_path,
                  double* t_newton_solve_s) {
  FILE* f = log_path ? fopen(log_path, "w") : NULL;
  FILE* fi = info_path ? fopen(info_path, "w") : NULL;
  FILE* fg = gauss_path ? fopen(gauss_path, "w") : NULL;
  double norm = 0., norm_0 = 0.;
  double t_first = -1.;
  for (int time_s = 0; time_s < P->o.ts; ++time_s) {
    if (f) fprintf(f, "\n\nTime Step = %d\n", time_s);
    double U = orc_get_displacement(P, time_s);
    orc_apply_bc_u(P, U);
    int newton_it = 0;
    while (newton_it < P->o.newton_max_its) {
      double t0 = now_s();
      if (f) fprintf(f, "\nNewton Iteration = %d\n", newton_it);
      orc_set_strains(P);
      orc_homogenize(P);
      orc_assembly_res(P);
      norm = orc_norm2(P, P->b);
      if (f) fprintf(f, "|RES| = %e\n", norm);
      if (newton_it == 0) norm_0 = norm;
      if (norm < P->o.newton_min_tol || norm < norm_0 * P->o.newton_rel_tol) break;
      orc_assembly_jac(P);
      int its, reason;
      double rn;
      orc_solve(P, &its, &rn, &reason, NULL);
      if (f) fprintf(f, "KSP : |Ax - b|/|Ax| = %e\tIts = %d\n", rn, its);
      orc_update_u(P);
      if (t_first < 0) t_first = now_s() - t0;
      newton_it++;
    }
    orc_update_vars(P);
    if (fg) fprintf(fg, "%d\t", time_s);
    int64_t nl = 0;
    for (int r = 0; r < P->nranks; r++) {
      const int64_t q = orc_rank_nonlinear_gps(P, r);
      if (fg) fprintf(fg, "%ld\t", (long)q);
      nl += q;
    }
    if (fg) fprintf(fg, "\n");
    if (f) fprintf(f, "Non-Linear Gauss points : %ld\n", (long)nl);
    const double force = orc_calc_force(P);
    double ftm = 0.;
    orc_nonlinear_gps(P, &ftm);
    if (f) fprintf(f, "F_trial_max             : %e\n", ftm);
    if (fi) fprintf(fi, "%d\t%e\t%e\t%e\t%e\t%d\n", time_s, time_s * P->o.dt, U, force, ftm, (int)nl);
  }
  if (f) fclose(f);
  if (fi) fclose(fi);
  if (fg) fclose(fg);
  if (t_newton_solve_s) *t_newton_solve_s = t_first;
  return 0;
}

int orc_run(orc_problem* P, const char* log_path, double* t_newton_solve_s) {
  return orc_run_files(P, log_path, NULL, NULL, t_newton_solve_s);
}

/* DMDA natural -> PETSc node numbering for any M,N,P >= 1 (used to pin the known answer of
   tests/test_dm_1.c:5-19, a 2-D 5x2 DMDA on 2 ranks = M=5,N=2,P=1) */
int orc_petsc_numbering(int64_t M, int64_t N, int64_t P, int size, int m, int n, int p, int64_t* out) {
  if (orc_dmda_decide(M, N, P, size, &m, &n, &p)) return 1;
  int64_t dims[3] = {M, N, P};
  int procs[3] = {m, n, p};
  int64_t *w[3], *s[3];
  for (int d = 0; d < 3; d++) {
    w[d] = malloc(procs[d] * sizeof(int64_t));
    s[d] = malloc(procs[d] * sizeof(int64_t));
    int64_t acc = 0;
    for (int q = 0; q < procs[d]; q++) {
      w[d][q] = dims[d] / procs[d] + ((dims[d] % procs[d]) > q);
      s[d][q] = acc;
      acc += w[d][q];
    }
  }
  int64_t* off = malloc((size + 1) * sizeof(int64_t));
  off[0] = 0;
  for (int r = 0; r < size; r++) {
    int a = r % m, b = (r % (m * n)) / m, c = r / (m * n);
    off[r + 1] = off[r] + w[0][a] * w[1][b] * w[2][c];
  }
  for (int64_t k = 0; k < P; k++)
    for (int64_t j = 0; j < N; j++)
      for (int64_t i = 0; i < M; i++) {
        int a = 0, b = 0, c = 0;
        while (a + 1 < m && s[0][a + 1] <= i) a++;
        while (b + 1 < n && s[1][b + 1] <= j) b++;
        while (c + 1 < p && s[2][c + 1] <= k) c++;
        int r = a + b * m + c * m * n;
        out[i + j * M + k * M * N] = off[r] + (i - s[0][a]) + (j - s[1][b]) * w[0][a] + (k - s[2][c]) * w[0][a] * w[1][b];
      }
  for (int d = 0; d < 3; d++) { free(w[d]); free(s[d]); }
  free(off);
  return 0;
}

/* -dm_mat_type sbaij -mat_ignore_lower_triangular [ext]: MATSBAIJ keeps the upper triangle
   (global column >= row) of what assembly_jac inserts and MatMult uses its transpose for the
   lower triangle (MatMult_SeqSBAIJ_3).  Emulated by mirroring the assembled AIJ values. */
void orc_sbaij_mirror(orc_problem* P) {
  /* MatMult_SeqSBAIJ_3's order (a block-row scatter) is not restated: the mirrored matrix is
     multiplied in plain ascending column order (the GPU SBAIJ kernels are held to rounding) */
  P->spmv_order = ORC_SPMV_SEQAIJ;
  for (int64_t row = 0; row < P->ndofs; row++)
    for (int64_t q = P->rowptr[row]; q < P->rowptr[row + 1]; q++) {
      int64_t col = P->colidx[q];
      if (col < row) P->val[q] = P->val[csr_find(P, col, row)];
    }
}

#ifdef _OPENMP
#include <omp.h>
#endif
/* threads used by the emulated ranks (bench cpu_baseline); returns the count in effect */
int orc_set_threads(int n) {
#ifdef _OPENMP
  if (n > 0) omp_set_num_threads(n);
  return omp_get_max_threads();
#else
  (void)n;
  return 1;
#endif
}
