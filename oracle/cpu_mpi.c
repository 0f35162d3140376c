/*
 * cpu_mpi.c — the reference's Newton step on host CPU cores under MPI, one rank per core, as
 * the reference runs (`mpirun -np N macroc -da_grid_x ...`, tests/CMakeLists.txt:21-32).
 *
 * TEST INFRASTRUCTURE ONLY: the timed CPU baseline of bench.py (cpu_baseline, kind "port") and
 * tests/test_cpu_mpi.py.  It is never loaded by the product (macroc_amd/), which has no CPU path.
 *
 * Each rank owns the DMDA box PETSc would give it (-da_processors_x/y/z, or PETSC_DECIDE through
 * orc_dmda_decide, widths M/m + (i < M%m)) and runs src/main.c:61-79 on it with the data
 * structures PETSc uses there:
 *   set_strains (src/assembly.c:25-66, after DMGlobalToLocal of u: the ghost exchange),
 *   homogenize (isotropic elastic law: the MicroPP stand-in of the oracle, E = 1e7, nu = 0.25),
 *   assembly_res (src/assembly.c:120-176) and VecNorm,
 *   assembly_jac with the reference's naive 4-nest element matrix (src/assembly.c:94-99) added
 *   into MPIAIJ storage: a diagonal CSR (owned columns) and an off-diagonal CSR (the ghost
 *   columns, compressed, ascending global order), 32-bit PetscInt indices, then
 *   MatZeroRowsColumns(diag 1) (apply_bc_on_jac, src/bcs.c:341-347),
 *   KSPSolve_CG + PCJacobi with KSP_NORM_PRECONDITIONED and KSPConvergedDefault: MatMult in the
 *   MATAIJ inode kernel's form (the three rows of a node share one column-index stream, each
 *   row adds its column pairs over the diagonal block, then the off-diagonal block term by term:
 *   oracle/oracle.c orc_spmv_order), VecScatter of the ghost values by MPI_Isend/Irecv with the <= 26 neighbour
 *   ranks, MPI_Allreduce for every dot product and norm,
 *   VecAXPY(u, 1, du).
 * Assembly is owner-computes: the rank evaluates every element touching an owned node and adds
 * only its own rows (the one element layer on a subdomain face is evaluated by both ranks
 * instead of being stashed and sent at MatAssemblyEnd).  Sums over elements therefore run in a
 * different order than PETSc's at subdomain faces: results agree with the oracle to rounding
 * (tests/test_cpu_mpi.py), and the operation count is PETSc's plus that layer.
 *
 *   mpirun -np N ./macroc_cpu_mpi -da_grid_x 128 -da_grid_y 128 -da_grid_z 128 [-da_processors_x ..]
 *          [-ksp_rtol 1e-8] [-ksp_max_it N] [-steps K] [-warmup W] [-dump du.bin]
 * Rank 0 prints one JSON line: per-phase seconds of the last timed step, the mean step time,
 * CG iterations, reason, |RES| and |du|.
 */
#include <math.h>
#include <mpi.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

#define NGP 8
#define NPE 8
#define NVOI 6
#define DIM 3

static double B[NGP][NVOI][NPE * DIM];

typedef struct {
  int64_t NX, NY, NZ;
  int m, n, p, rank, size, pi, pj, pk;
  int64_t *wx, *wy, *wz, *sx, *sy, *sz; /* ownership widths / starts per processor column */
  int64_t *node_off;                    /* first PETSc global node of every rank (size + 1) */
  int64_t xs, ys, zs, nx, ny, nz, nown; /* owned box */
  int64_t gxs, gys, gzs, gnx, gny, gnz; /* ghosted box (one layer where it exists) */
  int64_t nghost;                       /* ghost nodes (ghosted box minus owned), ascending global */
  int64_t *gl;                          /* ghosted-local node -> owned index (>= 0) or -(ghost index) - 1 */
  int64_t *ghost_g;                     /* ghost index -> PETSc global node */
  /* neighbour exchange */
  int nnbr, nbr[26];
  int64_t rcnt[26], roff[26];           /* ghosts received from nbr: count, first ghost index */
  int64_t scnt[26], soff[26], *sidx;    /* owned nodes sent to nbr (owned indices) */
  double *sbuf;
  /* elements touching owned nodes */
  int64_t ex0, ey0, ez0, nex, ney, nez, ne;
  /* matrix: per owned node, its column list = diag part (owned columns) + off part (ghosts) */
  int32_t *dcnt, *ocnt;                 /* neighbour blocks per node in each part */
  int64_t *drp, *orp;                   /* first value of node's row 0 in dval / oval (3 rows follow) */
  int32_t *dcol, *ocol;                 /* per node: column node (owned index / ghost index), 3 dofs each */
  int64_t *dcol_off, *ocol_off;         /* per node: first entry in dcol / ocol */
  int16_t *bpos;                        /* per node and neighbour nb: position in its part (-1 absent), part bit 0x100 */
  double *dval, *oval;
  int64_t dnnz, onnz;
  /* state */
  unsigned char *dir_own, *dir_ghost;   /* Dirichlet flags per DOF */
  double *u, *ug, *b, *du, *r, *z, *pv, *pg, *w, *dinv;
  double *eps, *sig;
  double dx, dy, dz, wg, C[36], lx, ly, lz, rad, dt;
  double rtol, abstol, dtol;
  int maxits;
} Ctx;

static int64_t owner_col(const int64_t* s, int cnt, int64_t i) {
  int a = 0;
  while (a + 1 < cnt && s[a + 1] <= i) a++;
  return a;
}

static int64_t petsc_node(const Ctx* c, int64_t i, int64_t j, int64_t k) {
  int a = (int)owner_col(c->sx, c->m, i), b = (int)owner_col(c->sy, c->n, j), d = (int)owner_col(c->sz, c->p, k);
  int r = a + c->m * (b + c->n * d);
  return c->node_off[r] + (i - c->sx[a]) + c->wx[a] * ((j - c->sy[b]) + c->wy[b] * (k - c->sz[d]));
}

/* analytic Dirichlet set of BC_CIRCLE (src/bcs.c:154-338, the union of the ranks' lists;
   tests/golden/make_golden.py restates the same): the bottom face's edge nodes (3 DOFs) and the
   loaded circle on the top face (DOF 1) */
static int dof_dirichlet(const Ctx* c, int64_t i, int64_t j, int64_t k, int d, double* val, double U) {
  if (j == 0 && (i == 0 || i == c->NX - 1 || k == 0 || k == c->NZ - 1)) {
    *val = 0.;
    return 1;
  }
  if (j == c->NY - 1 && d == 1) {
    const double x = c->lx / 2. - (i * c->dx + c->dx / 2.);
    const double z = c->lz / 2. - (k * c->dz + c->dz / 2.);
    if ((x * x + z * z) < 1 * (c->rad * c->rad)) {
      *val = U;
      return 1;
    }
  }
  return 0;
}

static void* xmalloc(size_t n) {
  void* p = calloc(1, n ? n : 1);
  if (!p) {
    fprintf(stderr, "cpu_mpi: out of memory (%zu B)\n", n);
    MPI_Abort(MPI_COMM_WORLD, 2);
  }
  return p;
}

static void setup(Ctx* c) {
  /* ownership (DMSetUp_DA_3D) */
  int64_t* W[3] = {c->wx = xmalloc(c->m * 8), c->wy = xmalloc(c->n * 8), c->wz = xmalloc(c->p * 8)};
  int64_t* S[3] = {c->sx = xmalloc(c->m * 8), c->sy = xmalloc(c->n * 8), c->sz = xmalloc(c->p * 8)};
  const int64_t M[3] = {c->NX, c->NY, c->NZ};
  const int cnt[3] = {c->m, c->n, c->p};
  for (int d = 0; d < 3; d++) {
    int64_t s = 0;
    for (int a = 0; a < cnt[d]; a++) {
      W[d][a] = M[d] / cnt[d] + ((M[d] % cnt[d]) > a);
      S[d][a] = s;
      s += W[d][a];
    }
  }
  c->node_off = xmalloc((c->size + 1) * 8);
  for (int r = 0; r < c->size; r++) {
    const int a = r % c->m, b = (r / c->m) % c->n, d = r / (c->m * c->n);
    c->node_off[r + 1] = c->node_off[r] + c->wx[a] * c->wy[b] * c->wz[d];
  }
  c->pi = c->rank % c->m;
  c->pj = (c->rank / c->m) % c->n;
  c->pk = c->rank / (c->m * c->n);
  c->xs = c->sx[c->pi]; c->nx = c->wx[c->pi];
  c->ys = c->sy[c->pj]; c->ny = c->wy[c->pj];
  c->zs = c->sz[c->pk]; c->nz = c->wz[c->pk];
  c->nown = c->nx * c->ny * c->nz;
  c->gxs = c->xs > 0 ? c->xs - 1 : 0; c->gnx = (c->xs + c->nx < c->NX ? c->xs + c->nx + 1 : c->NX) - c->gxs;
  c->gys = c->ys > 0 ? c->ys - 1 : 0; c->gny = (c->ys + c->ny < c->NY ? c->ys + c->ny + 1 : c->NY) - c->gys;
  c->gzs = c->zs > 0 ? c->zs - 1 : 0; c->gnz = (c->zs + c->nz < c->NZ ? c->zs + c->nz + 1 : c->NZ) - c->gzs;
  const int64_t gn = c->gnx * c->gny * c->gnz;
  /* ghosts: ascending PETSc global index (the compressed off-diagonal columns, garray) */
  c->gl = xmalloc(gn * 8);
  c->nghost = gn - c->nown;
  c->ghost_g = xmalloc(c->nghost * 8);
  int64_t q = 0;
  for (int64_t k = c->gzs; k < c->gzs + c->gnz; k++)
    for (int64_t j = c->gys; j < c->gys + c->gny; j++)
      for (int64_t i = c->gxs; i < c->gxs + c->gnx; i++) {
        const int64_t l = (i - c->gxs) + c->gnx * ((j - c->gys) + c->gny * (k - c->gzs));
        const int own = i >= c->xs && i < c->xs + c->nx && j >= c->ys && j < c->ys + c->ny && k >= c->zs &&
                        k < c->zs + c->nz;
        if (own) c->gl[l] = (i - c->xs) + c->nx * ((j - c->ys) + c->ny * (k - c->zs));
        else c->ghost_g[q++] = petsc_node(c, i, j, k);
      }
  /* sort the ghost globals (insertion into rank-contiguous ranges: a counting pass per rank) */
  {
    int64_t* tmp = xmalloc(c->nghost * 8);
    int64_t* cnt_r = xmalloc((c->size + 1) * 8);
    for (int64_t g = 0; g < c->nghost; g++) {
      int r = 0;
      while (c->node_off[r + 1] <= c->ghost_g[g]) r++;
      cnt_r[r + 1]++;
    }
    for (int r = 0; r < c->size; r++) cnt_r[r + 1] += cnt_r[r];
    int64_t* fill = xmalloc((c->size + 1) * 8);
    memcpy(fill, cnt_r, (c->size + 1) * 8);
    for (int64_t g = 0; g < c->nghost; g++) {
      int r = 0;
      while (c->node_off[r + 1] <= c->ghost_g[g]) r++;
      tmp[fill[r]++] = c->ghost_g[g];
    }
    /* within a rank the enumeration above is ascending k, j, i of the ghosted box, which is
       that rank's local order, hence ascending global: already sorted */
    memcpy(c->ghost_g, tmp, c->nghost * 8);
    /* neighbours and receive ranges */
    c->nnbr = 0;
    for (int r = 0; r < c->size; r++)
      if (cnt_r[r + 1] > cnt_r[r]) {
        c->nbr[c->nnbr] = r;
        c->roff[c->nnbr] = cnt_r[r];
        c->rcnt[c->nnbr] = cnt_r[r + 1] - cnt_r[r];
        c->nnbr++;
      }
    free(tmp);
    free(cnt_r);
    free(fill);
  }
  for (int64_t k = c->gzs; k < c->gzs + c->gnz; k++)
    for (int64_t j = c->gys; j < c->gys + c->gny; j++)
      for (int64_t i = c->gxs; i < c->gxs + c->gnx; i++) {
        const int own = i >= c->xs && i < c->xs + c->nx && j >= c->ys && j < c->ys + c->ny && k >= c->zs &&
                        k < c->zs + c->nz;
        if (own) continue;
        const int64_t l = (i - c->gxs) + c->gnx * ((j - c->gys) + c->gny * (k - c->gzs));
        const int64_t g = petsc_node(c, i, j, k);
        int64_t lo = 0, hi = c->nghost - 1;
        while (lo < hi) {
          const int64_t mid = (lo + hi) / 2;
          if (c->ghost_g[mid] < g) lo = mid + 1; else hi = mid;
        }
        c->gl[l] = -lo - 1;
      }
  /* sends: my owned nodes inside each neighbour's ghosted box, ascending local (= global) */
  int64_t total = 0;
  for (int t = 0; t < c->nnbr; t++) {
    const int r = c->nbr[t], a = r % c->m, b = (r / c->m) % c->n, d = r / (c->m * c->n);
    const int64_t x0 = c->sx[a] > 0 ? c->sx[a] - 1 : 0, x1 = c->sx[a] + c->wx[a] + 1;
    const int64_t y0 = c->sy[b] > 0 ? c->sy[b] - 1 : 0, y1 = c->sy[b] + c->wy[b] + 1;
    const int64_t z0 = c->sz[d] > 0 ? c->sz[d] - 1 : 0, z1 = c->sz[d] + c->wz[d] + 1;
    int64_t n = 0;
    for (int64_t k = c->zs; k < c->zs + c->nz; k++)
      for (int64_t j = c->ys; j < c->ys + c->ny; j++)
        for (int64_t i = c->xs; i < c->xs + c->nx; i++) n += i >= x0 && i < x1 && j >= y0 && j < y1 && k >= z0 && k < z1;
    c->scnt[t] = n;
    c->soff[t] = total;
    total += n;
  }
  c->sidx = xmalloc(total * 8);
  c->sbuf = xmalloc(total * 3 * 8);
  for (int t = 0; t < c->nnbr; t++) {
    const int r = c->nbr[t], a = r % c->m, b = (r / c->m) % c->n, d = r / (c->m * c->n);
    const int64_t x0 = c->sx[a] > 0 ? c->sx[a] - 1 : 0, x1 = c->sx[a] + c->wx[a] + 1;
    const int64_t y0 = c->sy[b] > 0 ? c->sy[b] - 1 : 0, y1 = c->sy[b] + c->wy[b] + 1;
    const int64_t z0 = c->sz[d] > 0 ? c->sz[d] - 1 : 0, z1 = c->sz[d] + c->wz[d] + 1;
    int64_t n = c->soff[t];
    for (int64_t k = c->zs; k < c->zs + c->nz; k++)
      for (int64_t j = c->ys; j < c->ys + c->ny; j++)
        for (int64_t i = c->xs; i < c->xs + c->nx; i++)
          if (i >= x0 && i < x1 && j >= y0 && j < y1 && k >= z0 && k < z1)
            c->sidx[n++] = (i - c->xs) + c->nx * ((j - c->ys) + c->ny * (k - c->zs));
  }
  /* elements touching owned nodes */
  c->ex0 = c->xs > 0 ? c->xs - 1 : 0; c->nex = (c->xs + c->nx - 1 < c->NX - 2 ? c->xs + c->nx - 1 : c->NX - 2) - c->ex0 + 1;
  c->ey0 = c->ys > 0 ? c->ys - 1 : 0; c->ney = (c->ys + c->ny - 1 < c->NY - 2 ? c->ys + c->ny - 1 : c->NY - 2) - c->ey0 + 1;
  c->ez0 = c->zs > 0 ? c->zs - 1 : 0; c->nez = (c->zs + c->nz - 1 < c->NZ - 2 ? c->zs + c->nz - 1 : c->NZ - 2) - c->ez0 + 1;
  c->ne = c->nex * c->ney * c->nez;
  /* MPIAIJ pattern (DMCreateMatrix_DA_3d_MPIAIJ: the clipped 27-point box, 3x3 dense blocks) */
  c->dcnt = xmalloc(c->nown * 4);
  c->ocnt = xmalloc(c->nown * 4);
  c->drp = xmalloc(c->nown * 8);
  c->orp = xmalloc(c->nown * 8);
  c->dcol_off = xmalloc(c->nown * 8);
  c->ocol_off = xmalloc(c->nown * 8);
  c->bpos = xmalloc(c->nown * 27 * 2);
  int64_t nd = 0, no = 0;
  for (int pass = 0; pass < 2; pass++) {
    nd = no = 0;
    for (int64_t n = 0; n < c->nown; n++) {
      const int64_t i = c->xs + n % c->nx, j = c->ys + (n / c->nx) % c->ny, k = c->zs + n / (c->nx * c->ny);
      int dn = 0, on = 0;
      /* the diagonal part in ascending owned index, the off part in ascending ghost index
         (= ascending global): collect, then order by index (27 entries: insertion sort) */
      int32_t dl[27], ol[27], dnb[27], onb[27];
      for (int nb = 0; nb < 27; nb++) {
        const int64_t ii = i + nb % 3 - 1, jj = j + (nb / 3) % 3 - 1, kk = k + nb / 9 - 1;
        if (pass) c->bpos[n * 27 + nb] = -1;
        if (ii < 0 || ii >= c->NX || jj < 0 || jj >= c->NY || kk < 0 || kk >= c->NZ) continue;
        const int64_t l = c->gl[(ii - c->gxs) + c->gnx * ((jj - c->gys) + c->gny * (kk - c->gzs))];
        if (l >= 0) { dl[dn] = (int32_t)l; dnb[dn++] = nb; }
        else { ol[on] = (int32_t)(-l - 1); onb[on++] = nb; }
      }
      for (int a = 1; a < dn; a++)
        for (int b2 = a; b2 > 0 && dl[b2 - 1] > dl[b2]; b2--) {
          int32_t t = dl[b2]; dl[b2] = dl[b2 - 1]; dl[b2 - 1] = t;
          t = dnb[b2]; dnb[b2] = dnb[b2 - 1]; dnb[b2 - 1] = t;
        }
      for (int a = 1; a < on; a++)
        for (int b2 = a; b2 > 0 && ol[b2 - 1] > ol[b2]; b2--) {
          int32_t t = ol[b2]; ol[b2] = ol[b2 - 1]; ol[b2 - 1] = t;
          t = onb[b2]; onb[b2] = onb[b2 - 1]; onb[b2 - 1] = t;
        }
      if (pass) {
        c->dcnt[n] = dn;
        c->ocnt[n] = on;
        c->drp[n] = 9 * nd;
        c->orp[n] = 9 * no;
        c->dcol_off[n] = 3 * nd;
        c->ocol_off[n] = 3 * no;
        for (int a = 0; a < dn; a++) {
          for (int d = 0; d < 3; d++) c->dcol[3 * (nd + a) + d] = 3 * dl[a] + d;
          c->bpos[n * 27 + dnb[a]] = (int16_t)a;
        }
        for (int a = 0; a < on; a++) {
          for (int d = 0; d < 3; d++) c->ocol[3 * (no + a) + d] = 3 * ol[a] + d;
          c->bpos[n * 27 + onb[a]] = (int16_t)(0x100 | a);
        }
      }
      nd += dn;
      no += on;
    }
    if (!pass) {
      c->dcol = xmalloc(3 * nd * 4);
      c->ocol = xmalloc(3 * no * 4 + 4);
    }
  }
  c->dnnz = 9 * nd;
  c->onnz = 9 * no;
  c->dval = xmalloc(c->dnnz * 8);
  c->oval = xmalloc(c->onnz * 8 + 8);
  /* vectors and Gauss-point arrays */
  const int64_t n3 = 3 * c->nown, g3 = 3 * c->nghost;
  c->u = xmalloc(n3 * 8); c->ug = xmalloc(g3 * 8 + 8); c->b = xmalloc(n3 * 8); c->du = xmalloc(n3 * 8);
  c->r = xmalloc(n3 * 8); c->z = xmalloc(n3 * 8); c->pv = xmalloc(n3 * 8); c->pg = xmalloc(g3 * 8 + 8);
  c->w = xmalloc(n3 * 8); c->dinv = xmalloc(n3 * 8);
  c->eps = xmalloc(c->ne * NGP * NVOI * 8);
  c->sig = xmalloc(c->ne * NGP * NVOI * 8);
  c->dir_own = xmalloc(n3);
  c->dir_ghost = xmalloc(g3 + 1);
  double v;
  for (int64_t n = 0; n < c->nown; n++) {
    const int64_t i = c->xs + n % c->nx, j = c->ys + (n / c->nx) % c->ny, k = c->zs + n / (c->nx * c->ny);
    for (int d = 0; d < 3; d++) c->dir_own[3 * n + d] = (unsigned char)dof_dirichlet(c, i, j, k, d, &v, 0.);
  }
  for (int64_t k = c->gzs; k < c->gzs + c->gnz; k++)
    for (int64_t j = c->gys; j < c->gys + c->gny; j++)
      for (int64_t i = c->gxs; i < c->gxs + c->gnx; i++) {
        const int64_t l = c->gl[(i - c->gxs) + c->gnx * ((j - c->gys) + c->gny * (k - c->gzs))];
        if (l >= 0) continue;
        for (int d = 0; d < 3; d++) c->dir_ghost[3 * (-l - 1) + d] = (unsigned char)dof_dirichlet(c, i, j, k, d, &v, 0.);
      }
}

/* VecScatter of the ghost values (DMGlobalToLocal / MatMult_MPIAIJ's lvec) */
static void exchange(Ctx* c, const double* own, double* ghost) {
  MPI_Request req[52];
  int nr = 0;
  for (int t = 0; t < c->nnbr; t++)
    MPI_Irecv(ghost + 3 * c->roff[t], (int)(3 * c->rcnt[t]), MPI_DOUBLE, c->nbr[t], 7, MPI_COMM_WORLD, &req[nr++]);
  for (int t = 0; t < c->nnbr; t++) {
    double* sb = c->sbuf + 3 * c->soff[t];
    for (int64_t q = 0; q < c->scnt[t]; q++) {
      const int64_t n = c->sidx[c->soff[t] + q];
      sb[3 * q] = own[3 * n];
      sb[3 * q + 1] = own[3 * n + 1];
      sb[3 * q + 2] = own[3 * n + 2];
    }
    MPI_Isend(sb, (int)(3 * c->scnt[t]), MPI_DOUBLE, c->nbr[t], 7, MPI_COMM_WORLD, &req[nr++]);
  }
  MPI_Waitall(nr, req, MPI_STATUSES_IGNORE);
}

static double dot(const Ctx* c, const double* a, const double* b2) {
  double s = 0.;
  for (int64_t q = 0; q < 3 * c->nown; q++) s += a[q] * b2[q];
  double t;
  MPI_Allreduce(&s, &t, 1, MPI_DOUBLE, MPI_SUM, MPI_COMM_WORLD);
  return t;
}

/* element ie's 8 nodes as ghosted-local indices, the reference's local node order */
static void elem_nodes(const Ctx* c, int64_t ie, int64_t* l) {
  const int64_t ex = c->ex0 + ie % c->nex, ey = c->ey0 + (ie / c->nex) % c->ney, ez = c->ez0 + ie / (c->nex * c->ney);
  static const int o[8][3] = {{0, 0, 0}, {1, 0, 0}, {1, 1, 0}, {0, 1, 0}, {0, 0, 1}, {1, 0, 1}, {1, 1, 1}, {0, 1, 1}};
  for (int a = 0; a < 8; a++)
    l[a] = (ex + o[a][0] - c->gxs) + c->gnx * ((ey + o[a][1] - c->gys) + c->gny * (ez + o[a][2] - c->gzs));
}

static double val_of(const Ctx* c, const double* own, const double* ghost, int64_t gli, int d) {
  const int64_t l = c->gl[gli];
  return l >= 0 ? own[3 * l + d] : ghost[3 * (-l - 1) + d];
}

static void set_strains(Ctx* c) {
  exchange(c, c->u, c->ug);
  for (int64_t ie = 0; ie < c->ne; ie++) {
    int64_t l[8];
    elem_nodes(c, ie, l);
    double ue[24];
    for (int a = 0; a < 8; a++)
      for (int d = 0; d < 3; d++) ue[3 * a + d] = val_of(c, c->u, c->ug, l[a], d);
    for (int gp = 0; gp < NGP; gp++) {
      double* e = c->eps + (ie * NGP + gp) * NVOI;
      for (int i = 0; i < NVOI; i++) {
        double s = 0.;
        for (int j = 0; j < 24; j++) s += B[gp][i][j] * ue[j];
        e[i] = s;
      }
    }
  }
}

static void homogenize(Ctx* c) {
  for (int64_t g = 0; g < c->ne * NGP; g++) {
    const double* e = c->eps + g * NVOI;
    double* s = c->sig + g * NVOI;
    for (int k = 0; k < NVOI; k++) {
      double acc = 0.;
      for (int l = 0; l < NVOI; l++) acc += c->C[k * NVOI + l] * e[l];
      s[k] = acc;
    }
  }
}

static int owned_index(const Ctx* c, int64_t gli) { return c->gl[gli] >= 0; }

static double assembly_res(Ctx* c) {
  memset(c->b, 0, 3 * c->nown * 8);
  for (int64_t ie = 0; ie < c->ne; ie++) {
    int64_t l[8];
    elem_nodes(c, ie, l);
    double be[24];
    memset(be, 0, sizeof(be));
    for (int gp = 0; gp < NGP; gp++) {
      const double* st = c->sig + (ie * NGP + gp) * NVOI;
      for (int i = 0; i < 24; i++)
        for (int j = 0; j < NVOI; j++) be[i] += B[gp][j][i] * st[j] * c->wg;
    }
    for (int a = 0; a < 8; a++)
      if (owned_index(c, l[a])) {
        const int64_t n = c->gl[l[a]];
        for (int d = 0; d < 3; d++) c->b[3 * n + d] += be[3 * a + d];
      }
  }
  for (int64_t q = 0; q < 3 * c->nown; q++) {
    if (c->dir_own[q]) c->b[q] = 0.;
    c->b[q] = c->b[q] * -1.;
  }
  return sqrt(dot(c, c->b, c->b));
}

static void assembly_jac(Ctx* c) {
  memset(c->dval, 0, c->dnnz * 8);
  memset(c->oval, 0, c->onnz * 8);
  static double Ae[24 * 24];
  for (int64_t ie = 0; ie < c->ne; ie++) {
    int64_t l[8];
    elem_nodes(c, ie, l);
    int any = 0;
    for (int a = 0; a < 8; a++) any |= owned_index(c, l[a]);
    if (!any) continue;
    memset(Ae, 0, sizeof(Ae));
    for (int gp = 0; gp < NGP; gp++)
      for (int i = 0; i < 24; i++)
        for (int j = 0; j < 24; j++)
          for (int k = 0; k < NVOI; k++)
            for (int m = 0; m < NVOI; m++) Ae[24 * i + j] += B[gp][k][i] * c->C[k * NVOI + m] * B[gp][m][j] * c->wg;
    for (int a = 0; a < 8; a++) {
      if (!owned_index(c, l[a])) continue;
      const int64_t n = c->gl[l[a]];
      const int64_t ai = l[a] % c->gnx, aj = (l[a] / c->gnx) % c->gny, ak = l[a] / (c->gnx * c->gny);
      for (int b2 = 0; b2 < 8; b2++) {
        const int64_t bi = l[b2] % c->gnx, bj = (l[b2] / c->gnx) % c->gny, bk = l[b2] / (c->gnx * c->gny);
        const int nb = (int)((bi - ai + 1) + 3 * (bj - aj + 1) + 9 * (bk - ak + 1));
        const int pos = c->bpos[n * 27 + nb];
        const int off = pos & 0xff;
        double* rowv = (pos & 0x100) ? c->oval + c->orp[n] : c->dval + c->drp[n];
        const int len = 3 * ((pos & 0x100) ? c->ocnt[n] : c->dcnt[n]);
        for (int r = 0; r < 3; r++)
          for (int d = 0; d < 3; d++) rowv[r * len + 3 * off + d] += Ae[24 * (3 * a + r) + 3 * b2 + d];
      }
    }
  }
  /* MatZeroRowsColumns(A, n, rows, 1.0, NULL, NULL) */
  for (int64_t n = 0; n < c->nown; n++) {
    const int dl = 3 * c->dcnt[n], ol = 3 * c->ocnt[n];
    const int32_t* dc = c->dcol + c->dcol_off[n];
    const int32_t* oc = c->ocol + c->ocol_off[n];
    for (int r = 0; r < 3; r++) {
      const int64_t row = 3 * n + r;
      double* dv = c->dval + c->drp[n] + r * dl;
      double* ov = c->oval + c->orp[n] + r * ol;
      for (int q = 0; q < dl; q++)
        if (c->dir_own[row]) dv[q] = dc[q] == row ? 1. : 0.;
        else if (c->dir_own[dc[q]]) dv[q] = 0.;
      for (int q = 0; q < ol; q++)
        if (c->dir_own[row] || c->dir_ghost[oc[q]]) ov[q] = 0.;
    }
  }
}

/* MatMult_MPIAIJ (oracle/oracle.c orc_spmv_order): the diagonal block with the SeqAIJ inode
   kernel (the node's column index stream read once for its three rows; each row adds its terms
   in column pairs from 0), then the off-diagonal block from that sum with MatMultAdd_SeqAIJ's
   plain loop, term by term (MatAssemblyEnd_MPIAIJ turns inodes off for it) */
static void matmult(Ctx* c, const double* x, double* y) {
  exchange(c, x, c->pg);
  for (int64_t n = 0; n < c->nown; n++) {
    double s[3] = {0., 0., 0.};
    for (int part = 0; part < 2; part++) {
      const int len = 3 * (part ? c->ocnt[n] : c->dcnt[n]);
      const int32_t* idx = part ? c->ocol + c->ocol_off[n] : c->dcol + c->dcol_off[n];
      const double* v1 = part ? c->oval + c->orp[n] : c->dval + c->drp[n];
      const double* v2 = v1 + len;
      const double* v3 = v2 + len;
      const double* xx = part ? c->pg : x;
      double s1 = s[0], s2 = s[1], s3 = s[2];
      int q = 0;
      if (part) {  // off-diagonal block: no inodes, one term at a time
        for (; q < len; q++) {
          const double t0 = xx[idx[q]];
          s1 += v1[q] * t0;
          s2 += v2[q] * t0;
          s3 += v3[q] * t0;
        }
      }
      for (; q < len - 1; q += 2) {
        const double t0 = xx[idx[q]], t1 = xx[idx[q + 1]];
        s1 += v1[q] * t0 + v1[q + 1] * t1;
        s2 += v2[q] * t0 + v2[q + 1] * t1;
        s3 += v3[q] * t0 + v3[q + 1] * t1;
      }
      if (q == len - 1) {
        const double t0 = xx[idx[q]];
        s1 += v1[q] * t0;
        s2 += v2[q] * t0;
        s3 += v3[q] * t0;
      }
      s[0] = s1, s[1] = s2, s[2] = s3;
    }
    y[3 * n] = s[0];
    y[3 * n + 1] = s[1];
    y[3 * n + 2] = s[2];
  }
}

static int converged(double rn, double ttol, double abstol, double dtol, double rn0) {
  if (isnan(rn) || isinf(rn)) return ORC_KSP_DIVERGED_NANORINF;
  if (rn <= ttol) return rn < abstol ? ORC_KSP_CONVERGED_ATOL : ORC_KSP_CONVERGED_RTOL;
  if (rn >= dtol * rn0) return ORC_KSP_DIVERGED_DTOL;
  return 0;
}

/* KSPSolve_CG + PCJacobi (oracle.c orc_solve), every reduction an MPI_Allreduce */
static int solve(Ctx* c, int* its_out, double* rn_out) {
  const int64_t N = 3 * c->nown;
  for (int64_t n = 0; n < c->nown; n++)
    for (int r = 0; r < 3; r++) {
      const int dl = 3 * c->dcnt[n];
      const int32_t* dc = c->dcol + c->dcol_off[n];
      const double* dv = c->dval + c->drp[n] + r * dl;
      double d = 0.;
      for (int q = 0; q < dl; q++)
        if (dc[q] == 3 * n + r) d = dv[q];
      if (d != 0.0) d = 1.0 / d;
      if (d == 0.0) d = 1.0;
      c->dinv[3 * n + r] = d;
    }
  double* X = c->du;
  memset(X, 0, N * 8);
  memcpy(c->r, c->b, N * 8);
  for (int64_t q = 0; q < N; q++) c->z[q] = c->r[q] * c->dinv[q];
  double dp = sqrt(dot(c, c->z, c->z));
  const double ttol = fmax(c->rtol * dp, c->abstol), rn0 = dp;
  int reason = converged(dp, ttol, c->abstol, c->dtol, rn0), its = 0, i = 0;
  double rn = dp, beta = 0., betaold = 0., dpi = 0., dpiold;
  if (!reason) {
    beta = dot(c, c->z, c->r);
    do {
      its = i + 1;
      if (beta == 0.0) { reason = ORC_KSP_CONVERGED_ATOL; break; }
      if (i > 0 && beta * betaold < 0.0) { reason = ORC_KSP_DIVERGED_INDEFINITE_PC; break; }
      if (!i) memcpy(c->pv, c->z, N * 8);
      else {
        const double bb = beta / betaold;
        for (int64_t q = 0; q < N; q++) c->pv[q] = c->z[q] + bb * c->pv[q];
      }
      dpiold = dpi;
      matmult(c, c->pv, c->w);
      dpi = dot(c, c->pv, c->w);
      betaold = beta;
      if (dpi == 0.0 || (i > 0 && dpi * dpiold <= 0.0)) { reason = ORC_KSP_DIVERGED_INDEFINITE_MAT; break; }
      const double a = beta / dpi;
      for (int64_t q = 0; q < N; q++) X[q] = X[q] + a * c->pv[q];
      for (int64_t q = 0; q < N; q++) c->r[q] = c->r[q] + (-a) * c->w[q];
      for (int64_t q = 0; q < N; q++) c->z[q] = c->r[q] * c->dinv[q];
      dp = sqrt(dot(c, c->z, c->z));
      rn = dp;
      reason = converged(dp, ttol, c->abstol, c->dtol, rn0);
      if (reason) break;
      beta = dot(c, c->z, c->r);
      i++;
    } while (i < c->maxits);
    if (!reason && i >= c->maxits) reason = ORC_KSP_DIVERGED_ITS;
  }
  *its_out = its;
  *rn_out = rn;
  return reason;
}

int main(int argc, char** argv) {
  MPI_Init(&argc, &argv);
  Ctx cx;
  memset(&cx, 0, sizeof(cx));
  Ctx* c = &cx;
  MPI_Comm_rank(MPI_COMM_WORLD, &c->rank);
  MPI_Comm_size(MPI_COMM_WORLD, &c->size);
  c->NX = 40; c->NY = 3; c->NZ = 40;   /* src/init.c defaults */
  c->lx = 50.; c->ly = 1.; c->lz = 50.; c->rad = 1.; c->dt = 0.001;
  c->rtol = 1e-5; c->abstol = 1e-50; c->dtol = 1e4; c->maxits = 10000;
  int steps = 1, warmup = 0, ts = 1;
  const char* dump = NULL;
  for (int a = 1; a + 1 < argc; a += 2) {
    const char *k = argv[a], *v = argv[a + 1];
    if (!strcmp(k, "-da_grid_x")) c->NX = atoll(v);
    else if (!strcmp(k, "-da_grid_y")) c->NY = atoll(v);
    else if (!strcmp(k, "-da_grid_z")) c->NZ = atoll(v);
    else if (!strcmp(k, "-da_processors_x")) c->m = atoi(v);
    else if (!strcmp(k, "-da_processors_y")) c->n = atoi(v);
    else if (!strcmp(k, "-da_processors_z")) c->p = atoi(v);
    else if (!strcmp(k, "-ksp_rtol")) c->rtol = atof(v);
    else if (!strcmp(k, "-ksp_max_it")) c->maxits = atoi(v);
    else if (!strcmp(k, "-steps")) steps = atoi(v);
    else if (!strcmp(k, "-warmup")) warmup = atoi(v);
    else if (!strcmp(k, "-ts")) ts = atoi(v);
    else if (!strcmp(k, "-dump")) dump = v;
    else {
      if (!c->rank) fprintf(stderr, "cpu_mpi: unknown option %s\n", k);
      MPI_Abort(MPI_COMM_WORLD, 1);
    }
  }
  if (orc_dmda_decide(c->NX, c->NY, c->NZ, c->size, &c->m, &c->n, &c->p) || c->m * c->n * c->p != c->size) {
    if (!c->rank) fprintf(stderr, "cpu_mpi: bad processor grid for %d ranks\n", c->size);
    MPI_Abort(MPI_COMM_WORLD, 1);
  }
  c->dx = c->lx / (c->NX - 1); c->dy = c->ly / (c->NY - 1); c->dz = c->lz / (c->NZ - 1);
  c->wg = c->dx * c->dy * c->dz / 8.;  /* src/init.c:137-140 */
  for (int gp = 0; gp < NGP; gp++) orc_calc_B(gp, B[gp]);
  {
    const double E = 1.0e7, nu = 0.25;
    const double lam = E * nu / ((1. + nu) * (1. - 2. * nu)), mu = E / (2. * (1. + nu));
    for (int a = 0; a < 3; a++)
      for (int b2 = 0; b2 < 3; b2++) c->C[a * 6 + b2] = lam + (a == b2 ? 2. * mu : 0.);
    for (int a = 3; a < 6; a++) c->C[a * 6 + a] = mu;
  }
  double t0 = MPI_Wtime();
  setup(c);
  MPI_Barrier(MPI_COMM_WORLD);
  const double t_setup = MPI_Wtime() - t0;
  const double U = -1.0 * (ts * c->dt / 1.0);  /* get_displacement (U_MAX = -1, FINAL_TIME = 1) */
  double ph[6] = {0}, res = 0., rn = 0., t_steps = 0.;
  int its = 0, reason = 0;
  for (int s = 0; s < warmup + steps; s++) {
    MPI_Barrier(MPI_COMM_WORLD);
    const double ts0 = MPI_Wtime();
    double tp[7];
    tp[0] = ts0;
    /* VecZeroEntries(u) + apply_bc_on_u(U) */
    for (int64_t n = 0; n < c->nown; n++) {
      const int64_t i = c->xs + n % c->nx, j = c->ys + (n / c->nx) % c->ny, k = c->zs + n / (c->nx * c->ny);
      for (int d = 0; d < 3; d++) {
        double v = 0.;
        dof_dirichlet(c, i, j, k, d, &v, U);
        c->u[3 * n + d] = v;
      }
    }
    set_strains(c);
    tp[1] = MPI_Wtime();
    homogenize(c);
    tp[2] = MPI_Wtime();
    res = assembly_res(c);
    tp[3] = MPI_Wtime();
    assembly_jac(c);
    tp[4] = MPI_Wtime();
    reason = solve(c, &its, &rn);
    tp[5] = MPI_Wtime();
    for (int64_t q = 0; q < 3 * c->nown; q++) c->u[q] = c->u[q] + 1. * c->du[q];
    MPI_Barrier(MPI_COMM_WORLD);
    tp[6] = MPI_Wtime();
    if (s >= warmup) {
      t_steps += tp[6] - ts0;
      for (int q = 0; q < 6; q++) ph[q] = tp[q + 1] - tp[q];
    }
  }
  const double dun = sqrt(dot(c, c->du, c->du));
  if (dump) {  /* du in PETSc global order: the ranks' owned parts in rank order */
    int* cnts = xmalloc(c->size * sizeof(int));
    int* displs = xmalloc(c->size * sizeof(int));
    for (int r = 0; r < c->size; r++) {
      cnts[r] = (int)(3 * (c->node_off[r + 1] - c->node_off[r]));
      displs[r] = (int)(3 * c->node_off[r]);
    }
    double* all = c->rank ? NULL : xmalloc(3 * c->node_off[c->size] * 8);
    MPI_Gatherv(c->du, (int)(3 * c->nown), MPI_DOUBLE, all, cnts, displs, MPI_DOUBLE, 0, MPI_COMM_WORLD);
    if (!c->rank) {
      FILE* f = fopen(dump, "wb");
      if (!f || fwrite(all, 8, 3 * c->node_off[c->size], f) != (size_t)(3 * c->node_off[c->size])) {
        fprintf(stderr, "cpu_mpi: cannot write %s\n", dump);
        MPI_Abort(MPI_COMM_WORLD, 3);
      }
      fclose(f);
    }
  }
  int64_t nnz_loc = c->dnnz + c->onnz, nnz = 0;
  MPI_Reduce(&nnz_loc, &nnz, 1, MPI_INT64_T, MPI_SUM, 0, MPI_COMM_WORLD);
  if (!c->rank)
    printf("{\"nranks\": %d, \"grid\": [%lld, %lld, %lld], \"procs\": [%d, %d, %d], \"nnz\": %lld, \"steps\": %d, "
           "\"warmup\": %d, \"setup_s\": %.6f, \"step_s\": %.6f, \"phases_s\": {\"strains\": %.6f, \"homogenize\": %.6f, "
           "\"residual\": %.6f, \"jacobian\": %.6f, \"solve\": %.6f, \"update\": %.6f}, \"its\": %d, \"reason\": %d, "
           "\"res\": %.17g, \"rnorm\": %.17g, \"du_norm\": %.17g}\n",
           c->size, (long long)c->NX, (long long)c->NY, (long long)c->NZ, c->m, c->n, c->p, (long long)nnz, steps,
           warmup, t_setup, t_steps / (steps > 0 ? steps : 1), ph[0], ph[1], ph[2], ph[3], ph[4], ph[5], its, reason,
           res, rn, dun);
  MPI_Finalize();
  return 0;
}
