// kernels.hip — gfx950 kernels of the MacroC Newton inner loop.
//
// HBM layout (one rank = one GPU subdomain):
//   * node vectors u, p: padded ghosted box [PX*PY*PZ][3] (1 ghost layer, zeros outside
//     the physical domain) — stencil kernels never branch on the boundary;
//   * owned vectors b, du, r, z, w, dinv: PETSc-local order [nx*ny*nz][3];
//   * matrix: "stencil blocks" — for every owned node the 27 neighbour 3x3 blocks (243
//     slots, slot = nb*9 + r*3 + c, nb = (dz+1)*9 + (dy+1)*3 + (dx+1)); stored AoSoA as
//     [node/64][122 slot pairs][node%64] double2 so one wave reads 1 KiB contiguous per load.
//     The column of a slot is implicit (DMDA box stencil), so no index array is read;
//   * Gauss-point arrays: [component][gp][element] (element fastest, coalesced).
// Compiled with -ffp-contract=off: each product / sum is rounded as the reference writes it,
// so element kinematics, strains, stresses, element matrices, the assembled matrix, the
// residual and the SpMV are bit-identical to the CPU restatement on one rank.
#include <algorithm>
#include <cstring>
#include <cmath>

#include "mcx_internal.h"

namespace mcx {

__constant__ double cB[8][6][24];

static constexpr int TPB = 256;

// ---------------------------------------------------------------------------- helpers
__device__ __forceinline__ void node_ijk(const Geo& g, int n, int& i, int& j, int& k) {
  i = n % g.nx;
  int t = n / g.nx;
  j = t % g.ny;
  k = t / g.ny;
}

__device__ __forceinline__ int pad_of(const Geo& g, int i, int j, int k) {
  return (i + 1) + (j + 1) * g.PX + (k + 1) * g.PX * g.PY;
}

// sbaij storage index of node (i, j, k), i, j, k in -1..n (DMDA padded box, 64-aligned rows);
// neighbour (dx, dy, dz) is u_of + dx + dy*UX + dz*UXY
__device__ __forceinline__ int u_of(const Geo& g, int i, int j, int k) {
  return 64 + i + (j + 1) * g.UX + (k + 1) * g.UXY;
}

// Dirichlet DOFs of a global node as a bit mask (bit d = DOF d).  The union over ranks of
// bc_init_circle's ghost-corner lists (src/bcs.c:254-338) is exactly: the four y=0 edges,
// all DOFs; dof 1 of the y=LY nodes inside the load circle (cell-centre offset dx/2, :324-327).
// bc_init_bending (:198-251): faces x=0 and x=LX, all DOFs.
__host__ __device__ inline int dirichlet_mask(const Geo& g, int gi, int gj, int gk) {
  if (g.bc_type == MCX_BC_CIRCLE) {
    if (gj == 0 && (gi == 0 || gi == g.NX - 1 || gk == 0 || gk == g.NZ - 1)) return 7;
    if (gj == g.NY - 1) {
      double x = g.lx / 2. - ((double)gi * g.dx + g.dx / 2.);
      double z = g.lz / 2. - ((double)gk * g.dz + g.dz / 2.);
      if ((x * x + z * z) < (g.rad * g.rad)) return 2;
    }
    return 0;
  }
  if (g.bc_type == MCX_BC_BENDING) return (gi == 0 || gi == g.NX - 1) ? 7 : 0;
  return 0;
}

// local Q1 node number of offset (ox,oy,oz) in {0,1}^3: order ---,+--,++-,-+-,--+,+-+,+++,-++
__device__ __forceinline__ int q1_local(int ox, int oy, int oz) {
  return 4 * oz + (oy ? (ox ? 2 : 3) : (ox ? 1 : 0));
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// deterministic block sum (fixed tree); result valid in thread 0
template <int NT>
__device__ __forceinline__ double block_sum(double v, double* sh) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) sh[w] = v;
  __syncthreads();
  double r = 0.;
  if (threadIdx.x == 0) {
    for (int q = 0; q < NT / 64; q++) r += sh[q];
  }
  __syncthreads();
  return r;
}

// XCD-aware remap: consecutive logical blocks land on one XCD (its L2 sees the stencil
// neighbours' x lines); observed dispatch is round-robin over the 8 XCDs (speed only).
__device__ __forceinline__ int xcd_remap(int b, int nblk_padded) {
  const int per = nblk_padded >> 3;
  return (b & 7) * per + (b >> 3);
}

static inline int64_t pad8(int64_t n) { return (n + 7) / 8 * 8; }

// SpMV block tiling, XCD-slab order.  A block = TX nodes along x (TX = 64*ceil(nx/64), <= 256)
// x LPB = 256/TX consecutive y-lines, at one z-plane.  The y-line groups are cut into 8
// contiguous slabs, one per XCD (blocks b and b+8 share an XCD under the observed round-robin
// placement — speed only), and each XCD sweeps its slab plane by plane, so the stencil's
// previous-plane neighbours (x values, sbaij mirror blocks) of a plane are still in that XCD's
// L2 when the next plane is processed.
struct SpmvTiling {
  int TX, LPB, nxc, jgroups, per_xcd;  // per_xcd = max blocks on one XCD
  int subl;                            // lines per sub-slab (0 = whole slab per plane)
};

static SpmvTiling spmv_tiling(const Geo& g, int subl) {
  SpmvTiling t;
  t.subl = subl;
  t.TX = (int)std::min<int64_t>(256, (g.nx + 63) / 64 * 64);
  t.LPB = 256 / t.TX;
  t.nxc = (g.nx + t.TX - 1) / t.TX;
  t.jgroups = (g.ny + t.LPB - 1) / t.LPB;
  const int slab = (t.jgroups + 7) / 8;
  t.per_xcd = slab * g.nz * t.nxc;
  return t;
}

// returns the owned node of this thread or -1.  Within an XCD's slab the lines are swept in
// sub-slabs of SUBL lines over all planes (sub-slab, k, line group, x chunk), so one plane of
// a sub-slab (SUBL x nx nodes, ~2 MB of sbaij blocks at nx = 256) stays in the XCD's 4 MB L2
// until the next plane reads its mirror blocks; only sub-slab edge lines miss.
__device__ __forceinline__ int spmv_node(const Geo& g, int TX, int LPB, int nxc, int jgroups, int subl, int& ii,
                                         int& jj, int& kk) {
  const int b = blockIdx.x;
  if (subl < 0) {  // linear order: consecutive blocks = consecutive lines (k, line group, x chunk)
    const int k = b / (jgroups * nxc);
    const int rem = b - k * (jgroups * nxc);
    const int i = (rem % nxc) * TX + (int)(threadIdx.x % TX), j = (rem / nxc) * LPB + (int)(threadIdx.x / TX);
    if (k >= g.nz || i >= g.nx || j >= g.ny) return -1;
    ii = i;
    jj = j;
    kk = k;
    return i + g.nx * (j + g.ny * k);
  }
  const int x = b & 7;
  int t = b >> 3;
  const int slab = (jgroups + 7) >> 3;
  const int g0 = x * slab;
  const int gcount = min(slab, jgroups - g0);
  if (gcount <= 0) return -1;
  const int SG = subl > 0 ? max(1, subl / LPB) : gcount;  // line groups per sub-slab
  const int full = gcount / SG;
  const int per_sub = SG * g.nz * nxc;
  int sub, sgn;
  if (t < full * per_sub) {
    sub = t / per_sub;
    t -= sub * per_sub;
    sgn = SG;
  } else {
    t -= full * per_sub;
    sub = full;
    sgn = gcount - full * SG;
    if (sgn <= 0 || t >= sgn * g.nz * nxc) return -1;
  }
  const int k = t / (sgn * nxc);
  const int rem = t - k * (sgn * nxc);
  const int gg = g0 + sub * SG + rem / nxc, c = rem % nxc;
  const int i = c * TX + (int)(threadIdx.x % TX), j = gg * LPB + (int)(threadIdx.x / TX);
  if (i >= g.nx || j >= g.ny) return -1;
  ii = i;
  jj = j;
  kk = k;
  return i + j * g.nx + k * g.nx * g.ny;
}

// ---------------------------------------------------------------------------- BC on u
// apply_bc_on_u -> bc_apply_on_u_circle / _bending (src/bcs.c:29-146)
__global__ void k_apply_bc_u(Geo g, double* __restrict__ u, double U) {
  int n = blockIdx.x * TPB + threadIdx.x;
  if (n >= g.nown) return;
  int i, j, k;
  node_ijk(g, n, i, j, k);
  int gi = g.xs + i, gj = g.ys + j, gk = g.zs + k;
  int m = dirichlet_mask(g, gi, gj, gk);
  if (!m) return;
  int pc = pad_of(g, i, j, k);
  for (int d = 0; d < 3; d++) {
    if (!(m >> d & 1)) continue;
    double v;
    if (g.bc_type == MCX_BC_CIRCLE) v = (m == 2) ? U : 0.;
    else v = (gi == g.NX - 1 && d == 1) ? U : 0.;
    u[3 * pc + d] = v;
  }
}

// ---------------------------------------------------------------------------- strains
// set_strains (src/assembly.c:25-66): eps_gp = B_gp . u_e; zero B entries skipped (adding
// +-0 is exact, so the sum is bit-identical to the reference's full 24-term loop).
__global__ void k_strains(Geo g, const double* __restrict__ u, double* __restrict__ eps) {
  int64_t le = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (le >= g.nelem) return;
  int lex = (int)(le % g.nex), t = (int)(le / g.nex), ley = t % g.ney, lez = t / g.ney;
  int ex = g.ex0 + lex, ey = g.ey0 + ley, ez = g.ez0 + lez;
  const int PXY = g.PX * g.PY;
  int p0 = (ex - g.xs + 1) + (ey - g.ys + 1) * g.PX + (ez - g.zs + 1) * PXY;
  const int noff[8] = {0, 1, 1 + g.PX, g.PX, PXY, 1 + PXY, 1 + g.PX + PXY, g.PX + PXY};
  double ue[24];
#pragma unroll
  for (int a = 0; a < 8; a++)
#pragma unroll
    for (int d = 0; d < 3; d++) ue[3 * a + d] = u[3 * (p0 + noff[a]) + d];
  const int64_t E = g.nelem;
#pragma unroll
  for (int gp = 0; gp < 8; gp++) {
#pragma unroll
    for (int kk = 0; kk < 6; kk++) {
      double s = 0.;
#pragma unroll
      for (int jj = 0; jj < 24; jj++) {
        const int d = jj % 3;
        const bool nz = (kk < 3) ? (d == kk) : (kk == 3 ? d != 2 : (kk == 4 ? d != 1 : d != 0));
        if (nz) s += cB[gp][kk][jj] * ue[jj];
      }
      eps[((int64_t)kk * 8 + gp) * E + le] = s;
    }
  }
}

// VTU cell data (write_pvtu src/output.c:180-248) for the rank's own elements as PETSc lists
// them ([lo, lo+cnt) per axis, x fastest): out[13 e + 0..5] = sum_gp wg * (B_gp u_e) recomputed
// from u (:204-223, strain_gp summed like set_strains), [6..11] = sum_gp wg * sigma_gp
// (:232-240), [12] = non-linear GPs (f_trial > 0, micropp_C_is_non_linear :197-201)
__global__ void k_vtu_cells(Geo g, const double* __restrict__ u, const double* __restrict__ sig,
                            const double* __restrict__ ftrial, int lx0, int ly0, int lz0, int cx, int cy, int cz,
                            double* __restrict__ out) {
  const int64_t e = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (e >= (int64_t)cx * cy * cz) return;
  const int ex = lx0 + (int)(e % cx), ey = ly0 + (int)((e / cx) % cy), ez = lz0 + (int)(e / ((int64_t)cx * cy));
  const int64_t le = (ex - g.ex0) + (int64_t)(ey - g.ey0) * g.nex + (int64_t)(ez - g.ez0) * g.nex * g.ney;
  const int PXY = g.PX * g.PY;
  const int p0 = (ex - g.xs + 1) + (ey - g.ys + 1) * g.PX + (ez - g.zs + 1) * PXY;
  const int noff[8] = {0, 1, 1 + g.PX, g.PX, PXY, 1 + PXY, 1 + g.PX + PXY, g.PX + PXY};
  double ue[24];
#pragma unroll
  for (int a = 0; a < 8; a++)
#pragma unroll
    for (int d = 0; d < 3; d++) ue[3 * a + d] = u[3 * (p0 + noff[a]) + d];
  double strain[6] = {0., 0., 0., 0., 0., 0.}, stress[6] = {0., 0., 0., 0., 0., 0.};
  int nl = 0;
  for (int gp = 0; gp < 8; gp++) {
#pragma unroll
    for (int kk = 0; kk < 6; kk++) {
      double s = 0.;
#pragma unroll
      for (int jj = 0; jj < 24; jj++) {
        const int d = jj % 3;
        const bool nz = (kk < 3) ? (d == kk) : (kk == 3 ? d != 2 : (kk == 4 ? d != 1 : d != 0));
        if (nz) s += cB[gp][kk][jj] * ue[jj];
      }
      strain[kk] += s * g.wg;
      stress[kk] += sig[((int64_t)kk * 8 + gp) * g.nelem + le] * g.wg;
    }
    if (ftrial && ftrial[(int64_t)gp * g.nelem + le] > 0.) nl++;
  }
#pragma unroll
  for (int kk = 0; kk < 6; kk++) {
    out[13 * e + kk] = strain[kk];
    out[13 * e + 6 + kk] = stress[kk];
  }
  out[13 * e + 12] = nl;
}

// ---------------------------------------------------------------------------- material
// Gauss-point callback, isotropic linear elastic (MicroPP surrogate): sigma = C eps per Gauss
// point (micropp_C_homogenize / get_stress3).  The tangent is the constant C (get_ctan3): the
// Jacobian evaluates it from the kernel argument, so no per-GP tangent array exists.
__global__ void k_homogenize_elastic(int64_t ngp, Material mat, const double* __restrict__ eps,
                                     double* __restrict__ sig) {
  int64_t q = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (q >= ngp) return;
  double e[6];
#pragma unroll
  for (int l = 0; l < 6; l++) e[l] = eps[l * ngp + q];
#pragma unroll
  for (int k = 0; k < 6; k++) {
    double s = 0.;
#pragma unroll
    for (int l = 0; l < 6; l++) s += mat.C[k * 6 + l] * e[l];
    sig[k * ngp + q] = s;
  }
}

__device__ __forceinline__ void j2_moduli(const Material& mat, double& G, double& K) {
  G = mat.E / (2. * (1. + mat.nu));
  K = mat.E / (3. * (1. - 2. * mat.nu));
}

// the J2 law's tangent on its elastic branch (f <= 0): every such Gauss point gets these bits
__device__ __forceinline__ void j2_elastic_tangent(double G, double K, double (&C)[36]) {
  const double lam = K - 2. * G / 3.;
#pragma unroll
  for (int k2 = 0; k2 < 36; k2++) C[k2] = 0.;
#pragma unroll
  for (int a = 0; a < 3; a++)
#pragma unroll
    for (int b = 0; b < 3; b++) C[a * 6 + b] = lam + (a == b ? 2. * G : 0.);
#pragma unroll
  for (int a = 3; a < 6; a++) C[a * 6 + a] = G;
}

// small-strain J2 plasticity with linear isotropic hardening (MicroPP material type 1: E, nu,
// Sy, Ka), radial return + consistent tangent; same operation order as orc_j2_point (oracle).
__global__ void k_homogenize_plastic(int64_t ngp, Material mat, const double* __restrict__ eps,
                                     const double* __restrict__ hold, double* __restrict__ sig,
                                     double* __restrict__ ctan, double* __restrict__ hnew,
                                     double* __restrict__ ftrial) {
  int64_t q = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (q >= ngp) return;
  const double Sy = mat.Sy, Ka = mat.Ka;
  double G, K;
  j2_moduli(mat, G, K);
  double e[6], h[7];
#pragma unroll
  for (int l = 0; l < 6; l++) e[l] = eps[l * ngp + q];
#pragma unroll
  for (int l = 0; l < 7; l++) h[l] = hold[l * ngp + q];
  const double tr = e[0] + e[1] + e[2];
  double dev[6], st[6];
#pragma unroll
  for (int i = 0; i < 3; i++) dev[i] = e[i] - tr / 3.;
#pragma unroll
  for (int i = 3; i < 6; i++) dev[i] = e[i] / 2.;
#pragma unroll
  for (int i = 0; i < 6; i++) st[i] = 2. * G * (dev[i] - h[i]);
  double nrm2 = st[0] * st[0] + st[1] * st[1] + st[2] * st[2];
  nrm2 = nrm2 + 2. * (st[3] * st[3] + st[4] * st[4] + st[5] * st[5]);
  const double snorm = sqrt(nrm2);
  const double alpha = h[6];
  const double f = snorm - sqrt(2. / 3.) * (Sy + Ka * alpha);
  ftrial[q] = f;
  double C[36], s[6];
  j2_elastic_tangent(G, K, C);
  if (f <= 0.) {
#pragma unroll
    for (int i = 0; i < 3; i++) s[i] = K * tr + st[i];
#pragma unroll
    for (int i = 3; i < 6; i++) s[i] = st[i];
#pragma unroll
    for (int i = 0; i < 7; i++) hnew[i * ngp + q] = h[i];
  } else {
    const double dg = f / (2. * G + 2. / 3. * Ka);
    double n[6];
#pragma unroll
    for (int i = 0; i < 6; i++) n[i] = st[i] / snorm;
#pragma unroll
    for (int i = 0; i < 3; i++) s[i] = K * tr + (st[i] - 2. * G * dg * n[i]);
#pragma unroll
    for (int i = 3; i < 6; i++) s[i] = st[i] - 2. * G * dg * n[i];
#pragma unroll
    for (int i = 0; i < 6; i++) hnew[i * ngp + q] = h[i] + dg * n[i];
    hnew[6 * ngp + q] = alpha + sqrt(2. / 3.) * dg;
    const double theta = 1. - 2. * G * dg / snorm;
    const double thetab = 1. / (1. + Ka / (3. * G)) - (1. - theta);
#pragma unroll
    for (int a = 0; a < 3; a++)
#pragma unroll
      for (int b = 0; b < 3; b++) C[a * 6 + b] = K + 2. * G * theta * ((a == b ? 1. : 0.) - 1. / 3.);
#pragma unroll
    for (int a = 3; a < 6; a++) C[a * 6 + a] = G * theta;
#pragma unroll
    for (int a = 0; a < 6; a++)
#pragma unroll
      for (int b = 0; b < 6; b++) C[a * 6 + b] = C[a * 6 + b] - 2. * G * thetab * n[a] * n[b];
  }
#pragma unroll
  for (int k2 = 0; k2 < 6; k2++) sig[k2 * ngp + q] = s[k2];
#pragma unroll
  for (int kl = 0; kl < 36; kl++) ctan[kl * ngp + q] = C[kl];
}

// ---------------------------------------------------------------------------- residual
// rows k of B with B[k][3a+r] != 0, ascending: K(0) = {0,3,4}, K(1) = {1,3,5}, K(2) = {2,4,5}
__device__ __forceinline__ constexpr int krow(int r, int q) { return q == 0 ? r : (r == 1 ? (q == 1 ? 3 : 5) : 3 + q - (r == 0)); }
// position of row k in K(r) (k in K(r))
__device__ __forceinline__ constexpr int kpos(int r, int k) { return k == r ? 0 : ((k == 3 || (k == 4 && r == 2)) ? 1 : 2); }
__device__ __forceinline__ constexpr bool kin(int r, int k) {
  return k == r || (r == 0 && (k == 3 || k == 4)) || (r == 1 && (k == 3 || k == 5)) || (r == 2 && (k == 4 || k == 5));
}

// assembly_res (src/assembly.c:120-176) node by node, without an element-vector array: the
// node's rows are 0 + be_e1 + be_e2 + ... over its elements in ascending element order (the
// order the reference's element loop adds into b_loc, :156-161), each be[3a+r] = sum_gp sum_j
// B[j][3a+r] * sigma_j * wg evaluated on the fly (gp outer, j ascending, :145-154; zero B terms
// skipped, exact); Dirichlet rows zeroed (apply_bc_on_res), then VecScale(b,-1) (:171-173).
// The element loop runs over the node's local offset (ox, oy, oz) in the element, descending =
// ascending element index, so the local node number a is wave-uniform (scalar B loads).
// Emits per-block partial sums of b.b for VecNorm.
__global__ __launch_bounds__(TPB) void k_residual(Geo g, const double* __restrict__ sig, double* __restrict__ b,
                                                  double* __restrict__ part) {
  __shared__ double sh[TPB / 64];
  const int n = blockIdx.x * TPB + threadIdx.x;
  double nrm = 0.;
  if (n < g.nown) {
    int i, j, k;
    node_ijk(g, n, i, j, k);
    const int gi = g.xs + i, gj = g.ys + j, gk = g.zs + k;
    const int64_t E = g.nelem, NG = 8 * E;
    double acc[3] = {0., 0., 0.};
    for (int oz = 1; oz >= 0; oz--) {
      const int ez = gk - oz;
      if (ez < 0 || ez > g.NZ - 2) continue;
      for (int oy = 1; oy >= 0; oy--) {
        const int ey = gj - oy;
        if (ey < 0 || ey > g.NY - 2) continue;
        for (int ox = 1; ox >= 0; ox--) {
          const int ex = gi - ox;
          if (ex < 0 || ex > g.NX - 2) continue;
          const int64_t le = (ex - g.ex0) + (int64_t)(ey - g.ey0) * g.nex + (int64_t)(ez - g.ez0) * g.nex * g.ney;
          const int a = q1_local(ox, oy, oz);
          double be[3] = {0., 0., 0.};
          for (int gp = 0; gp < 8; gp++) {
#pragma unroll
            for (int r = 0; r < 3; r++)
#pragma unroll
              for (int q = 0; q < 3; q++) {
                const int kk = krow(r, q);
                be[r] += cB[gp][kk][3 * a + r] * sig[kk * NG + gp * E + le] * g.wg;
              }
          }
#pragma unroll
          for (int r = 0; r < 3; r++) acc[r] += be[r];
        }
      }
    }
    const int m = dirichlet_mask(g, gi, gj, gk);
#pragma unroll
    for (int r = 0; r < 3; r++) {
      double v = (m >> r & 1) ? 0. : acc[r];
      v = v * -1.;
      b[3 * n + r] = v;
      nrm += v * v;
    }
  }
  const double s = block_sum<TPB>(nrm, sh);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

// ---------------------------------------------------------------------------- Jacobian
// Element-matrix block Ke[3a+r][3bn+c] (r, c = 0..2) of element le, evaluated on the fly for the
// isotropic elastic law (C from the kernel argument, no per-GP tangent array): assembly_jac's
// 4-nest (src/assembly.c:94-99) restricted to the block, Ke[i][j] += B[k][i]*C[k][l]*B[l][j]*wg
// with gp, k, l ascending, as ((B*C)*B)*wg.  Zero B terms and C's structural zeros are skipped:
// each skipped term is +-0 added to a sum that is never -0, so the block is bit-identical to the
// full loop.  a, bn are wave-uniform.
__device__ __forceinline__ void ke_block(const Geo& g, const Material& mat, int a, int bn, double (&ke)[9]) {
#pragma unroll
  for (int q = 0; q < 9; q++) ke[q] = 0.;
  const double wg = g.wg;
  for (int gp = 0; gp < 8; gp++) {
    double Ba[3][3], Bb[3][3];
#pragma unroll
    for (int r = 0; r < 3; r++)
#pragma unroll
      for (int q = 0; q < 3; q++) {
        Ba[r][q] = cB[gp][krow(r, q)][3 * a + r];
        Bb[r][q] = cB[gp][krow(r, q)][3 * bn + r];
      }
#pragma unroll
    for (int k = 0; k < 6; k++)
#pragma unroll
      for (int l = 0; l < 6; l++) {
        if (!((k < 3 && l < 3) || k == l)) continue;
        const double Ckl = mat.C[k * 6 + l];
#pragma unroll
        for (int r = 0; r < 3; r++) {
          if (!kin(r, k)) continue;
          const double t0 = Ba[r][kpos(r, k)] * Ckl;
#pragma unroll
          for (int c = 0; c < 3; c++) {
            if (!kin(c, l)) continue;
            ke[r * 3 + c] += t0 * Bb[c][kpos(c, l)] * wg;
          }
        }
      }
  }
}

// Laws with a per-GP tangent (plastic, external): the element matrices are formed once into
// Ke[576][elements] (each C_tan read once per element and thread group, not once per matrix
// block) and the blocks are summed from there.  Same 4-nest and term order as ke_block, all
// 36 C entries.  One thread = (element, node a, half of the column nodes b): 4 column blocks x
// 9 = 36 accumulators.  Grid: blocks b -> (XCD group, a, half, element group) so the 16 blocks
// that read one element group's ctan share an XCD's L2.
template <int BH>
__device__ __forceinline__ void ke_body(const Geo& g, int64_t le, int a, const double* __restrict__ ctan,
                                        double* __restrict__ Ke) {
  const int64_t E = g.nelem, NG = 8 * E;
  double acc[4][9];
#pragma unroll
  for (int bb = 0; bb < 4; bb++)
#pragma unroll
    for (int q = 0; q < 9; q++) acc[bb][q] = 0.;
  const double wg = g.wg;
  for (int gp = 0; gp < 8; gp++) {
    double Ba[3][3];
#pragma unroll
    for (int r = 0; r < 3; r++)
#pragma unroll
      for (int q = 0; q < 3; q++) Ba[r][q] = cB[gp][krow(r, q)][3 * a + r];
#pragma unroll
    for (int k = 0; k < 6; k++) {
#pragma unroll
      for (int l = 0; l < 6; l++) {
        const double Ckl = ctan[(k * 6 + l) * NG + gp * E + le];
#pragma unroll
        for (int r = 0; r < 3; r++) {
          if (!kin(r, k)) continue;
          const double t0 = Ba[r][kpos(r, k)] * Ckl;
#pragma unroll
          for (int c = 0; c < 3; c++) {
            if (!kin(c, l)) continue;
#pragma unroll
            for (int bb = 0; bb < 4; bb++) acc[bb][r * 3 + c] += t0 * cB[gp][l][3 * (BH * 4 + bb) + c] * wg;
          }
        }
      }
    }
  }
#pragma unroll
  for (int bb = 0; bb < 4; bb++)
#pragma unroll
    for (int q = 0; q < 9; q++) Ke[((int64_t)(a * 8 + BH * 4 + bb) * 9 + q) * E + le] = acc[bb][q];
}

// plain (optional): skip the elements whose tangent is the reference tangent (their matrix is
// kref, formed once by k_ref_ke)
__global__ __launch_bounds__(TPB) void k_element_ke(Geo g, const double* __restrict__ ctan, double* __restrict__ Ke,
                                                    int64_t ngroups, const unsigned char* __restrict__ plain) {
  // block -> (xcd, a, half, element group): blocks sharing an element group are 8 apart
  const int64_t b = blockIdx.x;
  const int x = (int)(b & 7);
  const int64_t t = b >> 3;
  const int ah = (int)(t & 15);
  const int64_t grp = (t >> 4) * 8 + x;
  if (grp >= ngroups) return;
  const int64_t le = grp * TPB + threadIdx.x;
  if (le >= g.nelem || (plain && plain[le])) return;
  const int a = ah >> 1;
  if (ah & 1) ke_body<1>(g, le, a, ctan, Ke);
  else ke_body<0>(g, le, a, ctan, Ke);
}

// The isotropic elastic law has one tangent C for every Gauss point, and the uniform grid one
// element shape (unit-cube B, one wg), so every element's matrix is the same 24x24 Ke: its 64
// blocks (a, bn) are evaluated once per assembly by ke_block — the arithmetic each element's
// on-the-fly evaluation would repeat, so the assembled values are bit-identical — into
// ke_uni[(a*8 + bn)*9 + r*3 + c], which matrix_block<false> then sums (a, bn wave-uniform: scalar
// loads).  Round 2 re-evaluated ke_block for every element block of every assembled block.
__global__ void k_elastic_ke(Geo g, Material mat, double* __restrict__ keu) {
  const int t = threadIdx.x;
  if (t >= 64) return;
  double ke[9];
  ke_block(g, mat, t >> 3, t & 7, ke);
#pragma unroll
  for (int q = 0; q < 9; q++) keu[t * 9 + q] = ke[q];
}

// One 3x3 block A(node g, node g+d) of the assembled matrix (MatSetValuesLocal(ADD) +
// MatAssembly + MatZeroRowsColumns(diag = 1), src/assembly.c:106-112, src/bcs.c:341-347):
// 0 + Ke_e1 + Ke_e2 + ... over the shared elements in ascending element order (the reference's
// insertion order on one rank), each element block read from the elastic law's one element
// matrix (Ke = ke_uni) or from the element matrices (TABLE: laws with a per-GP tangent, Ke =
// [576][nelem]), then the Dirichlet rows / columns.
template <bool TABLE>
__device__ __forceinline__ void matrix_block(const Geo& g, const Material& mat, const double* __restrict__ Ke,
                                             int gi, int gj, int gk, int dx, int dy, int dz, double (&val)[9],
                                             const double* __restrict__ kref = nullptr,
                                             const unsigned char* __restrict__ plain = nullptr) {
  const int hi = gi + dx, hj = gj + dy, hk = gk + dz;
#pragma unroll
  for (int q = 0; q < 9; q++) val[q] = 0.;
  if (gi < 0 || gj < 0 || gk < 0 || gi >= g.NX || gj >= g.NY || gk >= g.NZ) return;
  if (hi < 0 || hj < 0 || hk < 0 || hi >= g.NX || hj >= g.NY || hk >= g.NZ) return;
  for (int oz = 1; oz >= 0; oz--) {
    const int pz = oz + dz, ez = gk - oz;
    if (pz < 0 || pz > 1 || ez < 0 || ez > g.NZ - 2) continue;
    for (int oy = 1; oy >= 0; oy--) {
      const int py = oy + dy, ey = gj - oy;
      if (py < 0 || py > 1 || ey < 0 || ey > g.NY - 2) continue;
      for (int ox = 1; ox >= 0; ox--) {
        const int px = ox + dx, ex = gi - ox;
        if (px < 0 || px > 1 || ex < 0 || ex > g.NX - 2) continue;
        const int64_t le = (ex - g.ex0) + (int64_t)(ey - g.ey0) * g.nex + (int64_t)(ez - g.ez0) * g.nex * g.ney;
        const int a = q1_local(ox, oy, oz), bn = q1_local(px, py, pz);
        if constexpr (TABLE) {  // element matrices formed by k_element_ke (plain ones: kref)
          const bool ref = plain && plain[le];
          const double* src = ref ? kref + (a * 8 + bn) * 9 : Ke + (int64_t)((a * 8 + bn) * 9) * g.nelem + le;
          const int64_t st = ref ? 1 : g.nelem;
#pragma unroll
          for (int q = 0; q < 9; q++) val[q] += src[q * st];
        } else {  // the elastic law's one element matrix (k_elastic_ke: ke_block of every (a, bn))
          const double* src = Ke + (a * 8 + bn) * 9;
#pragma unroll
          for (int q = 0; q < 9; q++) val[q] += src[q];
        }
      }
    }
  }
  const int rm = dirichlet_mask(g, gi, gj, gk), cm = dirichlet_mask(g, hi, hj, hk);
  const bool self = !dx && !dy && !dz;
#pragma unroll
  for (int r = 0; r < 3; r++)
#pragma unroll
    for (int c = 0; c < 3; c++) {
      if (rm >> r & 1) val[r * 3 + c] = (self && r == c) ? 1.0 : 0.0;
      else if (cm >> c & 1) val[r * 3 + c] = 0.0;
    }
}

// AIJ stencil blocks: thread = (owned node, neighbour block nb)
template <bool TABLE>
__global__ __launch_bounds__(TPB) void k_gather_matrix(Geo g, Material mat, const double* __restrict__ Ke,
                                                       double* __restrict__ V) {
  const int n = blockIdx.x * TPB + threadIdx.x;
  const int nb = blockIdx.y;
  if (n >= g.nown) return;
  int i, j, k;
  node_ijk(g, n, i, j, k);
  double val[9];
  matrix_block<TABLE>(g, mat, Ke, g.xs + i, g.ys + j, g.zs + k, nb % 3 - 1, (nb / 3) % 3 - 1, nb / 9 - 1, val);
  double* Vg = V + (int64_t)(n >> 6) * (NPAIR * 128) + 2 * (n & 63);
#pragma unroll
  for (int q = 0; q < 9; q++) {
    const int s = nb * 9 + q;
    Vg[(s >> 1) * 128 + (s & 1)] = val[q];
  }
}

// sbaij storage (PETSc MATSBAIJ semantics): for every node of the padded box the upper
// triangle of its diagonal block (6 values) and its 13 upper neighbour blocks (nb > 13 =
// larger natural index).  Ghost-layer nodes store only the blocks pointing at owned nodes
// (the mirrors the owned rows need); owner-computes covers them (every element shared by a
// ghost and an owned node touches the owned node).  Thread = (padded node, t): t = 0 the
// diagonal block, t = 1..13 upper block nb = 13 + t.
template <bool TABLE>
__global__ __launch_bounds__(TPB) void k_gather_matrix_sym(Geo g, Material mat, const double* __restrict__ Ke,
                                                           double* __restrict__ U, int npad) {
  const int p = blockIdx.x * TPB + threadIdx.x;
  const int t = blockIdx.y;
  if (p >= npad) return;
  const int pi = p % g.PX, pj = (p / g.PX) % g.PY, pk = p / (g.PX * g.PY);
  const int nb = 13 + t;
  const int dx = nb % 3 - 1, dy = (nb / 3) % 3 - 1, dz = nb / 9 - 1;
  const bool owned = pi >= 1 && pi <= g.nx && pj >= 1 && pj <= g.ny && pk >= 1 && pk <= g.nz;
  const int qi = pi + dx, qj = pj + dy, qk = pk + dz;
  const bool nbr_owned = qi >= 1 && qi <= g.nx && qj >= 1 && qj <= g.ny && qk >= 1 && qk <= g.nz;
  double val[9];
  if (owned || (t > 0 && nbr_owned)) {
    matrix_block<TABLE>(g, mat, Ke, g.xs + pi - 1, g.ys + pj - 1, g.zs + pk - 1, dx, dy, dz, val);
  } else {
#pragma unroll
    for (int q = 0; q < 9; q++) val[q] = 0.;
  }
  const int pu = u_of(g, pi - 1, pj - 1, pk - 1);
  double* Ug = U + (int64_t)(pu >> 6) * (UPAIR * 128) + 2 * (pu & 63);
  if (t == 0) {
    const double up[6] = {val[0], val[1], val[2], val[4], val[5], val[8]};
#pragma unroll
    for (int s = 0; s < 6; s++) Ug[(s >> 1) * 128 + (s & 1)] = up[s];
  } else {
#pragma unroll
    for (int q = 0; q < 9; q++) {
      const int s = 6 + 9 * (t - 1) + q;
      Ug[(s >> 1) * 128 + (s & 1)] = val[q];
    }
  }
}

// AIJ-split corrections of one owned node and lower block nb < 13 (nb = 13: the diagonal
// block's strictly-lower entries against their mirrors): the AIJ value A(n,nb)[r][c]
// (matrix_block, exactly what k_gather_matrix stores) minus the mirrored upper value
// U(m, 26-nb)[c][r] of the neighbour m = n + off(nb), as f32 bits (bit q = r*3+c in *valid).
template <bool TABLE>
__device__ __forceinline__ void split_block(const Geo& g, const Material& mat, const double* __restrict__ Ke,
                                            const double* __restrict__ U, int n, int nb, unsigned (&f32)[9],
                                            unsigned& bits, unsigned& bad, unsigned& esc,
                                            double* __restrict__ dout = nullptr) {
  int i, j, k;
  node_ijk(g, n, i, j, k);
  bits = bad = 0;
  double low[9], mir[9];
  if (nb == 13) {
    matrix_block<TABLE>(g, mat, Ke, g.xs + i, g.ys + j, g.zs + k, 0, 0, 0, low);
#pragma unroll
    for (int r = 0; r < 3; r++)
#pragma unroll
      for (int c = 0; c < 3; c++) mir[r * 3 + c] = r > c ? low[c * 3 + r] : low[r * 3 + c];
  } else {
    const int dx = nb % 3 - 1, dy = (nb / 3) % 3 - 1, dz = nb / 9 - 1;
    matrix_block<TABLE>(g, mat, Ke, g.xs + i, g.ys + j, g.zs + k, dx, dy, dz, low);
    const int um = u_of(g, i + dx, j + dy, k + dz);
    const double* Um = U + (int64_t)(um >> 6) * (UPAIR * 128) + 2 * (um & 63);
    const int base = 6 + 9 * (12 - nb);  // the neighbour's upper block 26 - nb
#pragma unroll
    for (int r = 0; r < 3; r++)
#pragma unroll
      for (int c = 0; c < 3; c++) {
        const int s = base + c * 3 + r;
        mir[r * 3 + c] = Um[(s >> 1) * 128 + (s & 1)];
      }
  }
  esc = 0u;
#pragma unroll
  for (int q = 0; q < 9; q++) {
    const double d = low[q] - mir[q];
    if (dout) dout[q] = d;
    f32[q] = __float_as_uint((float)d);
    const unsigned fb = f32[q] & 0xffff0000u;
    const double df = (double)__uint_as_float(f32[q]), db = (double)__uint_as_float(fb);
    const bool strict = nb != 13 || q == 3 || q == 6 || q == 7;
    if (db != d || mir[q] + db != low[q]) {
      bad |= 1;  // not exact in bf16
      // escape (dense bf16 corrections): the truncated bf16 hi plus the exact double residual
      // d - hi, reconstructing the AIJ value as mirror + (hi + residual)
      if (strict) {
        if (db + (d - db) == d && mir[q] + d == low[q]) esc |= 1u << q;
        else bad |= 4;
      }
    }
    if (df != d || mir[q] + df != low[q]) bad |= 2;  // not exact in f32
    if (d != 0.) bits |= 1u << q;
  }
  if (nb == 13) bits &= (1u << 3) | (1u << 6) | (1u << 7);  // strictly lower: (1,0), (2,0), (2,1)
}

// AIJ-split assembly, pass 1: thread = (owned node, lower block nb <= 13); d_mask[nb] collects
// the correction slots that are non-zero anywhere, d_mask[14] bit 0 = some correction inexact
// in bf16, bit 1 = inexact in f32 (then the matrix is stored as plain AIJ blocks).
template <bool TABLE>
__global__ __launch_bounds__(TPB) void k_split_mask(Geo g, Material mat, const double* __restrict__ Ke,
                                                    const double* __restrict__ U, unsigned* __restrict__ mask,
                                                    unsigned* __restrict__ eflag) {
  __shared__ unsigned s_bits, s_bad;
  if (threadIdx.x == 0) s_bits = s_bad = 0;
  __syncthreads();
  const int n = blockIdx.x * TPB + threadIdx.x;
  const int nb = blockIdx.y;
  if (n < g.nown) {
    unsigned f32[9], bits, bad, esc;
    split_block<TABLE>(g, mat, Ke, U, n, nb, f32, bits, bad, esc);
    if (bits) atomicOr(&s_bits, bits);
    if (bad) atomicOr(&s_bad, bad);
    if (esc) {  // dense bf16 corrections with escapes: count them, flag the node
      atomicAdd(&mask[15], (unsigned)__builtin_popcount(esc));
      if (eflag) eflag[n] = 1u;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    if (s_bits) atomicOr(&mask[nb], s_bits);
    if (s_bad) atomicOr(&mask[14], s_bad);
  }
}

// AIJ-split assembly, pass 2: the same corrections recomputed and written to their packed
// positions (slot p of node u = u_of: D[(((u/64) * Lq + p/8) * 64 + u%64) * 8 + p%8] as bf16,
// or 4 f32 per quad); D is zeroed first (ghost nodes and padding hold zeros).
template <bool TABLE>
__global__ __launch_bounds__(TPB) void k_split_pack(Geo g, Material mat, const double* __restrict__ Ke,
                                                    const double* __restrict__ U, uint16_t* __restrict__ D, DSlots dl) {
  const int n = blockIdx.x * TPB + threadIdx.x;
  const int nb = blockIdx.y;
  const unsigned m9 = dl.m9[nb];
  if (n >= g.nown || !m9) return;
  unsigned f32[9], bits, bad, esc;
  split_block<TABLE>(g, mat, Ke, U, n, nb, f32, bits, bad, esc);
  int i, j, k;
  node_ijk(g, n, i, j, k);
  const int64_t u = u_of(g, i, j, k);
  int p = dl.pos[nb];
#pragma unroll
  for (int q = 0; q < 9; q++) {
    if (!(m9 >> q & 1)) continue;
    if (dl.wide) {
      reinterpret_cast<unsigned*>(D)[((((u >> 6) * dl.Lq + p / 4) * 64 + (u & 63)) * 4) + p % 4] = f32[q];
    } else {
      D[((((u >> 6) * dl.Lq + p / 8) * 64 + (u & 63)) * 8) + p % 8] = (uint16_t)(f32[q] >> 16);
    }
    p++;
  }
}

// AIJ-split, dense bf16 corrections with escapes: for every node flagged by k_split_mask (a
// correction not exact in bf16), its escaped slots' residuals d - hi in slot order (lower block nb
// ascending, then r*3 + c) at a base taken from an atomic counter: esc_node[n] = count << 24 |
// (base + 1).  The base order varies run to run, a node's entries and their order do not.
template <bool TABLE>
__global__ __launch_bounds__(TPB) void k_split_esc(Geo g, Material mat, const double* __restrict__ Ke,
                                                   const double* __restrict__ U, unsigned* __restrict__ eflag,
                                                   unsigned* __restrict__ cnt, unsigned cap, double* __restrict__ esc_res,
                                                   unsigned char* __restrict__ esc_slot) {
  const int n = blockIdx.x * TPB + threadIdx.x;
  if (n >= g.nown || !eflag[n]) return;
  unsigned m = 0;  // pass 1: the node's escapes (rare: recomputing its blocks twice is cheap)
  for (int nb = 0; nb < 14; nb++) {
    unsigned f32[9], bits, bad, esc;
    split_block<TABLE>(g, mat, Ke, U, n, nb, f32, bits, bad, esc);
    m += __builtin_popcount(esc);
  }
  const unsigned base = atomicAdd(cnt, m);
  if (base + m > cap || m > 126u) {  // more escapes than the host sized for: build_split reads the
    eflag[n] = 0xffffffffu;          // counter back and falls back to AIJ blocks (never dereferenced)
    return;
  }
  unsigned t = base;
  for (int nb = 0; nb < 14; nb++) {  // pass 2: residuals d - hi in slot order
    unsigned f32[9], bits, bad, esc;
    double d[9];
    split_block<TABLE>(g, mat, Ke, U, n, nb, f32, bits, bad, esc, d);
    for (int q = 0; q < 9; q++) {
      if (!(esc >> q & 1u)) continue;
      const double hi = (double)__uint_as_float(f32[q] & 0xffff0000u);
      esc_res[t] = d[q] - hi;
      esc_slot[t] = (unsigned char)(nb * 9 + q);
      t++;
    }
  }
  eflag[n] = m << 24 | (base + 1u);
}

// PCSetUp_Jacobi: diag, VecReciprocal (non-zeros only), zeros -> 1
__global__ void k_jacobi(Geo g, const double* __restrict__ V, double* __restrict__ dinv) {
  int n = blockIdx.x * TPB + threadIdx.x;
  if (n >= g.nown) return;
  const double* Vg = V + (int64_t)(n >> 6) * (NPAIR * 128) + 2 * (n & 63);
#pragma unroll
  for (int r = 0; r < 3; r++) {
    const int s = 13 * 9 + r * 4;
    double d = Vg[(s >> 1) * 128 + (s & 1)];
    if (d != 0.0) d = 1.0 / d;
    if (d == 0.0) d = 1.0;
    dinv[3 * n + r] = d;
  }
}

__global__ void k_jacobi_sym(Geo g, const double* __restrict__ U, double* __restrict__ dinv) {
  int n = blockIdx.x * TPB + threadIdx.x;
  if (n >= g.nown) return;
  int i, j, k;
  node_ijk(g, n, i, j, k);
  const int pu = u_of(g, i, j, k);
  const double* Ug = U + (int64_t)(pu >> 6) * (UPAIR * 128) + 2 * (pu & 63);
  const int sl[3] = {0, 3, 5};
#pragma unroll
  for (int r = 0; r < 3; r++) {
    double d = Ug[(sl[r] >> 1) * 128 + (sl[r] & 1)];
    if (d != 0.0) d = 1.0 / d;
    if (d == 0.0) d = 1.0;
    dinv[3 * n + r] = d;
  }
}

// ---------------------------------------------------------------------------- SpMV
// The exact SpMV kernels sum every row in the order of the kernel the reference's MatMult runs:
// PETSc's MatMult_SeqAIJ_Inode [ext] (src/mat/impls/aij/seq/inode.c; MatSeqAIJCheckInode makes
// the 3 rows of a DMDA node, dof 3, one inode of the reference's MATAIJ, src/init.c:85-95), whose
// unrolled loop adds a row's terms t = a x in column pairs, y = 0 + (t0 + t1) + (t2 + t3) + ...
// [+ t_last], over the row's stored columns in ascending order (oracle/oracle.c row_part).  A
// row's columns are its node's neighbours inside the global domain (the DMDA stencil is clipped
// there; MatZeroRowsColumns' zeros stay in the pattern), three per neighbour block, ascending
// (nb, c) = ascending global column on one rank.  So column c of block nb sits at position
// 3 q + c, q = the present blocks before nb, and its term either opens a pair (even position:
// held in e) or closes one (odd: s + (e + t)).  Blocks outside the domain (zero values, zero
// ghost x) are skipped: an added +0 would shift the pairing of every column after it.
// present_mask: bit nb set when neighbour nb = (dz+1)*9 + (dy+1)*3 + (dx+1) of owned node
// (i, j, k) lies inside the global domain (any rank grid: internal faces' ghosts are present).
constexpr unsigned PRES_ALL = (1u << 27) - 1u;
__device__ __forceinline__ unsigned present_mask(const Geo& g, int i, int j, int k) {
  const int gi = g.xs + i, gj = g.ys + j, gk = g.zs + k;
  const unsigned mx = 2u | (gi > 0 ? 1u : 0u) | (gi < g.NX - 1 ? 4u : 0u);
  const unsigned my = 2u | (gj > 0 ? 1u : 0u) | (gj < g.NY - 1 ? 4u : 0u);
  const unsigned mz = 2u | (gk > 0 ? 1u : 0u) | (gk < g.NZ - 1 ? 4u : 0u);
  const unsigned xb = mx * 0x1249249u;  // bit nb: dx = nb % 3 present (mx replicated every 3 bits)
  const unsigned y9 = ((my & 1u) ? 7u : 0u) | ((my & 4u) ? 0x1c0u : 0u) | 0x38u;
  const unsigned yb = y9 * 0x40201u;     // bit nb: dy = (nb / 3) % 3 present
  const unsigned zb = ((mz & 1u) ? 0x1ffu : 0u) | (0x1ffu << 9) | ((mz & 4u) ? (0x1ffu << 18) : 0u);
  return xb & yb & zb;
}

// one node's three rows in the inode order; FULL: every neighbour present (pairing fixed at
// compile time: block nb opens with an even position when nb is even)
template <bool FULL>
struct InodeRows {
  double s[3] = {0., 0., 0.}, e[3] = {0., 0., 0.};
  unsigned pres = PRES_ALL;
  // term t = a x of row r, column c of block nb (nb, r, c compile-time constants once unrolled)
  __device__ __forceinline__ void term(int nb, int r, int c, double t) {
    if (!FULL && !((pres >> nb) & 1u)) return;
    const bool odd = FULL ? ((nb + c) & 1) : ((__builtin_popcount(pres & ((1u << nb) - 1u)) + c) & 1);
    if (odd) s[r] = s[r] + (e[r] + t);
    else e[r] = t;
  }
  __device__ __forceinline__ double row(int r) const {
    const bool odd = FULL ? true : (__builtin_popcount(pres) & 1);  // 81 terms when every block is present
    return odd ? s[r] + e[r] : s[r];
  }
};

// y = A x for the owned rows.  One thread = one node = 3 rows; 122 x 16-B coalesced loads of
// the stencil blocks, x gathered from the padded box (L1/L2 resident neighbours).  Each row
// adds its slots in ascending (nb, c) = ascending global column on one rank, in the inode
// kernel's pairs (above), so y is bit-identical to the reference's AIJ MatMult (inode order, oracle/oracle.c row_part).  DOT: per-block p.w.
template <int S>
__device__ __forceinline__ void slot_acc(double v, const double (&xv)[27][3], InodeRows<false>& acc) {
  constexpr int nb = S / 9, r = (S % 9) / 3, c = S % 3;
  acc.term(nb, r, c, v * xv[nb][c]);
}

template <bool NT>
__device__ __forceinline__ double2 ldv(const double2* p) {
  if constexpr (NT) {
    double2 r;
    r.x = __builtin_nontemporal_load(&p->x);
    r.y = __builtin_nontemporal_load(&p->y);
    return r;
  } else {
    return *p;
  }
}

template <int Q, bool NT = false>
struct PairLoop {
  static __device__ __forceinline__ void run(const double2* __restrict__ v, const double (&xv)[27][3],
                                             InodeRows<false>& acc) {
    PairLoop<Q - 1, NT>::run(v, xv, acc);
    const double2 a = ldv<NT>(v + (Q - 1) * 64);
    slot_acc<2 * (Q - 1)>(a.x, xv, acc);
    if constexpr (2 * (Q - 1) + 1 < NSLOT) slot_acc<2 * (Q - 1) + 1>(a.y, xv, acc);
  }
};
template <bool NT>
struct PairLoop<0, NT> {
  static __device__ __forceinline__ void run(const double2* __restrict__, const double (&)[27][3],
                                             InodeRows<false>&) {}
};

template <bool DOT, bool GATED, int NT = 0>
__global__ __launch_bounds__(TPB) void k_spmv(Geo g, const double2* __restrict__ V, const double* __restrict__ x,
                                              double* __restrict__ y, double* __restrict__ part,
                                              const CgState* __restrict__ cg, SpmvTiling tl) {
  __shared__ double sh[TPB / 64];
  if (GATED && cg->reason) return;
  int i = 0, j = 0, k = 0;
  const int n = spmv_node(g, tl.TX, tl.LPB, tl.nxc, tl.jgroups, tl.subl, i, j, k);
  double dot = 0.;
  if (n >= 0) {
    const int PX = g.PX, PXY = g.PX * g.PY;
    const int pc = (i + 1) + (j + 1) * PX + (k + 1) * PXY;
    double xv[27][3];
#pragma unroll
    for (int nb = 0; nb < 27; nb++) {
      const int off = (nb % 3 - 1) + ((nb / 3) % 3 - 1) * PX + (nb / 9 - 1) * PXY;
      const double* xp = x + 3 * (int64_t)(pc + off);
      xv[nb][0] = xp[0];
      xv[nb][1] = xp[1];
      xv[nb][2] = xp[2];
    }
    const double2* v = V + (int64_t)(n >> 6) * (NPAIR * 64) + (n & 63);
    InodeRows<false> acc;
    acc.pres = present_mask(g, i, j, k);
    PairLoop<NPAIR, (NT > 0)>::run(v, xv, acc);
    const double y0 = acc.row(0), y1 = acc.row(1), y2 = acc.row(2);
    if constexpr (NT == 2) {
      __builtin_nontemporal_store(y0, &y[3 * n + 0]);
      __builtin_nontemporal_store(y1, &y[3 * n + 1]);
      __builtin_nontemporal_store(y2, &y[3 * n + 2]);
    } else {
      y[3 * n + 0] = y0;
      y[3 * n + 1] = y1;
      y[3 * n + 2] = y2;
    }
    if (DOT) dot = xv[13][0] * y0 + xv[13][1] * y1 + xv[13][2] * y2;
  }
  if (DOT) {
    double s = block_sum<TPB>(dot, sh);
    if (threadIdx.x == 0) part[blockIdx.x] = s;
  }
}

// sbaij SpMV: y_n = sum_nb A(n,nb) x_nb in ascending (nb, c) order, where A(n,nb) for nb < 13 is
// the transpose of the upper block 26-nb stored at node n+off(nb), the diagonal block is
// mirrored from its upper triangle, nb > 13 comes from node n's own storage.
template <int NB>
__device__ __forceinline__ double usl(const double* __restrict__ Ug, int s) {
  return Ug[(s >> 1) * 128 + (s & 1)];
}

template <bool DOT, bool GATED>
__global__ __launch_bounds__(TPB) void k_spmv_sym(Geo g, const double* __restrict__ U, const double* __restrict__ x,
                                                  double* __restrict__ y, double* __restrict__ part,
                                                  const CgState* __restrict__ cg, SpmvTiling tl) {
  __shared__ double sh[TPB / 64];
  if (GATED && cg->reason) return;
  int i = 0, j = 0, k = 0;
  const int n = spmv_node(g, tl.TX, tl.LPB, tl.nxc, tl.jgroups, tl.subl, i, j, k);
  double dot = 0.;
  if (n >= 0) {
    const int PX = g.PX, PXY = g.PX * g.PY;
    const int pc = (i + 1) + (j + 1) * PX + (k + 1) * PXY;
    const int uc = u_of(g, i, j, k);
    double y0 = 0., y1 = 0., y2 = 0.;
    double xc0 = 0., xc1 = 0., xc2 = 0.;
#pragma unroll
    for (int nb = 0; nb < 27; nb++) {
      const int off = (nb % 3 - 1) + ((nb / 3) % 3 - 1) * PX + (nb / 9 - 1) * PXY;
      const int q = pc + off;
      const int uq = uc + (nb % 3 - 1) + ((nb / 3) % 3 - 1) * g.UX + (nb / 9 - 1) * g.UXY;
      const double* xp = x + 3 * (int64_t)q;
      const double x0 = xp[0], x1 = xp[1], x2 = xp[2];
      double a[9];
      if (nb < 13) {
        const double* Ug = U + (int64_t)(uq >> 6) * (UPAIR * 128) + 2 * (uq & 63);
        const int base = 6 + 9 * (12 - nb);
#pragma unroll
        for (int r = 0; r < 3; r++)
#pragma unroll
          for (int c = 0; c < 3; c++) a[r * 3 + c] = usl<0>(Ug, base + c * 3 + r);
      } else if (nb == 13) {
        const double* Ug = U + (int64_t)(uc >> 6) * (UPAIR * 128) + 2 * (uc & 63);
        const double d00 = usl<0>(Ug, 0), d01 = usl<0>(Ug, 1), d02 = usl<0>(Ug, 2), d11 = usl<0>(Ug, 3),
                     d12 = usl<0>(Ug, 4), d22 = usl<0>(Ug, 5);
        a[0] = d00; a[1] = d01; a[2] = d02;
        a[3] = d01; a[4] = d11; a[5] = d12;
        a[6] = d02; a[7] = d12; a[8] = d22;
        xc0 = x0;
        xc1 = x1;
        xc2 = x2;
      } else {
        const double* Ug = U + (int64_t)(uc >> 6) * (UPAIR * 128) + 2 * (uc & 63);
        const int base = 6 + 9 * (nb - 14);
#pragma unroll
        for (int s = 0; s < 9; s++) a[s] = usl<0>(Ug, base + s);
      }
      y0 += a[0] * x0; y0 += a[1] * x1; y0 += a[2] * x2;
      y1 += a[3] * x0; y1 += a[4] * x1; y1 += a[5] * x2;
      y2 += a[6] * x0; y2 += a[7] * x1; y2 += a[8] * x2;
    }
    y[3 * n + 0] = y0;
    y[3 * n + 1] = y1;
    y[3 * n + 2] = y2;
    if (DOT) dot = xc0 * y0 + xc1 * y1 + xc2 * y2;
  }
  if (DOT) {
    double s = block_sum<TPB>(dot, sh);
    if (threadIdx.x == 0) part[blockIdx.x] = s;
  }
}


// ---------------------------------------------------------------------------- sbaij SpMV, z-marching
// A block owns a TX x TY (64 x 4) tile of (x,y) columns and marches up a z-chunk.  Each node's
// upper blocks are read once: the node's own rows use them directly, and the transposed
// products c = U(m,nb')^T x_m go to the targets inside the tile through LDS slots (9 slots
// for the next plane, 4 for the current one); targets at the tile edge or at the first plane
// of the chunk pull the few source blocks they need from HBM/L2 instead.  Every row is the sum
// of its 27 block products (each a 3-term partial sum) in ascending nb order, however the
// products were routed, so the result is independent of tiling and rank grid.
struct ZTiling {
  int ntx, nty, nzc, kc;  // tiles in x, y; z chunks and planes per chunk
  int dbg = 0;            // timing-only diagnostics (k_spmv_vibm: 1 = every wave takes the scalar path)
  int wmap = 1;           // k_spmv_vibm PATCH: 1 = patches on SIMDs as a Latin square, 0 = row-major (A/B)
  int xlist = VI_EXC_LIST;  // k_spmv_vibm EXC: exception nodes a tile defers (option vi_exc_list; the rest in their plane)
  int xskip = 0;          // k_spmv_vibm EXC: exception nodes are left to k_spmv_exc (option vi_exc_kernel)
  int ypair = 0;          // k_spmv_vibm UNI: y of lane pairs as 16-B stores (option vi_ypair; needs an even nx)
  const unsigned* wd = nullptr;  // k_spmv_vibm WD: the wave descriptors (build_wdesc), npx x npy 16 x 4 patches per plane
  int npx = 0, npy = 0;
  int wdm = 1;                   // WD: 1 = uniform waves, 2 = also two-set waves (FMA rows; option vi_wdesc)
};

static ZTiling z_tiling(const Geo& g, int ztx, int zty, int want) {
  ZTiling t;
  t.ntx = (g.nx + ztx - 1) / ztx;
  t.nty = (g.ny + zty - 1) / zty;
  const int tiles = t.ntx * t.nty;
  if (want <= 0) {
    // one resident round, but at least two planes per chunk: a one-plane chunk pulls all of
    // its lower terms (64^3: 0.083 ms at one plane, 0.071 ms at two, tools/spmv_ab.py)
    want = g.ncu * std::max(1, 1024 / (ztx * zty));
    want = std::min(want, tiles * std::max(1, g.nz / 2));
  }
  t.nzc = std::max(1, std::min(g.nz, (want + tiles - 1) / tiles));
  t.kc = (g.nz + t.nzc - 1) / t.nzc;
  t.nzc = (g.nz + t.kc - 1) / t.kc;
  return t;
}

__device__ __forceinline__ double uval(const double* __restrict__ U, int p, int s) {
  return U[(int64_t)(p >> 6) * (UPAIR * 128) + 2 * (p & 63) + (s >> 1) * 128 + (s & 1)];
}

// c = U(p, nb')^T x_p for upper block nb' (14..26) of padded node p
// U(m, nbp)^T x_m with the block's 9 slots read as the 5 covering 16-B pairs (a pulled block
// uses whole pairs: an 8-B scalar read would fetch the pair's line for half of it)
__device__ __forceinline__ void ut_x2(const double* __restrict__ U, const double* __restrict__ x, int pu, int p,
                                      int nbp, double& c0, double& c1, double& c2) {
  const int base = 6 + 9 * (nbp - 14);
  const double2* Ug = reinterpret_cast<const double2*>(U) + (int64_t)(pu >> 6) * (UPAIR * 64) + (pu & 63);
  double a[10];
  const int p0 = base >> 1, sh = base & 1;
#pragma unroll
  for (int q = 0; q < 5; q++) {
    const double2 w = Ug[(p0 + q) * 64];
    a[2 * q] = w.x;
    a[2 * q + 1] = w.y;
  }
  double b[9];
#pragma unroll
  for (int t = 0; t < 9; t++) b[t] = sh ? a[t + 1] : a[t];
  const double x0 = x[3 * (int64_t)p], x1 = x[3 * (int64_t)p + 1], x2 = x[3 * (int64_t)p + 2];
  c0 = b[0] * x0;
  c0 += b[3] * x1;
  c0 += b[6] * x2;
  c1 = b[1] * x0;
  c1 += b[4] * x1;
  c1 += b[7] * x2;
  c2 = b[2] * x0;
  c2 += b[5] * x1;
  c2 += b[8] * x2;
}

// U(m, nbp)^T x_m for the node m at U index pu / padded-vector index p
__device__ __forceinline__ void ut_x(const double* __restrict__ U, const double* __restrict__ x, int pu, int p,
                                     int nbp, double& c0, double& c1, double& c2) {
  const int base = 6 + 9 * (nbp - 14);
  const double x0 = x[3 * (int64_t)p], x1 = x[3 * (int64_t)p + 1], x2 = x[3 * (int64_t)p + 2];
  c0 = uval(U, pu, base + 0) * x0;
  c0 += uval(U, pu, base + 3) * x1;
  c0 += uval(U, pu, base + 6) * x2;
  c1 = uval(U, pu, base + 1) * x0;
  c1 += uval(U, pu, base + 4) * x1;
  c1 += uval(U, pu, base + 7) * x2;
  c2 = uval(U, pu, base + 2) * x0;
  c2 += uval(U, pu, base + 5) * x1;
  c2 += uval(U, pu, base + 8) * x2;
}

template <bool DOT, bool GATED, int ZTX, int ZTY>
__global__ __launch_bounds__(ZTX * ZTY, (ZTX * ZTY >= 512 ? 1 : 2)) void k_spmv_symz(Geo g, const double* __restrict__ U,
                                                         const double* __restrict__ x, double* __restrict__ y,
                                                         double* __restrict__ part, const CgState* __restrict__ cg,
                                                         ZTiling zt) {
  __shared__ double accN[9][3][ZTY * ZTX];  // next-plane contributions, by the target's lower nb (0..8)
  __shared__ double accC[4][3][ZTY * ZTX];  // current-plane contributions, lower nb 9..12
  __shared__ double sh[(ZTX * ZTY) / 64];
  if (GATED && cg->reason) return;
  // block -> (tile x, tile y, z chunk); tiles of one XCD form a y-slab (blocks b, b+8 share an XCD)
  const int b = blockIdx.x;
  const int xcd = b & 7, t8 = b >> 3;
  const int slab = (zt.nty + 7) >> 3;
  const int ty0 = xcd * slab;
  const int nty_here = min(slab, zt.nty - ty0);
  const int per = max(nty_here, 0) * zt.ntx * zt.nzc;
  double dot = 0.;
  const bool blk_ok = t8 < per;
  int tyi = 0, txi = 0, zc = 0;
  if (blk_ok) {
    zc = t8 % zt.nzc;
    const int r = t8 / zt.nzc;
    txi = r % zt.ntx;
    tyi = ty0 + r / zt.ntx;
  }
  const int lx = threadIdx.x % ZTX, ly = threadIdx.x / ZTX, me = threadIdx.x;
  const int i = txi * ZTX + lx, j = tyi * ZTY + ly;
  const bool active = blk_ok && i < g.nx && j < g.ny;
  const int k0 = zc * zt.kc, k1 = min(g.nz, k0 + zt.kc);
  const int PX = g.PX, PXY = g.PX * g.PY;
  // a source at tile-relative (lx+dx, ly+dy) is pushed by a thread of this block iff active
  auto in_tile = [&](int dx, int dy) {
    const int sx = lx + dx, sy = ly + dy;
    if (sx < 0 || sx >= ZTX || sy < 0 || sy >= ZTY) return false;
    const int si = i + dx, sj = j + dy;
    return si < g.nx && sj < g.ny;
  };
  for (int k = k0; blk_ok && k < k1; k++) {
    const int pc = (i + 1) + (j + 1) * PX + (k + 1) * PXY;
    const int uc = u_of(g, i, j, k);
    double y0 = 0., y1 = 0., y2 = 0.;
    // 1. lower blocks nb 0..8 (dz = -1), ascending nb
    if (active) {
#pragma unroll
      for (int nb = 0; nb < 9; nb++) {
        const int dx = nb % 3 - 1, dy = nb / 3 - 1;
        double c0, c1, c2;
        if (k > k0 && in_tile(dx, dy)) {
          c0 = accN[nb][0][me];
          c1 = accN[nb][1][me];
          c2 = accN[nb][2][me];
        } else {
          ut_x(U, x, uc + dx + dy * g.UX - g.UXY, pc + dx + dy * PX - PXY, 26 - nb, c0, c1, c2);
        }
        y0 += c0;
        y1 += c1;
        y2 += c2;
      }
    }
    __syncthreads();
    // 2. one pass over this node's upper storage: its own rows' upper sum (diagonal block, then
    //    nb 14..26 ascending) and the transposed products pushed to in-tile targets
    double s0 = 0., s1 = 0., s2 = 0.;
    double x0 = 0., x1 = 0., x2 = 0.;
    if (active) {
      x0 = x[3 * (int64_t)pc];
      x1 = x[3 * (int64_t)pc + 1];
      x2 = x[3 * (int64_t)pc + 2];
      const double* Ug = U + (int64_t)(uc >> 6) * (UPAIR * 128) + 2 * (uc & 63);
      {
        const double d00 = Ug[0], d01 = Ug[1], d02 = Ug[128], d11 = Ug[129], d12 = Ug[256], d22 = Ug[257];
        s0 = d00 * x0;
        s0 += d01 * x1;
        s0 += d02 * x2;
        s1 = d01 * x0;
        s1 += d11 * x1;
        s1 += d12 * x2;
        s2 = d02 * x0;
        s2 += d12 * x1;
        s2 += d22 * x2;
      }
#pragma unroll 2
      for (int nbp = 14; nbp < 27; nbp++) {
        const int dx = nbp % 3 - 1, dy = (nbp / 3) % 3 - 1, dz = nbp / 9 - 1;
        double a[9];
#pragma unroll
        for (int t = 0; t < 9; t++) {
          const int s = 6 + 9 * (nbp - 14) + t;
          a[t] = Ug[(s >> 1) * 128 + (s & 1)];
        }
        // own rows: U(m, nbp) x_{m + off}
        const int q = pc + dx + dy * PX + dz * PXY;
        const double z0 = x[3 * (int64_t)q], z1 = x[3 * (int64_t)q + 1], z2 = x[3 * (int64_t)q + 2];
        double u0 = a[0] * z0;
        u0 += a[1] * z1;
        u0 += a[2] * z2;
        double u1 = a[3] * z0;
        u1 += a[4] * z1;
        u1 += a[5] * z2;
        double u2 = a[6] * z0;
        u2 += a[7] * z1;
        u2 += a[8] * z2;
        s0 += u0;
        s1 += u1;
        s2 += u2;
        // push U(m, nbp)^T x_m to the target m + (dx,dy,dz) when it is inside this tile
        const int tx = lx + dx, ty = ly + dy;
        if (tx < 0 || tx >= ZTX || ty < 0 || ty >= ZTY) continue;
        if (i + dx >= g.nx || j + dy >= g.ny) continue;
        if (dz == 1 && k + 1 >= k1) continue;
        double c0 = a[0] * x0;
        c0 += a[3] * x1;
        c0 += a[6] * x2;
        double c1 = a[1] * x0;
        c1 += a[4] * x1;
        c1 += a[7] * x2;
        double c2 = a[2] * x0;
        c2 += a[5] * x1;
        c2 += a[8] * x2;
        const int tgt = ty * ZTX + tx;
        if (dz == 1) {
          accN[26 - nbp][0][tgt] = c0;
          accN[26 - nbp][1][tgt] = c1;
          accN[26 - nbp][2][tgt] = c2;
        } else {
          accC[26 - nbp - 9][0][tgt] = c0;
          accC[26 - nbp - 9][1][tgt] = c1;
          accC[26 - nbp - 9][2][tgt] = c2;
        }
      }
    }
    __syncthreads();
    if (active) {
      // 3. lower blocks nb 9..12 (dz = 0), then the upper sum: y = (lower, ascending nb) + upper
#pragma unroll
      for (int nb = 9; nb < 13; nb++) {
        const int dx = nb % 3 - 1, dy = (nb / 3) % 3 - 1;
        double c0, c1, c2;
        if (in_tile(dx, dy)) {
          c0 = accC[nb - 9][0][me];
          c1 = accC[nb - 9][1][me];
          c2 = accC[nb - 9][2][me];
        } else {
          ut_x(U, x, uc + dx + dy * g.UX, pc + dx + dy * PX, 26 - nb, c0, c1, c2);
        }
        y0 += c0;
        y1 += c1;
        y2 += c2;
      }
      y0 += s0;
      y1 += s1;
      y2 += s2;
      const int n = i + j * g.nx + k * g.nx * g.ny;
      y[3 * (int64_t)n + 0] = y0;
      y[3 * (int64_t)n + 1] = y1;
      y[3 * (int64_t)n + 2] = y2;
      if (DOT) dot += x0 * y0 + x1 * y1 + x2 * y2;
    }
  }
  if (DOT) {
    double s = block_sum<ZTX * ZTY>(dot, sh);
    if (threadIdx.x == 0) part[blockIdx.x] = s;
  }
}

// Phased z-marching sbaij SpMV.  Same tile march as k_spmv_symz, but the 13 upper blocks are
// processed in three phases (nbp 14..18 | 19..22 | 23..26) that reuse one 5-slot LDS buffer
// (120 B per node instead of 312), so a 128x4 tile runs two blocks per CU and only the tile's
// first and last rows pull across y edges.  Matrix values are loaded as 16-B slot pairs.
// Row order (fixed, tiling-independent: a term is the same 3-vector whether it arrives through
// LDS or is pulled by the target, and it is added at the same position):
//   lower dz=-1: nb 8 | 4 5 6 7 | 0 1 2 3,  lower dz=0: nb 9 10 11 12,  then the upper sum
//   (diagonal block, nbp 14..26 ascending).
// AIJ-split lower corrections: per owned node the 117 lower-block values minus their mirrored
// upper values, exact in bf16, as 15 x 16-B quads [node/64][15][node%64] (slot nb*9 + r*3 + c)
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <bool DOT, bool GATED, int TX, int TY, bool AIJS = false>
__global__ __launch_bounds__(TX * TY, 4) void k_spmv_symp(Geo g, const double* __restrict__ U,
                                                        const double* __restrict__ x, double* __restrict__ y,
                                                        double* __restrict__ part, const CgState* __restrict__ cg,
                                                        ZTiling zt, const uint16_t* __restrict__ Dq = nullptr,
                                                        DSlots dl = DSlots()) {
  constexpr int T = TX * TY;
  // y-edge terms computed by helper threads (TY >= 4: at most 4 TX = T of them per phase)
  constexpr bool HELP = TY >= 4;
  __shared__ double buf[5][3][T];
  __shared__ double edge[HELP ? 3 : 1][HELP ? T : 1];
  __shared__ double sh[T / 64];
  if (GATED && cg->reason) return;
  const int b = blockIdx.x;
  const int xcd = b & 7, t8 = b >> 3;
  const int slab = (zt.nty + 7) >> 3;
  const int ty0 = xcd * slab;
  const int nty_here = min(slab, zt.nty - ty0);
  const int per = max(nty_here, 0) * zt.ntx * zt.nzc;
  const bool blk_ok = t8 < per;
  int tyi = 0, txi = 0, zc = 0;
  if (blk_ok) {  // x fastest, then the slab's tile rows, then z-chunks
    txi = t8 % zt.ntx;
    const int r = t8 / zt.ntx;
    tyi = ty0 + r % nty_here;
    zc = r / nty_here;
  }
  if (!blk_ok) {  // whole block idle (uniform): still write the partial
    if (DOT && threadIdx.x == 0) part[blockIdx.x] = 0.;
    return;
  }
  const int lx = threadIdx.x % TX, ly = threadIdx.x / TX, me = threadIdx.x;
  const int i = txi * TX + lx, j = tyi * TY + ly;
  const bool active = i < g.nx && j < g.ny;
  const int k0 = zc * zt.kc, k1 = min(g.nz, k0 + zt.kc);
  const int PX = g.PX, PXY = g.PX * g.PY;
  // in-tile (pushed through LDS) test for a partner at (dx, dy) in the tile's plane
  auto in_tile = [&](int dx, int dy) {
    const int sx = lx + dx, sy = ly + dy;
    if (sx < 0 || sx >= TX || sy < 0 || sy >= TY) return false;
    return i + dx < g.nx && j + dy < g.ny;
  };
  double dot = 0.;
  double a0 = 0., a1 = 0., a2 = 0.;  // this plane's node: lower sum so far
  double n0 = 0., n1 = 0., n2 = 0.;  // next plane's node: lower dz=-1 sum so far
  // lower term nb of the node (i, j, kt) at padded index pcn: from LDS slot or pulled.  A source
  // outside the global domain is a zero ghost (x = 0 there): its term is +0 without the loads
  auto term = [&](int nb, int slot, bool from_lds, int pcn, int ucn, int kt, double& c0, double& c1, double& c2) {
    if (from_lds) {
      c0 = buf[slot][0][me];
      c1 = buf[slot][1][me];
      c2 = buf[slot][2][me];
    } else {
      const int dx = nb % 3 - 1, dy = (nb / 3) % 3 - 1, dz = nb / 9 - 1;
      const unsigned gx = g.xs + i + dx, gy = g.ys + j + dy, gz = g.zs + kt + dz;
      if (gx >= (unsigned)g.NX || gy >= (unsigned)g.NY || gz >= (unsigned)g.NZ) {
        c0 = c1 = c2 = 0.;
      } else {
        ut_x2(U, x, ucn + dx + dy * g.UX + dz * g.UXY, pcn + dx + dy * PX + dz * PXY, 26 - nb, c0, c1, c2);
      }
    }
  };
  for (int k = k0; k < k1; k++) {
    const int pc = (i + 1) + (j + 1) * PX + (k + 1) * PXY;
    const int uc = u_of(g, i, j, k);
    const bool has_next = k + 1 < k1;
    if (k == k0 && active) {  // chunk start: the previous plane is not marched here, pull all nine
      a0 = a1 = a2 = 0.;
#pragma unroll
      for (int q = 0; q < 9; q++) {  // canonical order 8 | 4 5 6 7 | 0 1 2 3
        double c0, c1, c2;
        term(q == 0 ? 8 : (q <= 4 ? q + 3 : q - 5), 0, false, pc, uc, k, c0, c1, c2);
        a0 += c0;
        a1 += c1;
        a2 += c2;
      }
    }
    double x0 = 0., x1 = 0., x2 = 0., s0 = 0., s1 = 0., s2 = 0.;
    const double2* Ug = reinterpret_cast<const double2*>(U) + (int64_t)(uc >> 6) * (UPAIR * 64) + (uc & 63);
    if (active) {
      x0 = x[3 * (int64_t)pc];
      x1 = x[3 * (int64_t)pc + 1];
      x2 = x[3 * (int64_t)pc + 2];
    }
    n0 = n1 = n2 = 0.;
    double cd0 = 0., cd1 = 0., cd2 = 0.;  // AIJ-split corrections of this plane's node
#pragma unroll
    for (int ph = 0; ph < 3; ph++) {
      const int lo = ph == 0 ? 14 : (ph == 1 ? 19 : 23), hi = ph == 0 ? 18 : (ph == 1 ? 22 : 26);
      if (active) {
        // slot s of this node = half (s & 1) of 16-B pair s >> 1; pairs shared by adjacent
        // blocks are the same load (read-only, merged by the compiler)
        auto sl = [&](int s) {
          const double2 w = Ug[(s >> 1) * 64];
          return (s & 1) ? w.y : w.x;
        };
        if (ph == 0) {
          const double d00 = sl(0), d01 = sl(1), d02 = sl(2), d11 = sl(3), d12 = sl(4), d22 = sl(5);
          s0 = d00 * x0;
          s0 += d01 * x1;
          s0 += d02 * x2;
          s1 = d01 * x0;
          s1 += d11 * x1;
          s1 += d12 * x2;
          s2 = d02 * x0;
          s2 += d12 * x1;
          s2 += d22 * x2;
        }
#pragma unroll 2
        for (int nbp = lo; nbp <= hi; nbp++) {
          const int dx = nbp % 3 - 1, dy = (nbp / 3) % 3 - 1, dz = nbp / 9 - 1;
          const int base = 6 + 9 * (nbp - 14);
          double a[9];
#pragma unroll
          for (int t = 0; t < 9; t++) a[t] = sl(base + t);
          const int q = pc + dx + dy * PX + dz * PXY;
          const double z0 = x[3 * (int64_t)q], z1 = x[3 * (int64_t)q + 1], z2 = x[3 * (int64_t)q + 2];
          double u0 = a[0] * z0;
          u0 += a[1] * z1;
          u0 += a[2] * z2;
          double u1 = a[3] * z0;
          u1 += a[4] * z1;
          u1 += a[5] * z2;
          double u2 = a[6] * z0;
          u2 += a[7] * z1;
          u2 += a[8] * z2;
          s0 += u0;
          s1 += u1;
          s2 += u2;
          if (!in_tile(dx, dy)) continue;
          if (dz == 1 && !has_next) continue;
          double c0 = a[0] * x0;
          c0 += a[3] * x1;
          c0 += a[6] * x2;
          double c1 = a[1] * x0;
          c1 += a[4] * x1;
          c1 += a[7] * x2;
          double c2 = a[2] * x0;
          c2 += a[5] * x1;
          c2 += a[8] * x2;
          const int tgt = me + dx + dy * TX;
          buf[nbp - lo][0][tgt] = c0;
          buf[nbp - lo][1][tgt] = c1;
          buf[nbp - lo][2][tgt] = c2;
        }
      }
      // AIJ-split corrections of this plane's node (independent of the LDS exchange), computed
      // while the block waits at the phase-2 barrier; exact AIJ lower blocks = mirrored upper
      // (summed in the gathers) + the bf16 corrections of the active slots, ascending nb then c
      // per row, added after the lower sum.  8 corrections per 16-B quad (prefetched at plane
      // start); one 8-B x gather per slot, all issued before the first product (see below).
      if (AIJS && ph == 2 && active) {
        const u32x4* Dn = reinterpret_cast<const u32x4*>(Dq) + (int64_t)(uc >> 6) * dl.Lq * 64 + (uc & 63);
        double d0 = 0., d1 = 0., d2 = 0.;
        const int per = dl.wide ? 4 : 8;
        // the slots held in wpre (24 bf16 / 12 f32) at unrolled positions: one 8-B x load per slot,
        // all issued before the first use (one round trip, not one per block)
        const int nfast = min(dl.L, 3 * per);
#ifndef MCX_SPLIT_WALK_GROUPED
#define MCX_SPLIT_WALK_GROUPED 0  // 1: the AIJ-split walk in quad groups (44 -> 12 B of spills per lane at 256x4, but 3.65 vs
                                   // 3.58 ms per SpMV at 256^3: profiles/r05d_split_walk_ab.log)
#endif
#if MCX_SPLIT_WALK_GROUPED
        // the first 24 corrections in three groups of one quad each: the quad and its x gathers
        // issued together, then its products (16 live VGPRs per group instead of 60 for all 24)
#pragma unroll
        for (int t = 0; t < 3; t++) {
          if (t * per >= nfast) break;  // (uniform)
          const u32x4 w = __builtin_nontemporal_load(Dn + t * 64);
          double xv[8];
#pragma unroll
          for (int e = 0; e < 8; e++) {
            const int p = t * per + e;
            xv[e] = 0.;
            if (e < per && p < nfast) xv[e] = x[3 * (int64_t)pc + (dl.xc[p] >> 2)];
          }
#pragma unroll
          for (int e = 0; e < 8; e++) {
            const int p = t * per + e;
            if (e >= per || p >= nfast) continue;
            const int r = dl.xc[p] & 3;
            double v;
            if (dl.wide) {
              v = (double)__uint_as_float(w[e & 3]);
            } else {
              const unsigned hw = w[e >> 1];
              v = (double)__uint_as_float((e & 1) ? (hw & 0xffff0000u) : (hw << 16));
            }
            const double tv = v * xv[e];
            if (r == 0) d0 += tv;
            else if (r == 1) d1 += tv;
            else d2 += tv;
          }
          __builtin_amdgcn_sched_barrier(0);
        }
#else
        // the first 24 corrections of this node (3 quads), loaded with the x gathers below
        u32x4 wpre[3] = {{0u, 0u, 0u, 0u}, {0u, 0u, 0u, 0u}, {0u, 0u, 0u, 0u}};
#pragma unroll
        for (int t = 0; t < 3; t++)
          if (t < dl.Lq) wpre[t] = __builtin_nontemporal_load(Dn + t * 64);
        double xv[24];
#pragma unroll
        for (int p = 0; p < 24; p++) {
          xv[p] = 0.;
          if (p < nfast) xv[p] = x[3 * (int64_t)pc + (dl.xc[p] >> 2)];
        }
#pragma unroll
        for (int p = 0; p < 24; p++) {
          if (p >= nfast) continue;
          const int r = dl.xc[p] & 3;
          double v;
          if (dl.wide) {
            v = (double)__uint_as_float(wpre[p >> 2][p & 3]);
          } else {
            const unsigned hw = wpre[p >> 3][(p & 7) >> 1];
            v = (double)__uint_as_float((p & 1) ? (hw & 0xffff0000u) : (hw << 16));
          }
          const double tv = v * xv[p];
          if (r == 0) d0 += tv;
          else if (r == 1) d1 += tv;
          else d2 += tv;
        }
#endif
        for (int p = nfast; p < dl.L; p++) {  // beyond wpre (dense corrections): one slot at a time
          const u32x4 w = __builtin_nontemporal_load(Dn + (p / per) * 64);
          const int s = dl.s[p], nb = s / 9, rc = s - 9 * nb, r = rc / 3, cc = rc - 3 * r, e = p % per;
          const int qn = pc + (nb % 3 - 1) + ((nb / 3) % 3 - 1) * PX + (nb / 9 - 1) * PXY;
          double v;
          if (dl.wide) {
            v = (double)__uint_as_float(w[e & 3]);
          } else {
            const unsigned hw = w[e >> 1];
            v = (double)__uint_as_float((e & 1) ? (hw & 0xffff0000u) : (hw << 16));
          }
          const double tv = v * x[3 * (int64_t)qn + cc];
          if (r == 0) d0 += tv;
          else if (r == 1) d1 += tv;
          else d2 += tv;
        }
        cd0 = d0;
        cd1 = d1;
        cd2 = d2;
      }
      // Edge terms: the lower terms the tile's y-edge rows would pull after the barrier (row 0:
      // sources at dy = -1, row TY-1: dy = +1), computed now by one helper thread each into
      // edge[][h] (the same expression as the pull), so no wave waits on a chain of pulls there.
      // (Helpers for every out-of-tile term, x-edge columns included, and squarer tiles were
      // slower: profiles/old/r02b_ab_tiles.log.)
      if constexpr (HELP) {
        //   ph 0: h < 3 TX: row 0, this plane, nb 9 + h / TX;  3 TX <= h < 4 TX: row TY-1, next plane, nb 8
        //   ph 1: h < 2 TX: row TY-1, next plane, nb 6 + h / TX;  ph 2: h < 3 TX: row 0, next plane, nb h / TX
        const int grp = me / TX, it = txi * TX + me % TX;  // group: wave-uniform (TX % 64 == 0)
#pragma unroll
        for (int q = 0; q < 4; q++) {
          const int nbh = ph == 0 ? (q < 3 ? 9 + q : 8) : (ph == 1 ? (q < 2 ? 6 + q : -1) : (q < 3 ? q : -1));
          if (nbh < 0 || grp != q) continue;
          const bool nxt = !(ph == 0 && q < 3);
          const int jt = tyi * TY + ((ph == 0 && q == 3) || ph == 1 ? TY - 1 : 0);
          if (it < g.nx && jt < g.ny && (!nxt || has_next)) {
            const int kt = k + (nxt ? 1 : 0);
            const int dx = nbh % 3 - 1, dy = (nbh / 3) % 3 - 1, dz = nbh / 9 - 1;
            const unsigned gx = g.xs + it + dx, gy = g.ys + jt + dy, gz = g.zs + kt + dz;
            double c0 = 0., c1 = 0., c2 = 0.;
            if (gx < (unsigned)g.NX && gy < (unsigned)g.NY && gz < (unsigned)g.NZ)
              ut_x2(U, x, u_of(g, it, jt, kt) + dx + dy * g.UX + dz * g.UXY,
                    (it + 1 + dx) + (jt + 1 + dy) * PX + (kt + 1 + dz) * PXY, 26 - nbh, c0, c1, c2);
            edge[0][me] = c0;
            edge[1][me] = c1;
            edge[2][me] = c2;
          }
        }
      }
      __syncthreads();
      if (active) {
        // lower term nb: from the helpers' edge[] (y-edge rows), the LDS exchange or pulled now
        auto term2 = [&](int nb, int pcn, int ucn, int kt, double& c0, double& c1, double& c2) {
          const int dx = nb % 3 - 1, dy = (nb / 3) % 3 - 1;
          if (HELP && dy != 0 && (ly + dy < 0 || ly + dy >= TY)) {
            const int eidx = (nb >= 9 ? (nb - 9) * TX : (nb == 8 ? 3 * TX : (nb >= 5 ? (nb - 6) * TX : nb * TX))) + lx;
            c0 = edge[0][eidx];
            c1 = edge[1][eidx];
            c2 = edge[2][eidx];
          } else {
            term(nb, (26 - nb) - lo, in_tile(dx, dy), pcn, ucn, kt, c0, c1, c2);
          }
        };
        if (ph == 0) {
          // this plane's node: dz = 0 lower terms nb 9..12 (sources pushed nbp 17..14)
#pragma unroll
          for (int nb = 9; nb <= 12; nb++) {
            double c0, c1, c2;
            term2(nb, pc, uc, k, c0, c1, c2);
            a0 += c0;
            a1 += c1;
            a2 += c2;
          }
        }
        if (has_next) {
          // next plane's node (pc + PXY): dz = -1 terms of this phase, nb = 26 - nbp for the
          // phase's dz = +1 blocks, in the canonical order (8 | 4..7 | 0..3)
          const int nb_lo = ph == 0 ? 8 : 26 - hi, nb_hi = 26 - max(lo, 18);
#pragma unroll
          for (int nb = 0; nb <= 8; nb++) {
            if (nb < nb_lo || nb > nb_hi) continue;
            double c0, c1, c2;
            term2(nb, pc + PXY, uc + g.UXY, k + 1, c0, c1, c2);
            n0 += c0;
            n1 += c1;
            n2 += c2;
          }
        }
      }
      __syncthreads();
    }
    if (active) {
      const int n = i + j * g.nx + k * g.nx * g.ny;
      if constexpr (AIJS) {
        a0 += cd0;
        a1 += cd1;
        a2 += cd2;
      }
      const double y0 = a0 + s0, y1 = a1 + s1, y2 = a2 + s2;
      __builtin_nontemporal_store(y0, &y[3 * (int64_t)n + 0]);
      __builtin_nontemporal_store(y1, &y[3 * (int64_t)n + 1]);
      __builtin_nontemporal_store(y2, &y[3 * (int64_t)n + 2]);
      if (DOT) dot += x0 * y0 + x1 * y1 + x2 * y2;
    }
    a0 = n0;
    a1 = n1;
    a2 = n2;
  }
  if (DOT) {
    double s = block_sum<T>(dot, sh);
    if (threadIdx.x == 0) part[blockIdx.x] = s;
  }
}

// AIJ-split with dense corrections (dl.dense): y += D x for every owned node, all 120 slots in
// canonical order — per row, lower block nb ascending then column c, then the diagonal block's
// strictly-lower entries — added to the z-march's (lower + upper) sum; with DOT the p.w partials
// of the finished y.  One thread per owned node: 15 (bf16) or 30 (f32) coalesced 16-B quads, the
// 13 source nodes' x (3 doubles each) gathered once per block.  No barriers, full occupancy.
// Escapes (bf16 storage, esc_node set): after the 120 slots, the node's escaped corrections add
// their residuals d - hi (the bf16 hi is in D), in slot order.
template <bool DOT, bool GATED, bool WIDE>
__global__ __launch_bounds__(TPB) void k_split_dense(Geo g, const uint16_t* __restrict__ Dq, int Lq,
                                                     const double* __restrict__ x, double* __restrict__ y,
                                                     double* __restrict__ part, const CgState* __restrict__ cg,
                                                     const unsigned* __restrict__ esc_node = nullptr,
                                                     const double* __restrict__ esc_res = nullptr,
                                                     const unsigned char* __restrict__ esc_slot = nullptr) {
  __shared__ double sh[TPB / 64];
  if (GATED && cg->reason) return;
  const int n = blockIdx.x * TPB + threadIdx.x;
  double dot = 0.;
  if (n < g.nown) {
    int i, j, k;
    node_ijk(g, n, i, j, k);
    const int pc = pad_of(g, i, j, k);
    const int64_t u = u_of(g, i, j, k);
    const u32x4* Dn = reinterpret_cast<const u32x4*>(Dq) + (u >> 6) * Lq * 64 + (u & 63);
    const int PX = g.PX, PXY = g.PX * g.PY;
    // all quads of the node issued up front (15 bf16 or 30 f32 quads)
    constexpr int NQ = WIDE ? 30 : 15;
    u32x4 wq[NQ];
#pragma unroll
    for (int t = 0; t < NQ; t++) wq[t] = __builtin_nontemporal_load(Dn + t * 64);
    auto corr = [&](int p) -> double {
      if (WIDE) return (double)__uint_as_float(wq[p >> 2][p & 3]);
      const unsigned hw = wq[p >> 3][(p & 7) >> 1];
      return (double)__uint_as_float((p & 1) ? (hw & 0xffff0000u) : (hw << 16));
    };
    double d0 = 0., d1 = 0., d2 = 0.;
#pragma unroll
    for (int nb = 0; nb < 13; nb++) {
      const int q = pc + (nb % 3 - 1) + ((nb / 3) % 3 - 1) * PX + (nb / 9 - 1) * PXY;
      const double xm[3] = {x[3 * (int64_t)q], x[3 * (int64_t)q + 1], x[3 * (int64_t)q + 2]};
#pragma unroll
      for (int c = 0; c < 3; c++) {
        d0 += corr(nb * 9 + c) * xm[c];
        d1 += corr(nb * 9 + 3 + c) * xm[c];
        d2 += corr(nb * 9 + 6 + c) * xm[c];
      }
    }
    const double x0 = x[3 * (int64_t)pc], x1 = x[3 * (int64_t)pc + 1];
    d1 += corr(117) * x0;  // (1,0)
    d2 += corr(118) * x0;  // (2,0)
    d2 += corr(119) * x1;  // (2,1)
    if (!WIDE && esc_node) {
      const unsigned e = esc_node[n];
      if (e) {  // rare: a branch almost no lane takes
        const unsigned m = e >> 24, base = (e & 0xffffffu) - 1u;
        for (unsigned t = 0; t < m; t++) {
          const int sl = esc_slot[base + t], nb = sl / 9, rc = sl - 9 * nb, r = rc / 3, cc = rc - 3 * r;
          const int q = nb < 13 ? pc + (nb % 3 - 1) + ((nb / 3) % 3 - 1) * PX + (nb / 9 - 1) * PXY : pc;
          const double tv = esc_res[base + t] * x[3 * (int64_t)q + cc];
          if (r == 0) d0 += tv;
          else if (r == 1) d1 += tv;
          else d2 += tv;
        }
      }
    }
    const double y0 = y[3 * (int64_t)n] + d0, y1 = y[3 * (int64_t)n + 1] + d1, y2 = y[3 * (int64_t)n + 2] + d2;
    y[3 * (int64_t)n] = y0;
    y[3 * (int64_t)n + 1] = y1;
    y[3 * (int64_t)n + 2] = y2;
    if (DOT) dot = x0 * y0 + x1 * y1 + x[3 * (int64_t)pc + 2] * y2;
  }
  if (DOT) {
    const double s = block_sum<TPB>(dot, sh);
    if (threadIdx.x == 0) part[blockIdx.x] = s;
  }
}

// ---------------------------------------------------------------------------- value-indexed AIJ
// FMT_VI.  The assembled AIJ values of the elastic law take few distinct values (the stencil of
// a uniform grid, its boundary variants and the Dirichlet 0 / 1 entries: 129 at 12^3, 89 at
// 256^3), and any one slot S = nb*9 + r*3 + c of a node's 27 blocks takes at most 12 of them
// (12^3 .. 40^3, tests/test_gpu_parity.py).  So the matrix is held exactly as small indices into
// dictionaries of its values (value-indexed CSR, Kourtis, Goumas & Koziris, CF'08):
//   vi_bits 4: one nibble per value into the slot's own dictionary (<= 16 entries per slot):
//              128 B per node (243 nibbles + pad) instead of 1,944;
//   vi_bits 8: one byte per value into one dictionary of <= 256 entries: 256 B per node.
// Built at every assembly in two passes over the on-the-fly blocks (matrix_block): k_vi_collect
// gathers the distinct values (per block and slot in LDS, then per slot and overall in global
// sets); the host sorts them into the dictionaries (so indices do not depend on the order the
// sets were filled in); k_vi_pack writes the indices.  More than 256 distinct values (a per-GP
// tangent) = overflow: the context falls back to AIJ-split / AIJ blocks.
constexpr unsigned long long VI_EMPTY = ~0ull;  // a NaN payload arithmetic does not produce

__device__ __forceinline__ unsigned vi_hash(unsigned long long k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  return (unsigned)k;
}

// index of slot S in a node's chunks: NIB 8 = byte S of 16 x 16 B, NIB 4 = nibble S of 8 x 16 B
template <int NIB>
__device__ __forceinline__ unsigned vi_index(const u32x4* w, int S) {
  if constexpr (NIB == 8) return (w[S >> 4][(S >> 2) & 3] >> (8 * (S & 3))) & 255u;
  else return (w[S >> 5][(S >> 3) & 3] >> (4 * (S & 7))) & 15u;
}
// dictionary entry of that index: one shared table (8) or the slot's own 16 entries (4)
template <int NIB>
__device__ __forceinline__ int vi_entry(int S, unsigned id) {
  return NIB == 8 ? (int)id : S * 16 + (int)id;
}
template <int NIB>
constexpr int vi_chunks() { return NIB == 8 ? 16 : 8; }

// insert key into an open-addressing set of SIZE entries; returns true when it was new, probe
// budget exhausted = *full
template <int SIZE>
__device__ __forceinline__ bool vi_insert(unsigned long long* set, unsigned long long key, bool* full) {
  unsigned h = vi_hash(key) & (SIZE - 1);
  for (int probe = 0; probe < SIZE; probe++) {
    const unsigned long long cur = __hip_atomic_load(&set[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (cur == key) return false;
    if (cur == VI_EMPTY) {
      const unsigned long long old = atomicCAS(&set[h], VI_EMPTY, key);
      if (old == VI_EMPTY) return true;
      if (old == key) return false;
    }
    h = (h + 1) & (SIZE - 1);
  }
  *full = true;
  return false;
}

// pass 1: thread = (owned node, block nb), block = 256 nodes x one nb (9 slots).  ctl[0] =
// distinct values, ctl[1] = more than VI_MAX (no value-indexed storage), ctl[2] = some slot has
// more than 16 (no nibble indices), ctl[3 + S] = distinct values of slot S; skeys[S][32] = the
// slot's set, keys[VI_HASH] = the whole matrix's
template <bool TABLE>
__global__ __launch_bounds__(TPB) void k_vi_collect(Geo g, Material mat, const double* __restrict__ Ke,
                                                    unsigned long long* __restrict__ keys,
                                                    unsigned long long* __restrict__ skeys, unsigned* __restrict__ ctl) {
  constexpr int LS = 64;  // per-slot block set (a slot takes <= 16 values, else nibbles are out)
  __shared__ unsigned long long s_keys[9][LS];
  __shared__ unsigned s_over;
  for (int t = threadIdx.x; t < 9 * LS; t += TPB) (&s_keys[0][0])[t] = VI_EMPTY;
  if (threadIdx.x == 0) s_over = __hip_atomic_load(&ctl[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  if (s_over) return;  // uniform: the dictionary already overflowed
  const int n = blockIdx.x * TPB + threadIdx.x;
  const int nb = blockIdx.y;
  bool full = false;
  if (n < g.nown) {
    int i, j, k;
    node_ijk(g, n, i, j, k);
    double val[9];
    matrix_block<TABLE>(g, mat, Ke, g.xs + i, g.ys + j, g.zs + k, nb % 3 - 1, (nb / 3) % 3 - 1, nb / 9 - 1, val);
#pragma unroll
    for (int q = 0; q < 9; q++) {
      const unsigned long long key = (unsigned long long)__double_as_longlong(val[q]);
      if (key == VI_EMPTY) {
        full = true;
        continue;
      }
      bool lfull = false;
      vi_insert<LS>(s_keys[q], key, &lfull);
      if (lfull) {
        // more than LS values of one slot in this block: the slot cannot take nibble indices,
        // but the whole matrix may still fit the byte dictionary, so the value goes straight to
        // the global set (the per-slot sets are only kept for nibble indices)
        bool gfull = false;
        if (vi_insert<VI_HASH>(keys, key, &gfull) && atomicAdd(&ctl[0], 1u) >= (unsigned)VI_MAX) full = true;
        if (gfull) full = true;
        atomicOr(&ctl[2], 1u);
      }
    }
  }
  if (full) s_over = 1;
  __syncthreads();
  if (s_over) {
    if (threadIdx.x == 0) atomicOr(&ctl[1], 1u);
    return;
  }
  for (int t = threadIdx.x; t < 9 * LS; t += TPB) {
    const int q = t / LS;
    const unsigned long long key = s_keys[q][t % LS];
    if (key == VI_EMPTY) continue;
    bool gfull = false;
    if (vi_insert<VI_HASH>(keys, key, &gfull) && atomicAdd(&ctl[0], 1u) >= (unsigned)VI_MAX) atomicOr(&ctl[1], 1u);
    if (gfull) atomicOr(&ctl[1], 1u);
    const int S = nb * 9 + q;
    if (__hip_atomic_load(&ctl[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) continue;
    bool sfull = false;
    if (vi_insert<32>(skeys + S * 32, key, &sfull) && atomicAdd(&ctl[3 + S], 1u) >= 16u) atomicOr(&ctl[2], 1u);
    if (sfull) atomicOr(&ctl[2], 1u);
  }
}

// pass 2: thread = owned node; its 27 blocks in slot order, each value's index (the sets and
// their index maps staged in LDS) packed into 16-B chunks [n/64][chunk][n%64]
template <bool TABLE, int NIB>
__global__ __launch_bounds__(TPB) void k_vi_pack(Geo g, Material mat, const double* __restrict__ Ke,
                                                 const unsigned long long* __restrict__ keys,
                                                 const unsigned char* __restrict__ slot, u32x4* __restrict__ I) {
  constexpr int NK = NIB == 8 ? VI_HASH : NSLOT * 32;  // one set, or 32 entries per slot
  constexpr int CH = vi_chunks<NIB>(), PER = 128 / NIB;  // chunks per node, indices per chunk
  __shared__ unsigned long long s_keys[NK];
  __shared__ unsigned char s_slot[NK];
  for (int t = threadIdx.x; t < NK; t += TPB) {
    s_keys[t] = keys[t];
    s_slot[t] = slot[t];
  }
  __syncthreads();
  const int n = blockIdx.x * TPB + threadIdx.x;
  if (n >= g.nown) return;
  int i, j, k;
  node_ijk(g, n, i, j, k);
  u32x4* dst = I + (int64_t)(n >> 6) * (CH * 64) + (n & 63);
  unsigned w0 = 0, w1 = 0, w2 = 0, w3 = 0;
  for (int nb = 0; nb < 27; nb++) {
    double val[9];
    matrix_block<TABLE>(g, mat, Ke, g.xs + i, g.ys + j, g.zs + k, nb % 3 - 1, (nb / 3) % 3 - 1, nb / 9 - 1, val);
#pragma unroll
    for (int q = 0; q < 9; q++) {
      const unsigned long long key = (unsigned long long)__double_as_longlong(val[q]);
      const int S = nb * 9 + q;
      const int base = NIB == 8 ? 0 : S * 32, size = NIB == 8 ? VI_HASH : 32;
      unsigned h = vi_hash(key) & (size - 1);
      for (int probe = 0; probe < size && s_keys[base + h] != key; probe++) h = (h + 1) & (size - 1);
      const unsigned idx = s_slot[base + h];
      const int b = S % PER, word = b / (PER / 4), sh = NIB * (b % (PER / 4));
      if (word == 0) w0 |= idx << sh;
      else if (word == 1) w1 |= idx << sh;
      else if (word == 2) w2 |= idx << sh;
      else w3 |= idx << sh;
      if (b == PER - 1 || S == NSLOT - 1) {  // uniform: chunk complete (the last one padded with zeros)
        u32x4 v = {w0, w1, w2, w3};
        dst[(S / PER) * 64] = v;
        w0 = w1 = w2 = w3 = 0;
      }
    }
  }
}

// PCSetUp_Jacobi on FMT_VI
template <int NIB>
__global__ void k_jacobi_vi(Geo g, const u32x4* __restrict__ I, const double* __restrict__ dict,
                            double* __restrict__ dinv) {
  constexpr int CH = vi_chunks<NIB>();
  const int n = blockIdx.x * TPB + threadIdx.x;
  if (n >= g.nown) return;
  u32x4 w[CH];
  const u32x4* ip = I + (int64_t)(n >> 6) * (CH * 64) + (n & 63);
#pragma unroll
  for (int q = 0; q < CH; q++) w[q] = ip[q * 64];
#pragma unroll
  for (int r = 0; r < 3; r++) {
    const int S = 13 * 9 + r * 4;
    double d = dict[vi_entry<NIB>(S, vi_index<NIB>(w, S))];
    if (d != 0.0) d = 1.0 / d;
    if (d == 0.0) d = 1.0;
    dinv[3 * n + r] = d;
  }
}

// y = A x on FMT_VI, x gathered: k_spmv with the 122 16-B value pairs replaced by 16 (8) 16-B
// index chunks and the values read from the dictionary in LDS (interior lanes of a wave share an
// index: LDS broadcast).  Same node sweep (XCD slabs), same slot order and products as k_spmv, so
// y is bit-identical to the reference's AIJ MatMult (inode order, oracle/oracle.c row_part).  DBG (timing-only diagnostics, wrong products):
// bit 0 = no dictionary lookups (the index is the value), bit 1 = no x gathers.
template <bool DOT, bool GATED, int NIB, int DBG = 0>
__global__ __launch_bounds__(TPB) void k_spmv_vi(Geo g, const u32x4* __restrict__ I, const double* __restrict__ dict,
                                                 const double* __restrict__ x, double* __restrict__ y,
                                                 double* __restrict__ part, const CgState* __restrict__ cg,
                                                 SpmvTiling tl) {
  constexpr int CH = vi_chunks<NIB>(), NT = NIB == 8 ? VI_MAX : NSLOT * 16;
  __shared__ double tab[NT];
  __shared__ double sh[TPB / 64];
  if (GATED && cg->reason) return;
  for (int t = threadIdx.x; t < NT; t += TPB) tab[t] = dict[t];
  __syncthreads();
  int i = 0, j = 0, k = 0;
  const int n = spmv_node(g, tl.TX, tl.LPB, tl.nxc, tl.jgroups, tl.subl, i, j, k);
  double dot = 0.;
  if (n >= 0) {
    const int PX = g.PX, PXY = g.PX * g.PY;
    const int pc = (i + 1) + (j + 1) * PX + (k + 1) * PXY;
    const u32x4* ip = I + (int64_t)(n >> 6) * (CH * 64) + (n & 63);
    u32x4 w[CH];
#pragma unroll
    for (int q = 0; q < CH; q++) w[q] = __builtin_nontemporal_load(ip + q * 64);
    double xc0 = 0., xc1 = 0., xc2 = 0.;
    InodeRows<false> acc;
    acc.pres = present_mask(g, i, j, k);
#pragma unroll
    for (int nb = 0; nb < 27; nb++) {
      const int off = (nb % 3 - 1) + ((nb / 3) % 3 - 1) * PX + (nb / 9 - 1) * PXY;
      const double* xp = x + 3 * (int64_t)(pc + off);
      double xv[3];
      if (DBG & 2) {
        xv[0] = (double)(pc + off);
        xv[1] = xv[0] + 0.5;
        xv[2] = xv[0] + 0.25;
      } else {
        xv[0] = xp[0];
        xv[1] = xp[1];
        xv[2] = xp[2];
      }
      if (nb == 13) {
        xc0 = xv[0];
        xc1 = xv[1];
        xc2 = xv[2];
      }
#pragma unroll
      for (int q = 0; q < 9; q++) {
        const int S = nb * 9 + q, r = q / 3, cc = q % 3;
        const unsigned id = vi_index<NIB>(w, S);
        const double v = (DBG & 1) ? (double)id : tab[vi_entry<NIB>(S, id)];
        acc.term(nb, r, cc, v * xv[cc]);
      }
    }
    const double y0 = acc.row(0), y1 = acc.row(1), y2 = acc.row(2);
    __builtin_nontemporal_store(y0, &y[3 * n + 0]);
    __builtin_nontemporal_store(y1, &y[3 * n + 1]);
    __builtin_nontemporal_store(y2, &y[3 * n + 2]);
    if (DOT) dot = xc0 * y0 + xc1 * y1 + xc2 * y2;
  }
  if (DOT) {
    double s = block_sum<TPB>(dot, sh);
    if (threadIdx.x == 0) part[blockIdx.x] = s;
  }
}

// ---- block-indexed: one byte per 3x3 block.  A block position nb takes at most 21 distinct
// blocks (the diagonal; <= 11 elsewhere; 187 in all at 12^3 .. 40^3), so each node's 27 blocks
// are held as 27 bytes (+5 pad: 32 B per node) indexing one dictionary of blocks (<= 256 x 9
// values).  A block's key is its position and its 9 per-slot nibbles (nb << 36 | nibbles), so
// it is exact; built from the nibble dictionaries by two more passes (k_vib_collect, k_vib_pack).
// per-slot nibble of value key in slot S (sets staged in LDS: 32 entries per slot)
__device__ __forceinline__ unsigned vi_nibble(const unsigned long long* skeys, const unsigned char* smap, int S,
                                              unsigned long long key) {
  unsigned h = vi_hash(key) & 31u;
  for (int probe = 0; probe < 32 && skeys[S * 32 + h] != key; probe++) h = (h + 1) & 31u;
  return smap[S * 32 + h];
}

// pass 3: thread = (owned node, nb): the block's key into a per-block LDS set, then the global
// block set bkeys[VI_HASH]; ctl[0] = distinct blocks, ctl[1] = more than VI_MAX
template <bool TABLE>
__global__ __launch_bounds__(TPB) void k_vib_collect(Geo g, Material mat, const double* __restrict__ Ke,
                                                     const unsigned long long* __restrict__ skeys,
                                                     const unsigned char* __restrict__ smap,
                                                     unsigned long long* __restrict__ bkeys, unsigned* __restrict__ ctl) {
  constexpr int LS = 64;
  __shared__ unsigned long long s_set[LS];
  __shared__ unsigned long long s_keys[9 * 32];
  __shared__ unsigned char s_map[9 * 32];
  __shared__ unsigned s_over;
  const int nb = blockIdx.y;
  for (int t = threadIdx.x; t < 9 * 32; t += TPB) {
    s_keys[t] = skeys[nb * 9 * 32 + t];
    s_map[t] = smap[nb * 9 * 32 + t];
  }
  for (int t = threadIdx.x; t < LS; t += TPB) s_set[t] = VI_EMPTY;
  if (threadIdx.x == 0) s_over = 0;
  __syncthreads();
  const int n = blockIdx.x * TPB + threadIdx.x;
  bool full = false;
  if (n < g.nown) {
    int i, j, k;
    node_ijk(g, n, i, j, k);
    double val[9];
    matrix_block<TABLE>(g, mat, Ke, g.xs + i, g.ys + j, g.zs + k, nb % 3 - 1, (nb / 3) % 3 - 1, nb / 9 - 1, val);
    unsigned long long key = (unsigned long long)nb << 36;
#pragma unroll
    for (int q = 0; q < 9; q++)
      key |= (unsigned long long)vi_nibble(s_keys, s_map, q, (unsigned long long)__double_as_longlong(val[q]))
             << (4 * q);
    vi_insert<LS>(s_set, key, &full);
  }
  if (full) s_over = 1;
  __syncthreads();
  if (s_over) {
    if (threadIdx.x == 0) atomicOr(&ctl[1], 1u);
    return;
  }
  for (int t = threadIdx.x; t < LS; t += TPB) {
    const unsigned long long key = s_set[t];
    if (key == VI_EMPTY) continue;
    bool gfull = false;
    if (vi_insert<VI_HASH>(bkeys, key, &gfull) && atomicAdd(&ctl[0], 1u) >= (unsigned)VI_MAX) atomicOr(&ctl[1], 1u);
    if (gfull) atomicOr(&ctl[1], 1u);
  }
}

// pass 4: thread = (owned node, nb): the block's byte index, byte nb of the node's 32
// ([n/64][2][64] x 16 B)
template <bool TABLE>
__global__ __launch_bounds__(TPB) void k_vib_pack(Geo g, Material mat, const double* __restrict__ Ke,
                                                  const unsigned long long* __restrict__ skeys,
                                                  const unsigned char* __restrict__ smap,
                                                  const unsigned long long* __restrict__ bkeys,
                                                  const unsigned char* __restrict__ bmap, unsigned char* __restrict__ I) {
  __shared__ unsigned long long s_keys[9 * 32];
  __shared__ unsigned char s_map[9 * 32];
  __shared__ unsigned long long s_bkeys[VI_HASH];
  __shared__ unsigned char s_bmap[VI_HASH];
  const int nb = blockIdx.y;
  for (int t = threadIdx.x; t < 9 * 32; t += TPB) {
    s_keys[t] = skeys[nb * 9 * 32 + t];
    s_map[t] = smap[nb * 9 * 32 + t];
  }
  for (int t = threadIdx.x; t < VI_HASH; t += TPB) {
    s_bkeys[t] = bkeys[t];
    s_bmap[t] = bmap[t];
  }
  __syncthreads();
  const int n = blockIdx.x * TPB + threadIdx.x;
  if (n >= g.nown) return;
  int i, j, k;
  node_ijk(g, n, i, j, k);
  double val[9];
  matrix_block<TABLE>(g, mat, Ke, g.xs + i, g.ys + j, g.zs + k, nb % 3 - 1, (nb / 3) % 3 - 1, nb / 9 - 1, val);
  unsigned long long key = (unsigned long long)nb << 36;
#pragma unroll
  for (int q = 0; q < 9; q++)
    key |= (unsigned long long)vi_nibble(s_keys, s_map, q, (unsigned long long)__double_as_longlong(val[q])) << (4 * q);
  unsigned h = vi_hash(key) & (VI_HASH - 1);
  for (int probe = 0; probe < VI_HASH && s_bkeys[h] != key; probe++) h = (h + 1) & (VI_HASH - 1);
  I[(((int64_t)(n >> 6) * 2 + (nb >> 4)) * 64 + (n & 63)) * 16 + (nb & 15)] = s_bmap[h];
}

// ---- block-indexed storage in one pass over the blocks (round 3).  Round 2 evaluated every
// matrix block three times (k_vi_collect, k_vib_collect, k_vib_pack) with a host round trip
// after each of the first two.  Here every block is evaluated once:
//   k_vib_build (thread = owned node x block position nb, 256 nodes per workgroup): the block's
//     9 values go into per-slot LDS sets, the sets into per-slot global sets (VB_GSV entries,
//     open addressing; an entry never moves once written, so its position is an exact 6-bit name
//     of the value within its slot); the block's code nb << 54 | the 9 positions (6 bits each)
//     is then exact too, and goes through an LDS set into the global block-code set, whose
//     position (< VI_HASH) is written per (nb, node) [27][nown] (2 B);
//   the host (one readback + sync) sorts each slot's values and the block codes into the
//     dictionary (by block position, then the 9 values' ranks in their slots: the order round 2
//     produced), and maps every block-set position to its dictionary index;
//   k_vib_remap (thread = owned node) streams the 27 positions through that map into the 27
//     index bytes ([n/64][2][n%64] x 16 B, as before).
// ctl[0] = distinct blocks, ctl[1] = overflow (a set full, a NaN-pattern value, > VI_MAX blocks).

// insert key into an open-addressing set; returns the key's position (new or found), -1 when the
// probe budget is exhausted; *isnew when this call wrote it
template <int SIZE>
__device__ __forceinline__ int vi_insert_pos(unsigned long long* set, unsigned long long key, bool* isnew) {
  unsigned h = vi_hash(key) & (SIZE - 1);
  *isnew = false;
  for (int probe = 0; probe < SIZE; probe++) {
    const unsigned long long cur = __hip_atomic_load(&set[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (cur == key) return (int)h;
    if (cur == VI_EMPTY) {
      const unsigned long long old = atomicCAS(&set[h], VI_EMPTY, key);
      if (old == VI_EMPTY) {
        *isnew = true;
        return (int)h;
      }
      if (old == key) return (int)h;
    }
    h = (h + 1) & (SIZE - 1);
  }
  return -1;
}

template <bool TABLE>
__global__ __launch_bounds__(TPB) void k_vib_build(Geo g, Material mat, const double* __restrict__ Ke,
                                                   unsigned long long* __restrict__ gsv,
                                                   unsigned long long* __restrict__ gbk,
                                                   unsigned short* __restrict__ bpos, unsigned* __restrict__ ctl,
                                                   const unsigned* __restrict__ xslot) {
  constexpr int LSV = 64, LSB = 64;
  __shared__ unsigned long long s_v[9][LSV];
  __shared__ unsigned char s_vp[9][LSV];
  __shared__ unsigned long long s_b[LSB];
  __shared__ unsigned short s_bp[LSB];
  __shared__ unsigned s_over;
  for (int t = threadIdx.x; t < 9 * LSV; t += TPB) (&s_v[0][0])[t] = VI_EMPTY;
  for (int t = threadIdx.x; t < LSB; t += TPB) s_b[t] = VI_EMPTY;
  if (threadIdx.x == 0) s_over = __hip_atomic_load(&ctl[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  if (s_over) return;  // uniform: the build already overflowed
  const int n = blockIdx.x * TPB + threadIdx.x;
  const int nb = blockIdx.y;
  const bool own = n < g.nown && !(xslot && xslot[n]);  // exception nodes stay out of the dictionary
  bool bad = false, isnew;
  int lp[9];
  if (own) {
    int i, j, k;
    node_ijk(g, n, i, j, k);
    double val[9];
    matrix_block<TABLE>(g, mat, Ke, g.xs + i, g.ys + j, g.zs + k, nb % 3 - 1, (nb / 3) % 3 - 1, nb / 9 - 1, val);
#pragma unroll
    for (int q = 0; q < 9; q++) {
      const unsigned long long key = (unsigned long long)__double_as_longlong(val[q]);
      lp[q] = key == VI_EMPTY ? -1 : vi_insert_pos<LSV>(s_v[q], key, &isnew);
      if (lp[q] < 0) bad = true;
    }
  }
  if (bad) s_over = 1;
  __syncthreads();
  if (s_over) {
    if (threadIdx.x == 0) atomicOr(&ctl[1], 1u);
    return;
  }
  for (int t = threadIdx.x; t < 9 * LSV; t += TPB) {  // this group's values of each slot -> the slot's set
    const int q = t / LSV;
    const unsigned long long key = s_v[q][t % LSV];
    if (key == VI_EMPTY) continue;
    const int gp = vi_insert_pos<VB_GSV>(gsv + (nb * 9 + q) * VB_GSV, key, &isnew);
    if (gp < 0) s_over = 1;
    (&s_vp[0][0])[t] = (unsigned char)(gp < 0 ? 0 : gp);
  }
  __syncthreads();
  if (s_over) {
    if (threadIdx.x == 0) atomicOr(&ctl[1], 1u);
    return;
  }
  int lb = 0;
  if (own) {
    unsigned long long code = (unsigned long long)nb << 54;
#pragma unroll
    for (int q = 0; q < 9; q++) code |= (unsigned long long)s_vp[q][lp[q]] << (6 * q);
    lb = vi_insert_pos<LSB>(s_b, code, &isnew);
    if (lb < 0) s_over = 1;
  }
  __syncthreads();
  if (s_over) {
    if (threadIdx.x == 0) atomicOr(&ctl[1], 1u);
    return;
  }
  for (int t = threadIdx.x; t < LSB; t += TPB) {  // this group's block codes -> the block set
    const unsigned long long key = s_b[t];
    if (key == VI_EMPTY) continue;
    const int gp = vi_insert_pos<VI_HASH>(gbk, key, &isnew);
    if (gp < 0 || (isnew && atomicAdd(&ctl[0], 1u) >= (unsigned)VI_MAX)) atomicOr(&ctl[1], 1u);
    s_bp[t] = (unsigned short)(gp < 0 ? 0 : gp);
  }
  __syncthreads();
  if (own) bpos[(int64_t)nb * g.nown + n] = s_bp[lb];
}

// the 27 block-set positions of every owned node -> its 27 index bytes (+5 zero pad); an
// exception node gets 27 zero bytes and its slot + 1 in bytes 28-31
__global__ __launch_bounds__(TPB) void k_vib_remap(Geo g, const unsigned short* __restrict__ bpos,
                                                   const unsigned char* __restrict__ bmap, u32x4* __restrict__ I,
                                                   const unsigned* __restrict__ xslot) {
  __shared__ unsigned char s_map[VI_HASH];
  for (int t = threadIdx.x; t < VI_HASH / 16; t += TPB)
    reinterpret_cast<u32x4*>(s_map)[t] = reinterpret_cast<const u32x4*>(bmap)[t];
  __syncthreads();
  const int n = blockIdx.x * TPB + threadIdx.x;
  if (n >= g.nown) return;
  unsigned w[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
  const unsigned xs = xslot ? xslot[n] : 0u;
  if (xs) w[7] = xs;
  else {
#pragma unroll
    for (int nb = 0; nb < 27; nb++) w[nb >> 2] |= (unsigned)s_map[bpos[(int64_t)nb * g.nown + n]] << (8 * (nb & 3));
  }
  u32x4* dst = I + (int64_t)(n >> 6) * 128 + (n & 63);
  dst[0] = u32x4{w[0], w[1], w[2], w[3]};
  dst[64] = u32x4{w[4], w[5], w[6], w[7]};
}

// ---- exception nodes (laws with a per-GP tangent).  A J2 law whose few plastic Gauss points sit
// under the load (config 5: 552-2,920 of 16.8 M) leaves every other element with the elastic
// branch's tangent, bit for bit, and so with one element matrix: the nodes whose elements are all
// such "plain" elements assemble into the same few blocks as the elastic law's matrix.  Only the
// nodes touching a non-plain element (the exceptions) keep their 27 blocks as plain values.
// cref: the plastic law's elastic-branch tangent; other laws: GP 0 of the context's first element.
// cref[36], then cref8[36][8] = the same tangent at the 8 Gauss points of a one-element box (the
// ctan layout k_ref_ke reads)
__global__ void k_cref(Material mat, const double* __restrict__ ctan, int64_t ngp, double* __restrict__ cref) {
  if (threadIdx.x) return;
  if (mat.law == MCX_LAW_PLASTIC) {
    double G, K, C[36];
    j2_moduli(mat, G, K);
    j2_elastic_tangent(G, K, C);
#pragma unroll
    for (int q = 0; q < 36; q++) cref[q] = C[q];
  } else {
    for (int q = 0; q < 36; q++) cref[q] = ctan[q * ngp];
  }
  for (int q = 0; q < 36 * 8; q++) cref[36 + q] = cref[q / 8];
}

// kref [8 a][8 b][9]: the element matrix of an element whose 8 tangents are cref — ke_body on a
// one-element box (E = 1: ctan index (kl, gp), Ke index (a*8 + b)*9 + q), the arithmetic
// k_element_ke performs for every such element, so kref equals their matrices bit for bit
__global__ void k_ref_ke(Geo g, const double* __restrict__ cref8, double* __restrict__ kref) {
  const int t = threadIdx.x;
  if (t >= 16) return;
  Geo g1 = g;
  g1.nelem = 1;
  if (t & 1) ke_body<1>(g1, 0, t >> 1, cref8, kref);
  else ke_body<0>(g1, 0, t >> 1, cref8, kref);
}

// plain[le] = the 8 Gauss points' tangents (ctan [36][8][nelem]) all equal cref bit for bit
__global__ __launch_bounds__(TPB) void k_elem_plain(Geo g, const double* __restrict__ ctan,
                                                    const double* __restrict__ cref, unsigned char* __restrict__ plain) {
  const int64_t le = (int64_t)blockIdx.x * TPB + threadIdx.x;
  const int64_t E = g.nelem, NG = 8 * E;
  if (le >= E) return;
  bool same = true;
  for (int kl = 0; kl < 36; kl++) {
    const long long r = __double_as_longlong(cref[kl]);
#pragma unroll
    for (int gp = 0; gp < 8; gp++) same = same && __double_as_longlong(ctan[kl * NG + gp * E + le]) == r;
  }
  plain[le] = same ? 1 : 0;
}

// Exception nodes (an owned node touching an element that is not plain) get their slots by an
// ordered compaction: slot = the number of exception nodes before n in owned-node order (three
// passes: per-block counts, one block's scan of the counts, per-node ranks).  Neighbouring
// exception nodes then hold neighbouring slots, so a wave of consecutive slots reads the
// slot-fastest exc array in whole lines, and the slots are deterministic (round 4 took them from
// an atomic counter, in arrival order).
__device__ __forceinline__ bool node_is_exc(const Geo& g, const unsigned char* __restrict__ plain, int n) {
  int i, j, k;
  node_ijk(g, n, i, j, k);
  const int gi = g.xs + i, gj = g.ys + j, gk = g.zs + k;
  bool exc = false;
  for (int oz = 0; oz < 2; oz++)
    for (int oy = 0; oy < 2; oy++)
      for (int ox = 0; ox < 2; ox++) {
        const int ex = gi - ox, ey = gj - oy, ez = gk - oz;
        if (ex < 0 || ex > g.NX - 2 || ey < 0 || ey > g.NY - 2 || ez < 0 || ez > g.NZ - 2) continue;
        const int64_t le = (ex - g.ex0) + (int64_t)(ey - g.ey0) * g.nex + (int64_t)(ez - g.ez0) * g.nex * g.ney;
        exc = exc || !plain[le];
      }
  return exc;
}

// pass 1: xslot[n] = 1 for an exception node (0 otherwise), cnt[block] = the block's count
__global__ __launch_bounds__(TPB) void k_exc_flag(Geo g, const unsigned char* __restrict__ plain,
                                                  unsigned* __restrict__ xslot, unsigned* __restrict__ cnt) {
  const int n = blockIdx.x * TPB + threadIdx.x;
  const bool e = n < g.nown && node_is_exc(g, plain, n);
  if (n < g.nown) xslot[n] = e ? 1u : 0u;
  const int c = __syncthreads_count(e);
  if (threadIdx.x == 0) cnt[blockIdx.x] = (unsigned)c;
}

// pass 2 (one block): cnt[0..nb) -> exclusive prefix sums, the total to *total (exceptions: the
// block build's ctl[2], read back with its sets)
__global__ __launch_bounds__(1024) void k_exc_scan(unsigned* __restrict__ cnt, int nb, unsigned* __restrict__ total) {
  __shared__ unsigned s[1024];
  const int t = threadIdx.x, per = (nb + 1023) / 1024, lo = min(nb, t * per), hi = min(nb, lo + per);
  unsigned sum = 0u;
  for (int q = lo; q < hi; q++) sum += cnt[q];
  s[t] = sum;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {  // inclusive scan of the 1024 chunk sums
    const unsigned v = t >= o ? s[t - o] : 0u;
    __syncthreads();
    s[t] += v;
    __syncthreads();
  }
  unsigned run = s[t] - sum;
  for (int q = lo; q < hi; q++) {
    const unsigned c = cnt[q];
    cnt[q] = run;
    run += c;
  }
  if (t == 1023) *total = s[1023];
}

// pass 3: slot = the block's offset + the node's rank among the block's exception nodes;
// xslot[n] = slot + 1, xlist[slot] = n
__global__ __launch_bounds__(TPB) void k_exc_assign(Geo g, unsigned* __restrict__ xslot, int* __restrict__ xlist,
                                                    const unsigned* __restrict__ cnt) {
  __shared__ unsigned wsum[TPB / 64];
  const int n = blockIdx.x * TPB + threadIdx.x;
  const bool e = n < g.nown && xslot[n] != 0u;
  const unsigned long long m = __ballot(e);
  const unsigned lane_rank = __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) wsum[w] = (unsigned)__popcll(m);
  __syncthreads();
  unsigned off = cnt[blockIdx.x];
  for (int q = 0; q < w; q++) off += wsum[q];
  if (n < g.nown) {
    const unsigned slot = off + lane_rank;
    xslot[n] = e ? slot + 1u : 0u;
    if (e) xlist[slot] = n;
  }
}

// the exception nodes' 27 blocks, value (nb, q) of slot s at exc[exc_base(s) + (nb * 9 + q) * 64]
// (AoSoA): thread = (slot, nb); each element block from kref (plain elements) or from Ke (the
// others: k_element_ke forms only those)
__global__ __launch_bounds__(TPB) void k_exc_fill(Geo g, Material mat, const double* __restrict__ Ke,
                                                  const double* __restrict__ kref,
                                                  const unsigned char* __restrict__ plain,
                                                  const int* __restrict__ xlist, int64_t nexc,
                                                  double* __restrict__ exc) {
  const int64_t t = (int64_t)blockIdx.x * TPB + threadIdx.x;
  const int nb = blockIdx.y;
  if (t >= nexc) return;
  const int n = xlist[t];
  int i, j, k;
  node_ijk(g, n, i, j, k);
  double val[9];
  matrix_block<true>(g, mat, Ke, g.xs + i, g.ys + j, g.zs + k, nb % 3 - 1, (nb / 3) % 3 - 1, nb / 9 - 1, val,
                     kref, plain);
#pragma unroll
  for (int q = 0; q < 9; q++) exc[exc_base(t) + (nb * 9 + q) * 64] = val[q];
}

__device__ __forceinline__ double jacobi_inv(double d) {
  if (d != 0.0) d = 1.0 / d;
  if (d == 0.0) d = 1.0;
  return d;
}

// dinv per owned DOF, and jix[n] = the node's diagonal-block index (block 13 = offset 0,0,0)
// (exc: an exception node's diagonal block is its plain block 13)
__global__ void k_jacobi_vib(Geo g, const unsigned char* __restrict__ I, const double* __restrict__ bdict,
                             double* __restrict__ dinv, unsigned char* __restrict__ jix, const double* __restrict__ exc) {
  const int n = blockIdx.x * TPB + threadIdx.x;
  if (n >= g.nown) return;
  const int id = I[(((int64_t)(n >> 6) * 2 + 0) * 64 + (n & 63)) * 16 + 13];
  const unsigned xs =
      exc ? *reinterpret_cast<const unsigned*>(I + (((int64_t)(n >> 6) * 2 + 1) * 64 + (n & 63)) * 16 + 12) : 0u;
  jix[n] = xs ? 255 : (unsigned char)id;  // 255: the CG kernels read dinv (jac_inv)
#pragma unroll
  for (int r = 0; r < 3; r++)
    dinv[3 * n + r] = jacobi_inv(xs ? exc[exc_base(xs - 1) + (13 * 9 + r * 4) * 64] : bdict[id * VIB_STRIDE + r * 4]);
}

// the dictionary's inverse diagonals [VI_MAX][3] (same values as k_jacobi_vib's dinv)
__global__ void k_jacobi_vib_dict(const double* __restrict__ bdict, double* __restrict__ jdd) {
  const int t = blockIdx.x * TPB + threadIdx.x;
  if (t >= 3 * VI_MAX) return;
  jdd[t] = jacobi_inv(bdict[(t / 3) * VIB_STRIDE + (t % 3) * 4]);
}

// y = A x on block-indexed FMT_VI: 2 16-B index chunks per node (27 block bytes), each block's
// 9 values from the dictionary in LDS (4 x 16-B + 8-B reads), x gathered.  Same slot order and
// products as k_spmv: bit-identical to the reference's AIJ MatMult (inode order, oracle/oracle.c row_part).
// EXC: exception nodes (slot + 1 in bytes 28-31) read their blocks from exc [slot][27][9].
template <bool DOT, bool GATED, bool EXC = false>
__global__ __launch_bounds__(TPB) void k_spmv_vib(Geo g, const u32x4* __restrict__ I,
                                                  const double* __restrict__ bdict, const double* __restrict__ x,
                                                  double* __restrict__ y, double* __restrict__ part,
                                                  const CgState* __restrict__ cg, SpmvTiling tl,
                                                  const double* __restrict__ exc = nullptr) {
  __shared__ double2 tab[VI_MAX * VIB_STRIDE / 2];
  __shared__ double sh[TPB / 64];
  if (GATED && cg->reason) return;
  for (int t = threadIdx.x; t < VI_MAX * VIB_STRIDE / 2; t += TPB) tab[t] = reinterpret_cast<const double2*>(bdict)[t];
  __syncthreads();
  int i = 0, j = 0, k = 0;
  const int n = spmv_node(g, tl.TX, tl.LPB, tl.nxc, tl.jgroups, tl.subl, i, j, k);
  double dot = 0.;
  if (n >= 0) {
    const int PX = g.PX, PXY = g.PX * g.PY;
    const int pc = (i + 1) + (j + 1) * PX + (k + 1) * PXY;
    const u32x4* ip = I + (int64_t)(n >> 6) * (2 * 64) + (n & 63);
    const u32x4 w0 = __builtin_nontemporal_load(ip), w1 = __builtin_nontemporal_load(ip + 64);
    double xc0 = 0., xc1 = 0., xc2 = 0.;
    InodeRows<false> acc;
    acc.pres = present_mask(g, i, j, k);
#pragma unroll
    for (int nb = 0; nb < 27; nb++) {
      const int off = (nb % 3 - 1) + ((nb / 3) % 3 - 1) * PX + (nb / 9 - 1) * PXY;
      const double* xp = x + 3 * (int64_t)(pc + off);
      const double xv[3] = {xp[0], xp[1], xp[2]};
      if (nb == 13) {
        xc0 = xv[0];
        xc1 = xv[1];
        xc2 = xv[2];
      }
      const unsigned word = nb < 16 ? w0[nb >> 2] : w1[(nb - 16) >> 2];
      const unsigned id = (word >> (8 * (nb & 3))) & 255u;
      double a[9];
      if (EXC && w1[3]) {
#pragma unroll
        for (int q = 0; q < 9; q++) a[q] = exc[exc_base(w1[3] - 1) + (nb * 9 + q) * 64];
      } else {
        const double2* e = tab + id * (VIB_STRIDE / 2);
        const double2 a01 = e[0], a23 = e[1], a45 = e[2], a67 = e[3], a8 = e[4];
        a[0] = a01.x, a[1] = a01.y, a[2] = a23.x, a[3] = a23.y, a[4] = a45.x, a[5] = a45.y, a[6] = a67.x;
        a[7] = a67.y, a[8] = a8.x;
      }
#pragma unroll
      for (int q = 0; q < 9; q++) acc.term(nb, q / 3, q % 3, a[q] * xv[q % 3]);
    }
    const double y0 = acc.row(0), y1 = acc.row(1), y2 = acc.row(2);
    __builtin_nontemporal_store(y0, &y[3 * n + 0]);
    __builtin_nontemporal_store(y1, &y[3 * n + 1]);
    __builtin_nontemporal_store(y2, &y[3 * n + 2]);
    if (DOT) dot = xc0 * y0 + xc1 * y1 + xc2 * y2;
  }
  if (DOT) {
    double s = block_sum<TPB>(dot, sh);
    if (threadIdx.x == 0) part[blockIdx.x] = s;
  }
}

// y = A x on block-indexed FMT_VI with x staged in LDS, z-marching: k_spmv_vim's ring of three x
// planes (rows j0-1 .. j0+TY, prefetched in registers one plane ahead) with the block dictionary
// in LDS beside it.  The gathered kernel (k_spmv_vib) spends most of its time in the 81 8-B x
// loads per node at a 24-B lane stride; here x comes from LDS and HBM streams 32 B of indices
// per node.  Same slot order and products as k_spmv: bit-identical to the reference's AIJ MatMult (inode order, oracle/oracle.c row_part).
// FP: the CG's p update (VecAYPX) fused into the SpMV's staging of p (single rank,
// value-indexed block storage, Jacobi from the diagonal index).  The kernel of CG iteration i
// reads p(i-1) from pb[(i-1)&1], r and the index bytes while it marches, computes
// p(i) = z + (beta/betaold) p(i-1) with z = r D^-1 (p(0) = z) for every staged node — its own and
// the halo rows of the neighbouring tiles alike, the operations k_cg_pupdate performs — writes
// p(i) of its own nodes to pb[i&1] and multiplies the staged p(i).  p is double-buffered because
// a tile reads its neighbours' p(i-1) while they write their p(i); the two buffers also let
// VecAXPY(x) run every second iteration in the update kernel (k_cg_update_x: x + a(i-1) p(i-1)
// + a(i) p(i), in PETSc's order).  Results are bitwise those of k_cg_pupdate + k_spmv_vibm +
// k_cg_update; p is read once per iteration instead of twice, x half as often.
struct FusedP {
  const double* r = nullptr;
  const double* jdd = nullptr;          // [VI_MAX][3] inverse diagonals of the dictionary blocks
  const unsigned char* jix = nullptr;   // owned nodes' diagonal-block index
  double* pb[2] = {nullptr, nullptr};   // padded p, double-buffered
};

// PATCH: a wave covers a 16 x 4 node patch of the tile instead of 64 nodes of one row, and the
// staged rows are padded to RL = 16 mod 32 doubles (the two rows a 32-lane ds_read_b64 group reads
// then fall on disjoint banks).  A tile row's two x-edge nodes then sit in 2 of the tile's 16
// patches instead of 2 of its 4 row quarters: with UNI, 14 of 16 waves of an interior tile plane
// take the scalar-dictionary path instead of 8 of 16.
template <int TX, bool PATCH>
constexpr int vibm_rl() {
  return PATCH ? 3 * (TX + 2) + ((16 - (3 * (TX + 2)) % 32) + 32) % 32 : 3 * (TX + 2);
}

template <bool DOT, bool GATED, int TX, int TY, bool XV = true, bool UNI = false, bool PATCH = false, bool FMA = false,
          bool FP = false, bool RING3 = false, bool EXC = false, bool WD = false, int LG = 1>
__global__ __launch_bounds__(TX * TY) void k_spmv_vibm(Geo g, const u32x4* __restrict__ I,
                                                       const double* __restrict__ bdict, const double* __restrict__ x,
                                                       double* __restrict__ y, double* __restrict__ part,
                                                       const CgState* __restrict__ cg, ZTiling zt, FusedP fp = {},
                                                       const double* __restrict__ exc = nullptr) {
  static_assert(!PATCH || (TX % 16 == 0 && TY % 4 == 0 && TX * TY == 1024), "16 x 4 patches");
  constexpr int T = TX * TY, RL = vibm_rl<TX, PATCH>(), PR = TY + 2, PLANE = PR * RL;  // doubles per staged plane
  constexpr int NL = (PLANE + T - 1) / T;                                      // x loads per thread per plane
  // ring of x planes: 4 slots where they fit the LDS (TX <= 128: plane k+2 then goes to the slot
  // of plane k-2, which plane k does not read, so one barrier per plane), else 3 (256x4 tiles:
  // plane k+2 overwrites plane k-1's slot after a barrier, and a second barrier publishes it)
  constexpr int R = TX <= 128 && !RING3 ? 4 : 3;  // RING3: A/B of the 3-slot ring (option vi_ring3)
  __shared__ double xs[R][PLANE];
  __shared__ double2 tab[VI_MAX * VIB_STRIDE / 2];
  __shared__ double sh[T / 64];
  __shared__ double s_jdd[FP ? 3 * VI_MAX : 1];
  // EXC: the tile's exception nodes, computed after the march by the whole block (one node per
  // thread) instead of inside their plane, where each one's nine dependent rounds of global
  // loads held the plane's barrier for every wave of the block
  // The list is split into one segment per wave, filled in (plane, lane) order from a ballot, so
  // every node's list position, hence the pass's thread -> node map and the block's p.w partial,
  // is a function of the tile alone: run-to-run deterministic (an LDS atomic counter handed out
  // positions in wave arrival order).
  constexpr int XL = EXC ? VI_EXC_LIST : 1;
  constexpr int NW = T / 64, SEG = XL / NW > 0 ? XL / NW : 1;
  __shared__ int s_xl[XL];
  __shared__ int s_wn[EXC ? NW : 1];
  if (GATED && cg->reason) return;
  const int b = blockIdx.x;
  const int xcd = b & 7, t8 = b >> 3;
  const int slab = (zt.nty + 7) >> 3;
  const int ty0 = xcd * slab;
  const int nty_here = min(slab, zt.nty - ty0);
  const int per = max(nty_here, 0) * zt.ntx * zt.nzc;
  if (t8 >= per) {  // whole block idle (uniform): still write the partial
    if (DOT && threadIdx.x == 0) part[blockIdx.x] = 0.;
    return;
  }
  const int txi = t8 % zt.ntx, r8 = t8 / zt.ntx;  // x tiles fastest, then the slab's tile rows, then z-chunks
  const int tyi = ty0 + r8 % nty_here, zc = r8 / nty_here;
  const int i0 = txi * TX, j0 = tyi * TY;
  const int k0 = zc * zt.kc, k1 = min(g.nz, k0 + zt.kc);
  const int me = threadIdx.x;
  // FP: the CG step's scalars and the p buffers of this iteration
  const int cgi = FP ? cg->i : 0;
  const double cb = FP ? cg->bcoef : 0.;
  const double* psrc = FP ? fp.pb[(cgi & 1) ^ 1] : x;
  double* pdst = FP ? fp.pb[cgi & 1] : nullptr;
  const int wv = me >> 6, ln = me & 63;
  // PATCH: wave wv -> 16 x 4 patch (px, py).  The waves of a workgroup go to the CU's 4 SIMDs
  // round robin (SIMD wv % 4), and the patches holding a tile's x-edge column (px = 0 or the
  // last) or y-edge row (py = 0 or the last) are the ones whose nodes differ in their block
  // indices (domain boundary, Dirichlet neighbours): they take the slower LDS-dictionary path.
  // Row-major numbering put a tile's 4 x-edge patches on one SIMD, whose waves then finished
  // the plane last; the Latin square (SIMD = (px + py) mod 4 within each group of 4 columns)
  // puts any column's and any row's patches on different SIMDs.
  constexpr int TYP = TY / 4;
  auto lane_xy = [&](int tid, int& lxo, int& lyo) {  // thread -> node of the tile
    const int wq = tid >> 6, lq = tid & 63;
    int px = wq % (TX / 16), py = wq / (TX / 16);
    if (PATCH && zt.wmap) {
      py = (wq >> 2) % TYP;
      px = (wq / (4 * TYP)) * 4 + (((wq & 3) - py) & 3);
    }
    lxo = PATCH ? px * 16 + (lq & 15) : tid % TX;
    lyo = PATCH ? py * 4 + (lq >> 4) : tid / TX;
  };
  int lx, ly;
  lane_xy(me, lx, ly);
  const int i = i0 + lx, j = j0 + ly;
  const bool inxy = i < g.nx && j < g.ny;
  const int PX = g.PX, PXY = g.PX * g.PY;
  // WD: this wave's 16 x 4 patch in the descriptor grid (a patch wholly outside the domain has
  // none: its planes count as not uniform, and its lanes compute nothing)
  static_assert(!WD || (UNI && PATCH && !FP && !EXC), "wave descriptors: the scalar-dictionary patch kernels");
  // FP's fstore reads the Jacobi entry from the dictionary's s_jdd without jac_inv's jix 255
  // redirect: a matrix with exception nodes never takes the fused p update (fusep checks vi_nexc)
  static_assert(!(FP && EXC), "the fused p update has no exception-node Jacobi redirect");
  const int gpx = (i0 + (lx & ~15)) >> 4, gpy = (j0 + (ly & ~3)) >> 2;  // (wave-uniform)
  const bool wdv = WD && gpx < zt.npx && gpy < zt.npy;
  // lane ln holds descriptor word ln & 31 of plane k (build_wdesc's layout)
  auto dload = [&](int k) -> unsigned {
    if (!wdv || k >= k1) return 0u;
    return __builtin_nontemporal_load(zt.wd + ((((int64_t)k * zt.npy + gpy) * zt.npx + gpx) << 5) + (me & 31));
  };
  // the planes whose waves skip the per-lane index words: uniform, or (FMA rows, wdm 2) two-set
  auto wskip = [&](unsigned f) -> bool {
    return FMA ? (f & 1u) || (zt.wdm == 2 && (f & 4u)) : (f & 3u) == 3u;
  };
  const int len = 3 * min(TX + 2, g.nx + 2 - i0);  // doubles of a staged row that exist in the padded box
  const int rows = min(TY + 2, g.ny + 2 - j0);      // staged rows (j0-1 ..) that exist (padded j <= ny)
  auto xload = [&](int p, int m) -> double {        // x of node plane p (-1 .. nz), staged element me + m T
    const int e = me + m * T;
    const int rr = e / RL, o = e - rr * RL;
    if (e >= PLANE || o >= len || rr >= rows) return 0.;
    return x[3 * (int64_t)(i0 + (j0 + rr) * PX + (p + 1) * PXY) + o];
  };
  auto xstore = [&](int slot, int m, double v) {
    const int e = me + m * T;
    if (e < PLANE) xs[slot][e] = v;
  };
  auto iload = [&](int k, u32x4& w0, u32x4& w1) {
    if (inxy) {
      const int n = i + g.nx * (j + g.ny * k);
      const u32x4* ip = I + (int64_t)(n >> 6) * (2 * 64) + (n & 63);
      w0 = __builtin_nontemporal_load(ip);
      w1 = __builtin_nontemporal_load(ip + 64);
    }
  };
  // FP staging of element me + m T of plane p: load p(i-1), r, the index byte and (own nodes) x;
  // then p(i) into the ring (and, own nodes, to pb[i&1] and x).  Elements outside the domain are
  // the zero ghost layer.
  struct Fe {
    double po, rv;
    unsigned jx;
  };
  auto fload = [&](int p, int m, Fe& f) {
    f.po = f.rv = 0.;
    f.jx = 0u;
    const int e = me + m * T;
    const int rr = e / RL, o = e - rr * RL;
    if (e >= PLANE || o >= len || rr >= rows) return;
    const int gi = i0 - 1 + o / 3, gj = j0 - 1 + rr;
    if (gi < 0 || gi >= g.nx || gj < 0 || gj >= g.ny || p < 0 || p >= g.nz) return;
    const int64_t n = gi + (int64_t)g.nx * (gj + (int64_t)g.ny * p);
    const int d = o - 3 * (o / 3);
    f.rv = fp.r[3 * n + d];
    f.jx = fp.jix[n];
    if (cgi > 0) f.po = psrc[3 * (int64_t)(i0 + (j0 + rr) * PX + (p + 1) * PXY) + o];
  };
  auto fstore = [&](int slot, int p, int m, const Fe& f) {
    int e = me + m * T;
    // recompute the element's indices here instead of keeping fload's live across the plane's
    // products (an opaque copy stops the compiler from reusing them: 128 VGPRs and spills else)
    asm volatile("" : "+v"(e));
    if (e >= PLANE) return;
    const int rr = e / RL, o = e - rr * RL;
    const int gi = i0 - 1 + o / 3, gj = j0 - 1 + rr;
    double pn = 0.;
    if (o < len && rr < rows && gi >= 0 && gi < g.nx && gj >= 0 && gj < g.ny && p >= 0 && p < g.nz) {
      const int d = o - 3 * (o / 3);
      // z = D^-1 r (k_cg_pupdate's z_of<DIX>); s_jdd holds the dictionary's entries only, so FP
      // requires a matrix without exception nodes (jix 255 would redirect): fusep() checks vi_nexc
      const double z = f.rv * s_jdd[3 * f.jx + d];
      pn = cgi == 0 ? z : z + cb * f.po;
      if (gi >= i0 && gi < i0 + TX && gj >= j0 && gj < j0 + TY && p >= k0 && p < k1)
        pdst[3 * (int64_t)(i0 + (j0 + rr) * PX + (p + 1) * PXY) + o] = pn;
    }
    xs[slot][e] = pn;
  };
  for (int t = me; t < VI_MAX * VIB_STRIDE / 2; t += T) tab[t] = reinterpret_cast<const double2*>(bdict)[t];
  if (FP) {
    for (int t = me; t < 3 * VI_MAX; t += T) s_jdd[t] = fp.jdd[t];
    __syncthreads();
#pragma unroll
    for (int s = 0; s < 3; s++) {  // prologue: planes k0-1, k0, k0+1 in ring slots 0, 1, 2
      Fe fe[NL];
#pragma unroll
      for (int m = 0; m < NL; m++) fload(k0 - 1 + s, m, fe[m]);
#pragma unroll
      for (int m = 0; m < NL; m++) fstore(s, k0 - 1 + s, m, fe[m]);
    }
  } else {
#pragma unroll
    for (int s = 0; s < 3; s++)  // prologue: planes k0-1, k0, k0+1 in ring slots 0, 1, 2
#pragma unroll
      for (int m = 0; m < NL; m++) xstore(s, m, xload(k0 - 1 + s, m));
  }
  // EXC: this wave's list entries so far (wave-uniform) and its segment's capacity
  const int wcap = EXC ? min(SEG, (min(XL, zt.xlist) + NW - 1) / NW) : 0;
  int wn = 0;
  u32x4 c0 = {0u, 0u, 0u, 0u}, c1 = c0, n0 = c0, n1 = c0;
  // WD: descriptors of planes k and k+1 (dc, dn); a plane's per-lane index words are loaded only
  // where its descriptor says the wave is not uniform
  unsigned dc = 0u, dn = 0u;
  auto wflag = [&](unsigned d) -> unsigned { return (unsigned)__builtin_amdgcn_readlane((int)d, 0); };
  if (WD) {
    dc = dload(k0);
    dn = dload(k0 + 1);
    if (!wdv || !wskip(wflag(dc))) iload(k0, c0, c1);
  } else {
    iload(k0, c0, c1);
  }
  __syncthreads();
  double dot = 0.;
  for (int k = k0; k < k1; k++) {
    const bool more = k + 1 < k1;
    double xr[FP ? 1 : NL];
    Fe fe[FP ? NL : 1];
    unsigned dn2 = 0u;
    if (more) {  // in flight during this plane: x (p) of plane k+2, indices of plane k+1
      if (FP) {
#pragma unroll
        for (int m = 0; m < NL; m++) fload(k + 2, m, fe[m]);
      } else {
#pragma unroll
        for (int m = 0; m < NL; m++) xr[m] = xload(k + 2, m);
      }
      if (WD) {
        dn2 = dload(k + 2);
        if (!wdv || !wskip(wflag(dn))) iload(k + 1, n0, n1);  // (uniform)
      } else {
        iload(k + 1, n0, n1);
      }
    }
    // UNI: a wave whose 64 nodes have the same 27 block indices (interior x-lines: no domain
    // boundary, no Dirichlet neighbour) reads the block values with scalar loads (s_load from
    // the dictionary in global memory, scalar cache) and multiplies them as SGPR operands: the
    // dictionary's 486 LDS cycles per wave and plane leave the LDS, which then only serves the x
    // ring.  Other waves read the dictionary from LDS.  Same values, same products, same order.
    // exact rows (!FMA): a node on the global domain boundary has clipped stencil columns, so its
    // inode pairing depends on which neighbours exist; those rows are computed by k_spmv_vib_faces
    // after the march, and every row here has all 27 neighbours: the pairing is fixed at compile
    // time (InodeRows<true>) on every path
    const bool full = FMA || present_mask(g, i, j, k) == PRES_ALL;
    unsigned sw[7] = {0u, 0u, 0u, 0u, 0u, 0u, 0u}, sb[7] = {0u, 0u, 0u, 0u, 0u, 0u, 0u};
    bool uni = false, two = false;
    unsigned long long mb = 0ull;
    if (WD) {
      // the descriptor: bit 0 = the 64 lanes are in the domain with the same 27 block indices
      // (words 1-7), bit 1 = every lane has all 27 neighbours (exact rows need it), bit 2 = the
      // lanes hold two index sets, the first lane's (words 1-7) and set B (words 8-14) on the
      // lanes of mask words 16-17
      const unsigned f = wdv ? wflag(dc) : 0u;
#pragma unroll
      for (int q = 0; q < 7; q++) sw[q] = (unsigned)__builtin_amdgcn_readlane((int)dc, q + 1);
      uni = (FMA ? (f & 1u) != 0u : (f & 3u) == 3u) || (zt.dbg & 1);
      two = !uni && FMA && zt.wdm == 2 && (f & 4u);
      if (two) {
#pragma unroll
        for (int q = 0; q < 7; q++) sb[q] = (unsigned)__builtin_amdgcn_readlane((int)dc, q + 8);
        mb = (unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)dc, 16) |
             ((unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)dc, 17) << 32);
      }
    } else if (UNI) {
#pragma unroll
      for (int q = 0; q < 7; q++) sw[q] = __builtin_amdgcn_readfirstlane(q < 4 ? c0[q] : c1[q - 4]);
      unsigned diff = 0u;
#pragma unroll
      for (int q = 0; q < 7; q++) diff |= (q < 4 ? c0[q] : c1[q - 4]) ^ sw[q];
      uni = __all(inxy && full && diff == 0u && (!EXC || c1[3] == 0u)) || (zt.dbg & 1);
    }
    // EXC: the wave's exception lanes of this plane take the next positions of its segment in
    // lane order (ballot + mbcnt, converged here); those beyond the capacity stay in the plane
    bool deferred = false;
    if constexpr (EXC) {
      const bool xh = !(UNI && uni) && inxy && full && c1[3] != 0u;
      const unsigned long long xm = zt.xskip ? 0ull : __ballot(xh);
      deferred = zt.xskip && xh;  // (xskip: k_spmv_exc computes the row)
      if (xm) {  // uniform
        const int pos = wn + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(xm >> 32),
                                                              __builtin_amdgcn_mbcnt_lo((unsigned)xm, 0u));
        deferred = xh && pos < wcap;
        if (deferred) s_xl[wv * SEG + pos] = (k - k0) * T + me;
        wn = min(wcap, wn + (int)__popcll(xm));
      }
    }
    if (UNI && (uni || two)) {  // (every lane is inxy)
      double y0 = 0., y1 = 0., y2 = 0., xc0 = 0., xc1 = 0., xc2 = 0.;
      InodeRows<true> acc;  // !FMA: the inode pairs of a node whose 27 neighbours are present
      typedef const volatile __attribute__((address_space(3))) double lds_vdouble;
      lds_vdouble* xsv = (lds_vdouble*)&xs[0][0];
      // blocks in groups of 3 (one dy row of the stencil): the 3 blocks' scalar loads are issued
      // together and waited for once (an SMEM result can only be waited for with lgkmcnt(0), so
      // a load issued ahead of the block in use would be waited for with it)
      // (FP: one block per group, its SGPRs being needed for the fused p update's scalars)
      constexpr int GB = FP ? 1 : 3;
      // two-set waves (WD): the pass below runs once per set, each lane in its own set's pass
      // (exec mask), so every row still gets its 27 terms in nb order
      auto pass = [&](const unsigned (&sw)[7]) {
#pragma unroll
      for (int nb0 = 0; nb0 < 27; nb0 += GB) {
        double av[GB][9], xv[GB][3];
#pragma unroll
        for (int t = 0; t < GB; t++) {
          const int nb = nb0 + t;
          const int dx = nb % 3 - 1, dy = (nb / 3) % 3 - 1, dz = nb / 9 - 1;
          const int xo = ((k + dz - k0 + 1) % R) * PLANE + (ly + 1 + dy) * RL + 3 * (lx + 1 + dx);
          lds_vdouble* xp = xsv + xo;
          xv[t][0] = xp[0];
          xv[t][1] = xp[1];
          xv[t][2] = xp[2];
          // wave-uniform (readfirstlane: without it the compiler took set B's run for divergent)
          const unsigned id = __builtin_amdgcn_readfirstlane((sw[nb >> 2] >> (8 * (nb & 3))) & 255u);
          const double* e = bdict + id * VIB_STRIDE;  // values 0-7: one s_load_dwordx16
#pragma unroll
          for (int q = 0; q < 8; q++) av[t][q] = e[q];
          // value 8 from the LDS copy (one broadcast ds_read_b64, 2 LDS cycles): an s_load_dwordx2
          // per block needs an SGPR pair of its own, and the compiler reused one pair for every
          // block, so each block's loads waited for the previous block's
          av[t][8] = reinterpret_cast<const double*>(tab + id * (VIB_STRIDE / 2))[8];
        }
        // the group's loads first, then its products: one lgkmcnt(0) wait per group, while the
        // SIMD's other waves compute (the scheduler would otherwise issue the next group's loads
        // among these products, and the wait for one value would wait for those too)
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int t = 0; t < GB; t++) {
          if (nb0 + t == 13) {
            xc0 = xv[t][0];
            xc1 = xv[t][1];
            xc2 = xv[t][2];
          }
#pragma unroll
          for (int q = 0; q < 9; q++) {
            const int r = q / 3, cc = q % 3;
            double& yr = r == 0 ? y0 : (r == 1 ? y1 : y2);
            if constexpr (FMA) yr = __builtin_fma(av[t][q], xv[t][cc], yr);
            else acc.term(nb0 + t, r, cc, av[t][q] * xv[t][cc]);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      };
      pass(sw);
      if (WD && two) {  // (uniform) set B's run on every lane; the lanes of set A keep their first run's rows
        // (FMA rows start from 0 in each run; a loop over the sets, or a branch on the lane's set,
        // made the compiler turn the dictionary's scalar loads into vector loads)
        const double a0 = y0, a1 = y1, a2 = y2, ax0 = xc0, ax1 = xc1, ax2 = xc2;
        y0 = y1 = y2 = 0.;
        pass(sb);
        if (!((mb >> ln) & 1ull)) {
          y0 = a0, y1 = a1, y2 = a2;
          xc0 = ax0, xc1 = ax1, xc2 = ax2;
        }
      }
      if constexpr (!FMA) y0 = acc.row(0), y1 = acc.row(1), y2 = acc.row(2);
      const int64_t n = i + g.nx * (j + (int64_t)g.ny * k);
      if (zt.ypair) {
        // y of a lane pair (even lane = even node, its odd neighbour in x on the next lane: 48
        // contiguous, 16-B aligned bytes) as three 16-B stores instead of six 8-B ones: the even
        // lane (y0, y1) and (y2, the odd lane's y0), the odd lane (y1, y2); the odd lane's y0
        // moves over by a DPP row shift (ypair needs an even nx and every lane of the wave here)
        const unsigned long long b0 = __double_as_longlong(y0);
        const unsigned lo = __builtin_amdgcn_mov_dpp((int)(unsigned)b0, 0x101, 0xf, 0xf, false);        // row_shl:1
        const unsigned hi = __builtin_amdgcn_mov_dpp((int)(unsigned)(b0 >> 32), 0x101, 0xf, 0xf, false);
        const double n0 = __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
        typedef double d2v __attribute__((ext_vector_type(2)));
        const bool even = (ln & 1) == 0;
        d2v a, b;
        a.x = even ? y0 : y1;
        a.y = even ? y1 : y2;
        __builtin_nontemporal_store(a, reinterpret_cast<d2v*>(&y[3 * n + (even ? 0 : 1)]));
        if (even) {
          b.x = y2;
          b.y = n0;
          __builtin_nontemporal_store(b, reinterpret_cast<d2v*>(&y[3 * n + 2]));
        }
      } else {
        __builtin_nontemporal_store(y0, &y[3 * n + 0]);
        __builtin_nontemporal_store(y1, &y[3 * n + 1]);
        __builtin_nontemporal_store(y2, &y[3 * n + 2]);
      }
      if (DOT) dot += xc0 * y0 + xc1 * y1 + xc2 * y2;
    } else if (EXC && deferred) {
      // deferred to the block's exception pass below
    } else if (EXC && inxy && full && c1[3]) {
      // an exception node (EXC instantiations only) that found the tile's list full: its 27
      // plain blocks from exc [slot][27][9], a rolled loop of its own so the indexed path below
      // keeps its registers; same order and products as the indexed rows
      // Blocks in groups of 3 (one dy row): the group's 27 values are loaded together, one
      // round trip per group instead of per block.
      double y0 = 0., y1 = 0., y2 = 0., xc0 = 0., xc1 = 0., xc2 = 0.;
      InodeRows<true> acc;  // !FMA: all 27 neighbours present (full)
      const double* eb = exc + exc_base(c1[3] - 1);  // value v at eb[v * 64]
#pragma unroll 1
      for (int nb0 = 0; nb0 < 27; nb0 += 3) {
        double av[27];
#pragma unroll
        for (int q = 0; q < 27; q++) av[q] = eb[(nb0 * 9 + q) * 64];
        const int dy = (nb0 / 3) % 3 - 1, dz = nb0 / 9 - 1;
        const int xo = ((k + dz - k0 + 1) % R) * PLANE + (ly + 1 + dy) * RL + 3 * lx;
#pragma unroll
        for (int t = 0; t < 3; t++) {
          const double xv[3] = {xs[0][xo + 3 * t], xs[0][xo + 3 * t + 1], xs[0][xo + 3 * t + 2]};
          if (nb0 + t == 13) {
            xc0 = xv[0];
            xc1 = xv[1];
            xc2 = xv[2];
          }
#pragma unroll
          for (int q = 0; q < 9; q++) {
            const int r = q / 3, cc = q % 3;
            double& yr = r == 0 ? y0 : (r == 1 ? y1 : y2);
            if constexpr (FMA) yr = __builtin_fma(av[t * 9 + q], xv[cc], yr);
            else acc.term(nb0 + t, r, cc, av[t * 9 + q] * xv[cc]);
          }
        }
      }
      if constexpr (!FMA) y0 = acc.row(0), y1 = acc.row(1), y2 = acc.row(2);
      const int64_t n = i + g.nx * (j + (int64_t)g.ny * k);
      __builtin_nontemporal_store(y0, &y[3 * n + 0]);
      __builtin_nontemporal_store(y1, &y[3 * n + 1]);
      __builtin_nontemporal_store(y2, &y[3 * n + 2]);
      if (DOT) dot += xc0 * y0 + xc1 * y1 + xc2 * y2;
    } else if (inxy && full) {
      double y0 = 0., y1 = 0., y2 = 0., xc0 = 0., xc1 = 0., xc2 = 0.;
      InodeRows<true> acc;  // !FMA: all 27 neighbours present (full)
      // x as separate 8-B LDS reads (ds_read_b64: 2 LDS cycles each): the compiler would pair
      // them into ds_read2_b64, 8 cycles for the same 16 B (MI355X_MICROARCH.md, LDS table);
      // volatile reads are not paired.
      typedef const volatile __attribute__((address_space(3))) double lds_vdouble;
      lds_vdouble* xsv = (lds_vdouble*)&xs[0][0];
      // LG > 1 (option vi_lg): the reads of LG blocks issued together and waited for once (the
      // compiler otherwise waits for each block's reads before its products: 27 LDS round trips
      // per wave and plane on these waves, which set the plane's pace at its barrier)
#pragma unroll
      for (int nb0 = 0; nb0 < 27; nb0 += LG) {
        double xv[LG][3], a[LG][9];
#pragma unroll
        for (int t = 0; t < LG; t++) {
          const int nb = nb0 + t;
          if (nb >= 27) break;
          const int dx = nb % 3 - 1, dy = (nb / 3) % 3 - 1, dz = nb / 9 - 1;
          const int xo = ((k + dz - k0 + 1) % R) * PLANE + (ly + 1 + dy) * RL + 3 * (lx + 1 + dx);
          if (XV) {
            lds_vdouble* xp = xsv + xo;
            xv[t][0] = xp[0];
            xv[t][1] = xp[1];
            xv[t][2] = xp[2];
          } else {
            const double* xp = &xs[0][0] + xo;
            xv[t][0] = xp[0];
            xv[t][1] = xp[1];
            xv[t][2] = xp[2];
          }
          const unsigned word = nb < 16 ? c0[nb >> 2] : c1[(nb - 16) >> 2];
          const unsigned id = (word >> (8 * (nb & 3))) & 255u;
          const double2* e = tab + id * (VIB_STRIDE / 2);
          const double2 a01 = e[0], a23 = e[1], a45 = e[2], a67 = e[3];
          const double a8 = reinterpret_cast<const double*>(e)[8];  // 8 B, not the padded 16: 18 LDS cycles per block
          a[t][0] = a01.x, a[t][1] = a01.y, a[t][2] = a23.x, a[t][3] = a23.y, a[t][4] = a45.x;
          a[t][5] = a45.y, a[t][6] = a67.x, a[t][7] = a67.y, a[t][8] = a8;
        }
        if (LG > 1) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int t = 0; t < LG; t++) {
          const int nb = nb0 + t;
          if (nb >= 27) break;
          if (nb == 13) {
            xc0 = xv[t][0];
            xc1 = xv[t][1];
            xc2 = xv[t][2];
          }
#pragma unroll
          for (int q = 0; q < 9; q++) {
            const int r = q / 3, cc = q % 3;
            double& yr = r == 0 ? y0 : (r == 1 ? y1 : y2);
            if constexpr (FMA) yr = __builtin_fma(a[t][q], xv[t][cc], yr);
            else acc.term(nb, r, cc, a[t][q] * xv[t][cc]);
          }
        }
        if (LG > 1) __builtin_amdgcn_sched_barrier(0);
      }
      if constexpr (!FMA) y0 = acc.row(0), y1 = acc.row(1), y2 = acc.row(2);
      const int64_t n = i + g.nx * (j + (int64_t)g.ny * k);
      __builtin_nontemporal_store(y0, &y[3 * n + 0]);
      __builtin_nontemporal_store(y1, &y[3 * n + 1]);
      __builtin_nontemporal_store(y2, &y[3 * n + 2]);
      if (DOT) dot += xc0 * y0 + xc1 * y1 + xc2 * y2;
    }
    if (more) {  // uniform
      if (R == 3) __syncthreads();  // plane k-1's slot is free
      if (FP) {
#pragma unroll
        for (int m = 0; m < NL; m++) fstore((k + 2 - k0 + 1) % R, k + 2, m, fe[m]);
      } else {
#pragma unroll
        for (int m = 0; m < NL; m++) xstore((k + 2 - k0 + 1) % R, m, xr[m]);
      }
      c0 = n0;
      c1 = n1;
      if (WD) {
        dc = dn;
        dn = dn2;
      }
      __syncthreads();
    }
  }
  if (EXC && !zt.xskip) {
    // the exception pass: one listed node per thread, x gathered from the padded vector (the
    // values the ring held), rows in the indexed path's order and products: y bit-identical.
    // Only the block's dot partial adds these nodes' terms in another order.
    if (ln == 0) s_wn[wv] = wn;
    __syncthreads();
    int ne = 0;
#pragma unroll
    for (int w = 0; w < NW; w++) ne += s_wn[w];
    for (int t = me; t < ne; t += T) {
      int w = 0, o = t;  // entry t of the segments in wave order
      while (o >= s_wn[w]) o -= s_wn[w++];
      const int code = s_xl[w * SEG + o];
      const int kk = k0 + code / T;
      int ex, ey;
      lane_xy(code % T, ex, ey);
      const int ei = i0 + ex, ej = j0 + ey;
      const int64_t n = ei + g.nx * (ej + (int64_t)g.ny * kk);
      const unsigned slot = I[(int64_t)(n >> 6) * (2 * 64) + (n & 63) + 64][3];
      const double* eb = exc + exc_base(slot - 1);  // value v at eb[v * 64]
      double y0 = 0., y1 = 0., y2 = 0., xc0 = 0., xc1 = 0., xc2 = 0.;
      InodeRows<true> acc;  // !FMA: listed nodes are full (boundary nodes go to k_spmv_vib_faces)
#pragma unroll 1
      for (int nb0 = 0; nb0 < 27; nb0 += 3) {
        double av[27];
#pragma unroll
        for (int q = 0; q < 27; q++) av[q] = eb[(nb0 * 9 + q) * 64];
        const int dy = (nb0 / 3) % 3 - 1, dz = nb0 / 9 - 1;
        const double* xr = x + 3 * ((int64_t)ei + (ej + 1 + dy) * (int64_t)PX + (kk + 1 + dz) * (int64_t)PXY);
        double xw[9];
#pragma unroll
        for (int q = 0; q < 9; q++) xw[q] = xr[q];  // nodes i-1, i, i+1 of the row (padded i = node i + 1)
#pragma unroll
        for (int t3 = 0; t3 < 3; t3++) {
          const double xv[3] = {xw[3 * t3], xw[3 * t3 + 1], xw[3 * t3 + 2]};
          if (nb0 + t3 == 13) {
            xc0 = xv[0];
            xc1 = xv[1];
            xc2 = xv[2];
          }
#pragma unroll
          for (int q = 0; q < 9; q++) {
            const int r = q / 3, cc = q % 3;
            double& yr = r == 0 ? y0 : (r == 1 ? y1 : y2);
            if constexpr (FMA) yr = __builtin_fma(av[t3 * 9 + q], xv[cc], yr);
            else acc.term(nb0 + t3, r, cc, av[t3 * 9 + q] * xv[cc]);
          }
        }
      }
      if constexpr (!FMA) y0 = acc.row(0), y1 = acc.row(1), y2 = acc.row(2);
      __builtin_nontemporal_store(y0, &y[3 * n + 0]);
      __builtin_nontemporal_store(y1, &y[3 * n + 1]);
      __builtin_nontemporal_store(y2, &y[3 * n + 2]);
      if (DOT) dot += xc0 * y0 + xc1 * y1 + xc2 * y2;
    }
  }
  if (DOT) {
    double s = block_sum<T>(dot, sh);
    if (threadIdx.x == 0) part[blockIdx.x] = s;
  }
}

// ---------------------------------------------------------------------------- default-stencil SpMV
// buffer resource over `bytes` from `base` (a raw buffer: out-of-range loads return 0, out-of-range
// stores are dropped; at most 2 GB, the offsets used are 32-bit)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t sp_rsrc(const double* base, int64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(base), (short)0,
                                           (int)(bytes > 0x7fffffffLL ? 0x7fffffff : bytes), 0x00020000);
}
constexpr unsigned SP_OOB = 0x80000000u;  // a buffer offset past every record: load 0 / store dropped

// Round 5 (vi_st).  On the block-indexed storage almost every node carries the same 27 block
// indices: the interior stencil of the uniform grid (at 256^3 all but the 2.3 % of nodes on the
// domain faces, next to Dirichlet nodes, or exception nodes).  The matrix is then held as
//   * the stencil classes (k_st_setup): the interior and the 6 domain faces, 27 blocks each
//     (st_coef, rows of VIB_STRIDE doubles, read with scalar loads),
//   * a 64-bit mask per 16 x 4 node patch and plane: the lanes the march leaves (face nodes,
//     listed nodes, outside the domain),
//   * the list of the other nodes (ordered compaction, owned-node order: edges, neighbours of
//     Dirichlet nodes, exception nodes, nodes unlike their class), whose rows come from their own
//     index bytes / exception blocks exactly as before.
// k_spmv_st marches a 64 x 16 tile up its z-chunk two planes per step (nodes k and k+1 per lane):
// each group of 3 blocks (one (dy, dz) stencil row) is loaded once for two nodes, so the scalar
// loads and their waits per node halve; the x ring in LDS holds planes k-1 .. k+2, and planes k+3,
// k+4 are loaded into registers during the step and stored after a barrier.  The default path
// reads no index bytes.  Rows are the FMA rows of k_spmv_vibm (one fused multiply-add per term in
// (nb, c) order), so y is bitwise what k_spmv_vibm computes; a face node's row is computed by
// k_spmv_face from its class stencil, a listed node's from its index bytes or exception blocks, x
// gathered, in the same order.  p.w partials: the march's blocks, then k_spmv_face's.
// k_spmv_st TAIL: this block's share of the listed (non-default) rows, in list order, the
// dictionary staged in tab (the freed ring); x gathered, one stencil row (9 x, 3 blocks) per
// round; the FMA rows of k_spmv_vibm (an exception node's blocks from exc)
template <int T>
__device__ __forceinline__ void st_tail(const Geo& g, const int* __restrict__ list, int64_t lo, int64_t hi,
                                        const u32x4* __restrict__ I, const double* __restrict__ bdict,
                                        const double* __restrict__ exc, const double* __restrict__ x,
                                        double* __restrict__ y, double2* tabg, double& dot, int nd = VI_MAX) {
  typedef __attribute__((address_space(3))) double lds_double;
  lds_double* tab = (lds_double*)tabg;  // (the ring's LDS: ds_read, not flat loads)
  const int me = threadIdx.x;
  if (lo >= hi) return;  // (uniform) no share: no dictionary staging
  const int ndv = min(nd, VI_MAX) * VIB_STRIDE;  // staged dictionary doubles (the blocks in use)
  // the first node's list entry and index words are loaded before the dictionary staging and its
  // barrier (which waits for LDS only), so their round trips overlap the staging's
  int n = 0;
  u32x4 w0 = {0u, 0u, 0u, 0u}, w1 = {0u, 0u, 0u, 0u};
  auto fetch = [&](int64_t t) {
    if (t < hi) {
      n = list[t];
      const u32x4* ip = I + (int64_t)(n >> 6) * (2 * 64) + (n & 63);
      w0 = ip[0];
      w1 = ip[64];
    }
  };
  fetch(lo + me);
  {
    constexpr int ND = (VI_MAX * VIB_STRIDE + T - 1) / T;
    double dv[ND];  // all the staging loads in flight before the LDS stores
#pragma unroll
    for (int m = 0; m < ND; m++) dv[m] = me + m * T < ndv ? bdict[me + m * T] : 0.;
#pragma unroll
    for (int m = 0; m < ND; m++)
      if (me + m * T < ndv) tab[me + m * T] = dv[m];
  }
  __syncthreads();
  const int PX = g.PX, PXY = g.PX * g.PY;
  for (int64_t t = lo + me; t < hi; t += T) {
    if (t != lo + me) fetch(t);
    int i, j, k;
    node_ijk(g, n, i, j, k);
    const unsigned slot = w1[3];  // exception slot + 1
    const double* eb = exc + exc_base(slot ? slot - 1 : 0);
    double y0 = 0., y1 = 0., y2 = 0., xc0 = 0., xc1 = 0., xc2 = 0.;
    // a rolled loop over the stencil rows (unrolled, the compiler hoisted the rows' loads and spilled)
#pragma unroll 1
    for (int g9 = 0; g9 < 9; g9++) {
      const int dy = g9 % 3 - 1, dz = g9 / 3 - 1;
      const double* xr = x + 3 * ((int64_t)i + (j + 1 + dy) * (int64_t)PX + (k + 1 + dz) * (int64_t)PXY);
      double xw[9], av[27];
#pragma unroll
      for (int q = 0; q < 9; q++) xw[q] = xr[q];
#pragma unroll
      for (int t3 = 0; t3 < 3; t3++) {
        const int nb = g9 * 3 + t3;
        if (slot) {
#pragma unroll
          for (int q = 0; q < 9; q++) av[t3 * 9 + q] = eb[(nb * 9 + q) * 64];
        } else {
          const int wi = nb >> 2;  // (run-time, uniform): a select chain, not a private array
          const unsigned word = wi == 0 ? w0[0] : wi == 1 ? w0[1] : wi == 2 ? w0[2] : wi == 3 ? w0[3]
                              : wi == 4 ? w1[0] : wi == 5 ? w1[1] : w1[2];
          const lds_double* e = tab + ((word >> (8 * (nb & 3))) & 255u) * VIB_STRIDE;
#pragma unroll
          for (int q = 0; q < 9; q++) av[t3 * 9 + q] = e[q];
        }
      }
      if (g9 == 4) xc0 = xw[3], xc1 = xw[4], xc2 = xw[5];
#pragma unroll
      for (int t3 = 0; t3 < 3; t3++)
#pragma unroll
        for (int q = 0; q < 9; q++) {
          const int r = q / 3, cc = q % 3;
          double& yr = r == 0 ? y0 : (r == 1 ? y1 : y2);
          yr = __builtin_fma(av[t3 * 9 + q], xw[3 * t3 + cc], yr);
        }
    }
    __builtin_nontemporal_store(y0, &y[3 * (int64_t)n + 0]);
    __builtin_nontemporal_store(y1, &y[3 * (int64_t)n + 1]);
    __builtin_nontemporal_store(y2, &y[3 * (int64_t)n + 2]);
    dot += xc0 * y0 + xc1 * y1 + xc2 * y2;
  }
}

// The listed rows with their loads in parallel (round 6): 16 lanes per
// listed node, lane g9 = 0..8 holding stencil row g9 -- its 9 x values and its 3 blocks (exception
// blocks from exc, else the dictionary staged in tab) -- all loaded at once, one memory round trip
// instead of st_tail's nine dependent ones per node.  The row's three accumulators then pass lane
// to lane (a 16-lane DPP row shift per round), lane g9 applying its 27 fused multiply-adds in round
// g9: per output row the same FMAs in the same (nb, c) order as st_tail / k_spmv_vibm, so y is
// bitwise theirs.  Lane 8 stores the row and its p.w term (the node's own x from lane 4).
constexpr int ST16 = 16;  // lanes per listed node
__device__ __forceinline__ double dpp_shr1(double v) {  // lane l takes lane l-1's value within its 16-lane row
  const unsigned lo = __builtin_amdgcn_update_dpp(0, (int)__double2loint(v), 0x111, 0xf, 0xf, false);
  const unsigned hi = __builtin_amdgcn_update_dpp(0, (int)__double2hiint(v), 0x111, 0xf, 0xf, false);
  return __hiloint2double((int)hi, (int)lo);
}
template <int T>
__device__ __forceinline__ void st_tail16(const Geo& g, const int* __restrict__ list, int64_t lo, int64_t hi,
                                          const u32x4* __restrict__ I, const double* __restrict__ bdict,
                                          const double* __restrict__ exc, const double* __restrict__ x,
                                          double* __restrict__ y, double2* tabg, double& dot, int nd = VI_MAX) {
  typedef __attribute__((address_space(3))) double lds_double;
  lds_double* tab = (lds_double*)tabg;
  const int me = threadIdx.x;
  if (lo >= hi) return;  // (uniform)
  const int PX = g.PX, PXY = g.PX * g.PY;
  const int g9 = me & (ST16 - 1);
  const int ndv = min(nd, VI_MAX) * VIB_STRIDE;  // staged dictionary doubles (the blocks in use)
  // a pass's global loads (list entry, x row, index words): the first pass's are issued before the
  // dictionary staging and its barrier, so the two round trips overlap (k_spmv_face gives a block
  // one pass; the barrier waits for LDS only, the loads stay in flight)
  int64_t n = 0;
  double xw[9];
  u32x4 w0 = {0u, 0u, 0u, 0u}, w1 = {0u, 0u, 0u, 0u};
  auto fetch = [&](int64_t t0) {
    const int64_t t = t0 + me / ST16;
    n = 0;
#pragma unroll
    for (int q = 0; q < 9; q++) xw[q] = 0.;
    w0 = w1 = u32x4{0u, 0u, 0u, 0u};
    if (t < hi && g9 < 9) {
      n = list[t];
      int i, j, k;
      node_ijk(g, (int)n, i, j, k);
      const int dy = g9 % 3 - 1, dz = g9 / 3 - 1;
      const double* xr = x + 3 * ((int64_t)i + (j + 1 + dy) * (int64_t)PX + (k + 1 + dz) * (int64_t)PXY);
#pragma unroll
      for (int q = 0; q < 9; q++) xw[q] = xr[q];
      const u32x4* ip = I + (n >> 6) * (2 * 64) + (n & 63);
      w0 = ip[0];
      w1 = ip[64];
    }
  };
  fetch(lo);
  {
    constexpr int ND = (VI_MAX * VIB_STRIDE + T - 1) / T;
    double dv[ND];  // all the staging loads in flight before the LDS stores
#pragma unroll
    for (int m = 0; m < ND; m++) dv[m] = me + m * T < ndv ? bdict[me + m * T] : 0.;
#pragma unroll
    for (int m = 0; m < ND; m++)
      if (me + m * T < ndv) tab[me + m * T] = dv[m];
  }
  __syncthreads();
  for (int64_t t0 = lo; t0 < hi; t0 += T / ST16) {  // (uniform)
    if (t0 != lo) fetch(t0);
    const int64_t t = t0 + me / ST16;
    const bool has = t < hi;
    const bool row = has && g9 < 9;
    double av[27];
#pragma unroll
    for (int q = 0; q < 27; q++) av[q] = 0.;
    if (row) {
      const unsigned slot = w1[3];  // exception slot + 1
      const double* eb = exc + exc_base(slot ? slot - 1 : 0);
#pragma unroll
      for (int t3 = 0; t3 < 3; t3++) {
        const int nb = g9 * 3 + t3;
        if (slot) {
#pragma unroll
          for (int q = 0; q < 9; q++) av[t3 * 9 + q] = eb[(nb * 9 + q) * 64];
        } else {
          const int wi = nb >> 2;
          const unsigned word = wi == 0 ? w0[0] : wi == 1 ? w0[1] : wi == 2 ? w0[2] : wi == 3 ? w0[3]
                              : wi == 4 ? w1[0] : wi == 5 ? w1[1] : w1[2];
          const lds_double* e = tab + ((word >> (8 * (nb & 3))) & 255u) * VIB_STRIDE;
#pragma unroll
          for (int q = 0; q < 9; q++) av[t3 * 9 + q] = e[q];
        }
      }
    }
    double y0 = 0., y1 = 0., y2 = 0.;
#pragma unroll
    for (int rnd = 0; rnd < 9; rnd++) {
      if (g9 == rnd) {
#pragma unroll
        for (int t3 = 0; t3 < 3; t3++)
#pragma unroll
          for (int q = 0; q < 9; q++) {
            const int r = q / 3, cc = q % 3;
            double& yr = r == 0 ? y0 : (r == 1 ? y1 : y2);
            yr = __builtin_fma(av[t3 * 9 + q], xw[3 * t3 + cc], yr);
          }
      }
      if (rnd < 8) {  // lane rnd's sums to lane rnd + 1
        y0 = dpp_shr1(y0);
        y1 = dpp_shr1(y1);
        y2 = dpp_shr1(y2);
      }
    }
    // lane 8: the row; the node's own x (block 13) from lane 4 (xw[3..5]), 4 lanes up
    const double xc0 = __shfl(xw[3], (me & ~(ST16 - 1)) + 4, 64), xc1 = __shfl(xw[4], (me & ~(ST16 - 1)) + 4, 64),
                 xc2 = __shfl(xw[5], (me & ~(ST16 - 1)) + 4, 64);
    if (row && g9 == 8) {
      __builtin_nontemporal_store(y0, &y[3 * n + 0]);
      __builtin_nontemporal_store(y1, &y[3 * n + 1]);
      __builtin_nontemporal_store(y2, &y[3 * n + 2]);
      dot += xc0 * y0 + xc1 * y1 + xc2 * y2;
    }
  }
}

// The face phase: the domain faces' nodes of a usable stencil class (k_st_setup) in patches of 64
// nodes along the face's fast axis (x-faces: j; y- and z-faces: i) x 4 along its slow axis, 256
// threads each.  The patch's x is staged in LDS first (SFP_N doubles: 9-double chunks (i-1 .. i+1)
// of the 66 x 6 neighbour grid for an x-face, 198-double row segments (66 nodes) for y- and
// z-faces, loaded in address order -- an x-face node's rows are PX apart, so gathered per lane
// they cost a cache line each), then a thread's node takes the class's 27 blocks from the scalar
// cache (the patch's class is uniform) and its x from LDS in the FMA rows' order of k_spmv_vibm, so
// y is bitwise the same.  A face node that is listed (slot != 0: an edge node, next to a Dirichlet
// node, an exception node, or not its class's stencil) is left to the listed rows.
constexpr int SFP_S = 4;                     // patch rows along the slow axis (a wave each; 6: 42.8 vs 40.7 us, r05w)
constexpr int SFP_T = 64 * SFP_S;            // threads per patch
constexpr int SFP_N = 66 * (SFP_S + 2) * 9;  // staged doubles per patch (= (SFP_S+2) * 3 * 198)

struct SfPatch {  // patch p's class, axis, side and origin
  int c, ax, f0, s0;
  bool hi;
};

__device__ __forceinline__ SfPatch sf_patch(const Geo& g, const StFaces& sf, int64_t p) {
  SfPatch q;
  q.c = 1;
  while (q.c < 6 && p >= sf.u[q.c]) q.c++;
  q.ax = (q.c - 1) >> 1;
  q.hi = !(q.c & 1);
  const int fb = ((q.ax == 0 ? g.ny : g.nx) + 63) >> 6;
  const int64_t lp = p - sf.u[q.c - 1];
  q.s0 = (int)(lp / fb) * SFP_S;
  q.f0 = (int)(lp - (int64_t)(q.s0 / SFP_S) * fb) * 64;
  return q;
}

// stage patch q's x into S (t = 0 .. SFP_T-1: the patch's threads).  Branch-free buffer loads from
// the patch's origin (a position outside the neighbour grid, or the outward ghost the rows leave
// out, is the out-of-range offset: the load returns 0), the face axis's index arithmetic chosen once
// per patch (uniform), all loads in flight before the LDS stores
__device__ __forceinline__ void sf_stage(const Geo& g, const SfPatch& q, const double* __restrict__ x, double* S,
                                         int t) {
  const int PX = g.PX;
  const int64_t PXY = (int64_t)g.PX * g.PY;
  const int gh = q.hi ? 2 : 0;
  constexpr int NE = (SFP_N + SFP_T - 1) / SFP_T;
  // origin: padded node (i', j', k') of the staged grid's first element
  const int iface = q.hi ? g.nx - 1 : 0, jface = q.hi ? g.ny - 1 : 0, kface = q.hi ? g.nz - 1 : 0;
  int64_t o0;
  if (q.ax == 0) o0 = iface + (int64_t)q.f0 * PX + (int64_t)q.s0 * PXY;
  else if (q.ax == 1) o0 = q.f0 + (int64_t)jface * PX + (int64_t)q.s0 * PXY;
  else o0 = q.f0 + (int64_t)q.s0 * PX + (int64_t)kface * PXY;
  const __amdgpu_buffer_rsrc_t rx = sp_rsrc(x + 3 * o0, (PXY * g.PZ - o0) * 24);
  const int PX3 = 3 * PX, PXY3 = (int)(3 * PXY);
  unsigned off[NE];
  if (q.ax == 0) {  // 9-double chunks (i-1 .. i+1) of the (SFP_S+2) x 66 (k', j') grid
    const int jmax = g.ny + 1 - q.f0, kmax = g.nz + 1 - q.s0;  // last staged jj / kk inside the padded box
#pragma unroll
    for (int m = 0; m < NE; m++) {
      const int e = t + m * SFP_T, ch = e / 9, o = e - ch * 9, kk = ch / 66, jj = ch - kk * 66;
      const bool ok = e < SFP_N && jj <= jmax && kk <= kmax && o / 3 != gh;
      off[m] = ok ? 8u * (unsigned)(jj * PX3 + kk * PXY3 + o) : SP_OOB;
    }
  } else {  // 198-double segments: y-face (kk, dy) of (SFP_S+2) x 3, z-face (dz, jj) of 3 x (SFP_S+2)
    const int omax = 3 * (g.nx + 2 - q.f0);
    const int smax = (q.ax == 1 ? g.nz : g.ny) + 1 - q.s0;  // last staged slow-axis row inside the box
#pragma unroll
    for (int m = 0; m < NE; m++) {
      const int e = t + m * SFP_T, r = e / 198, o = e - r * 198;
      int nr, sr;  // the row's normal-axis position (0 .. 2) and slow-axis position (0 .. SFP_S+1)
      if (q.ax == 1) nr = r % 3, sr = r / 3;
      else sr = r % (SFP_S + 2), nr = r / (SFP_S + 2);
      const bool ok = e < SFP_N && o < omax && sr <= smax && nr != gh;
      const int ro = q.ax == 1 ? nr * PX3 + sr * PXY3 : sr * PX3 + nr * PXY3;
      off[m] = ok ? 8u * (unsigned)(ro + o) : SP_OOB;
    }
  }
  double v[NE];
#pragma unroll
  for (int m = 0; m < NE; m++) v[m] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rx, off[m], 0, 0));
#pragma unroll
  for (int m = 0; m < NE; m++)
    if (t + m * SFP_T < SFP_N) S[t + m * SFP_T] = v[m];
}

// the rows of patch q's nodes from S (after a barrier)
__device__ __forceinline__ void sf_rows(const Geo& g, const SfPatch& q, const double* __restrict__ coef,
                                        const unsigned* __restrict__ slot, const double* S, double* __restrict__ y,
                                        double& dot, int t) {
  typedef const __attribute__((address_space(3))) double lds_double;
  lds_double* Sl = (lds_double*)S;
  const int w = t >> 6, ln = t & 63;
  const int nfast = q.ax == 0 ? g.ny : g.nx, nslow = q.ax == 2 ? g.ny : g.nz;
  const int f = q.f0 + ln, sl = q.s0 + w;
  const int i = q.ax == 0 ? (q.hi ? g.nx - 1 : 0) : f;
  const int j = q.ax == 0 ? f : (q.ax == 1 ? (q.hi ? g.ny - 1 : 0) : sl);
  const int k = q.ax == 2 ? (q.hi ? g.nz - 1 : 0) : sl;
  const bool in = f < nfast && sl < nslow;
  const int64_t n = in ? i + g.nx * (j + (int64_t)g.ny * k) : 0;
  const bool live = in && slot[n] == 0u;
  const double* cf = coef + q.c * 27 * VIB_STRIDE;  // (uniform) the class's stencil
  double y0 = 0., y1 = 0., y2 = 0., xc0 = 0., xc1 = 0., xc2 = 0.;
  // The outward neighbours of a face node are the global boundary's ghosts (x = 0; their blocks are
  // zero blocks): their terms are left out (fma(a, 0, y) = y, and y, summed from +0, is never -0),
  // so y is bitwise the full row's with a third fewer LDS reads, scalar loads and FMAs.
  const int gh = q.hi ? 2 : 0;  // the ghost's position in the (dx | dy | dz) + 1 range of the face normal
  // a rolled loop over the stencil rows (unrolled, the compiler hoists the rows' scalar loads and spills)
#pragma unroll 1
  for (int g9 = 0; g9 < 9; g9++) {
    const int dy = g9 % 3 - 1, dz = g9 / 3 - 1;
    if ((q.ax == 1 && dy + 1 == gh) || (q.ax == 2 && dz + 1 == gh)) continue;  // (uniform) a ghost row
    const int base = q.ax == 0 ? ((w + 1 + dz) * 66 + (ln + 1 + dy)) * 9
                   : q.ax == 1 ? ((w + 1 + dz) * 3 + (dy + 1)) * 198 + 3 * ln
                               : ((dz + 1) * (SFP_S + 2) + (w + 1 + dy)) * 198 + 3 * ln;
    double xw[9], av[27];
#pragma unroll
    for (int t3 = 0; t3 < 3; t3++) {
      if (q.ax == 0 && t3 == gh) continue;  // (uniform) the ghost column
#pragma unroll
      for (int qq = 0; qq < 3; qq++) xw[3 * t3 + qq] = Sl[base + 3 * t3 + qq];
#pragma unroll
      for (int qq = 0; qq < 9; qq++) av[t3 * 9 + qq] = cf[(g9 * 3 + t3) * VIB_STRIDE + qq];
    }
    if (g9 == 4) xc0 = xw[3], xc1 = xw[4], xc2 = xw[5];
#pragma unroll
    for (int t3 = 0; t3 < 3; t3++) {
      if (q.ax == 0 && t3 == gh) continue;
#pragma unroll
      for (int qq = 0; qq < 9; qq++) {
        const int r = qq / 3, cc = qq % 3;
        double& yr = r == 0 ? y0 : (r == 1 ? y1 : y2);
        yr = __builtin_fma(av[t3 * 9 + qq], xw[3 * t3 + cc], yr);
      }
    }
  }
  if (live) {
    __builtin_nontemporal_store(y0, &y[3 * n + 0]);
    __builtin_nontemporal_store(y1, &y[3 * n + 1]);
    __builtin_nontemporal_store(y2, &y[3 * n + 2]);
    dot += xc0 * y0 + xc1 * y1 + xc2 * y2;
  }
}

// a 1024-thread block's share of the patches [b P / nb, (b+1) P / nb), 1024 / SFP_T at a time
// (SFP_T threads and SFP_N doubles of S each); every thread takes part in every barrier
__device__ __forceinline__ void st_faces(const Geo& g, const StFaces& sf, const double* __restrict__ coef,
                                         const unsigned* __restrict__ slot, const double* __restrict__ x,
                                         double* __restrict__ y, double& dot, double* S) {
  const int64_t P = sf.u[6], lo = (int64_t)blockIdx.x * P / gridDim.x, hi = (int64_t)(blockIdx.x + 1) * P / gridDim.x;
  constexpr int NPB = 1024 / SFP_T;
  const int q4 = threadIdx.x / SFP_T, t = threadIdx.x - q4 * SFP_T;
  for (int64_t p0 = lo; p0 < hi; p0 += NPB) {  // (uniform)
    const int64_t p = p0 + q4;
    const bool has = q4 < NPB && p < hi;
    SfPatch q{};
    if (has) {
      q = sf_patch(g, sf, p);
      sf_stage(g, q, x, S + q4 * SFP_N, t);
    }
    __syncthreads();
    if (has) sf_rows(g, q, coef, slot, S + q4 * SFP_N, y, dot, t);
    __syncthreads();
  }
}

// TAIL (option vi_st_tail, off): the face patches and the listed rows are computed by the same
// blocks after their march, each block a fixed share (idle blocks too), in the freed x ring.  The
// march is one resident round of blocks, so the tail adds its latency to every block: 0.326 vs
// 0.285 ms with k_spmv_face (profiles/r05p_*).  Same rows; the p.w terms go to the block's partial.
template <bool DOT, bool GATED, bool TAIL = false, bool PF2 = false, bool NOSTAGE = false>
__global__ __launch_bounds__(1024) void k_spmv_st(Geo g, const double* __restrict__ coef,
                                                  const unsigned long long* __restrict__ mask, int npx, int npy,
                                                  const double* __restrict__ x, double* __restrict__ y,
                                                  double* __restrict__ part, const CgState* __restrict__ cg,
                                                  ZTiling zt, const int* __restrict__ list = nullptr, int64_t cnt = 0,
                                                  const u32x4* __restrict__ I = nullptr,
                                                  const double* __restrict__ bdict = nullptr,
                                                  const double* __restrict__ exc = nullptr,
                                                  const unsigned* __restrict__ slot = nullptr, StFaces sf = {}) {
  constexpr int TX = 64, TY = 16, T = TX * TY, RL = vibm_rl<TX, true>(), PR = TY + 2, PLANE = PR * RL;
  constexpr int NL = (PLANE + T - 1) / T, R = 4;
  __shared__ double xs[R][PLANE];
  __shared__ double sh[T / 64];
  __shared__ double s9[27];  // value 8 of the default stencil's blocks
  if (GATED && cg->reason) return;
  const int b = blockIdx.x;
  const int xcd = b & 7, t8 = b >> 3;
  const int slab = (zt.nty + 7) >> 3;
  const int ty0 = xcd * slab;
  const int nty_here = min(slab, zt.nty - ty0);
  const int per = max(nty_here, 0) * zt.ntx * zt.nzc;
  const int me = threadIdx.x;
  double dot = 0.;
  if (t8 >= per) {  // whole block idle (uniform): the listed rows' share only (TAIL), the partial
    if (TAIL) {
      st_faces(g, sf, coef, slot, x, y, dot, &xs[0][0]);
      st_tail<T>(g, list, (int64_t)b * cnt / gridDim.x, (int64_t)(b + 1) * cnt / gridDim.x, I, bdict, exc, x, y,
                 reinterpret_cast<double2*>(&xs[0][0]), dot);
    }
    if (DOT) {
      const double s = block_sum<T>(dot, sh);
      if (threadIdx.x == 0) part[blockIdx.x] = s;
    }
    return;
  }
  const int txi = t8 % zt.ntx, r8 = t8 / zt.ntx;
  const int tyi = ty0 + r8 % nty_here, zc = r8 / nty_here;
  const int i0 = txi * TX, j0 = tyi * TY;
  const int k0 = zc * zt.kc, k1 = min(g.nz, k0 + zt.kc);
  const int wv = me >> 6, ln = me & 63;
  if (me < 27) s9[me] = coef[me * VIB_STRIDE + 8];
  const int px = wv & 3, py = wv >> 2;  // 16 x 4 patch of the tile (every wave does the same work)
  const int lx = px * 16 + (ln & 15), ly = py * 4 + (ln >> 4);
  const int i = i0 + lx, j = j0 + ly;
  const bool inxy = i < g.nx && j < g.ny;
  const int PX = g.PX, PXY = g.PX * g.PY;
  const int gpx = __builtin_amdgcn_readfirstlane((i0 >> 4) + px), gpy = __builtin_amdgcn_readfirstlane((j0 >> 2) + py);
  const bool wvin = gpx < npx && gpy < npy;  // (uniform) the patch has a mask
  const int len = 3 * min(TX + 2, g.nx + 2 - i0);
  const int rows = min(TY + 2, g.ny + 2 - j0);
  // x of padded plane p + 1 (p = -1 .. nz), staged element me + m T: a buffer load, 0 outside the box
  // (no branch: the compiler counts the loads, and the step's wait for them leaves the y stores in flight)
  auto xload = [&](int p, int m) -> double {
    const int e = me + m * T;
    const int rr = e / RL, o = e - rr * RL;
    const __amdgpu_buffer_rsrc_t rx = sp_rsrc(x + (int64_t)(p + 1) * PXY * 3, p > g.nz ? 0 : (int64_t)PXY * 24);
    const unsigned off = e >= PLANE || o >= len || rr >= rows ? SP_OOB : 8u * (unsigned)(3 * (i0 + (j0 + rr) * PX) + o);
    typedef unsigned u32x2v __attribute__((ext_vector_type(2)));
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rx, off, 0, 0));
  };
  // PF2 (option vi_st_pf 2): the planes a step stores into the ring were loaded one step earlier, so
  // each load has two steps of rows to land (xa: planes k+3, k+4 at step k)
  double pfa[2][NL], pfb[2][NL];
  {  // prologue: planes k0-1 .. k0+2 in ring slots 0 .. 3, every load issued before the first store
    double v[4][NL];
#pragma unroll
    for (int s = 0; s < 4; s++)
#pragma unroll
      for (int m = 0; m < NL; m++) v[s][m] = xload(k0 - 1 + s, m);
    if (PF2) {
#pragma unroll
      for (int m = 0; m < NL; m++) {
        pfa[0][m] = xload(k0 + 3, m);
        pfa[1][m] = xload(k0 + 4, m);
      }
    }
#pragma unroll
    for (int s = 0; s < 4; s++)
#pragma unroll
      for (int m = 0; m < NL; m++) {
        const int e = me + m * T;
        if (e < PLANE) xs[s][e] = v[s][m];
      }
  }
  __syncthreads();
  typedef const volatile __attribute__((address_space(3))) double lds_vdouble;
  lds_vdouble* xsv = (lds_vdouble*)&xs[0][0];
  // one two-plane step; PF2 alternates the two register sets between consecutive steps (no copies:
  // a copy of a register still being loaded waits for the load)
  auto step = [&](int k, double (&cur)[2][NL], double (&nxt)[2][NL]) {
    const bool two = k + 1 < k1, more = k + 2 < k1;
    // PF2: planes k+3, k+4 (cur) were loaded a step earlier; k+5, k+6 go in flight into nxt
    // (unconditional: a plane past the grid reads zeros, and the compiler keeps counting the loads)
    double xr[2][NL];
    if (PF2) {
#pragma unroll
      for (int m = 0; m < NL; m++) {
        nxt[0][m] = xload(k + 5, m);
        nxt[1][m] = xload(k + 6, m);
      }
    } else if (more) {  // planes k+3 and k+4, in flight during the step
#pragma unroll
      for (int m = 0; m < NL; m++) {
        xr[0][m] = xload(k + 3, m);
        xr[1][m] = xload(k + 4, m);
      }
    }
    unsigned long long m0 = ~0ull, m1 = ~0ull;  // lanes the march leaves (faces, listed rows)
    if (wvin) {
      m0 = mask[((int64_t)k * npy + gpy) * npx + gpx];
      if (two) m1 = mask[((int64_t)(k + 1) * npy + gpy) * npx + gpx];
    }
    double ya0 = 0., ya1 = 0., ya2 = 0., yb0 = 0., yb1 = 0., yb2 = 0.;
    double ca0 = 0., ca1 = 0., ca2 = 0., cb0 = 0., cb1 = 0., cb2 = 0.;
    // a rolled loop over the 9 stencil rows: unrolled, the compiler hoisted every group's scalar
    // loads to the top of the step (or out of the plane loop: 486 SGPRs) and spilled
#pragma unroll 1
    for (int g9 = 0; g9 < 9; g9++) {  // stencil row (dy, dz): blocks nb = 3 g9 .. 3 g9 + 2 (dx = -1, 0, 1)
      const int dy = g9 % 3 - 1, dz = g9 / 3 - 1;
      double av[27], xa[9], xb[9];
      // the group's 27 values from the scalar cache at every step: an opaque (uniform) zero in the
      // offset keeps the compiler from hoisting all 243 loop-invariant loads out of the plane loop
      // (486 SGPRs, spilled to VGPRs and scratch); an opaque pointer instead turned them into flat
      // vector loads
      // values 0-7 of each block by one s_load_dwordx16 (coef rows of VIB_STRIDE doubles: 16-B
      // aligned), value 8 from the LDS copy s9 (a broadcast ds_read_b64): 48 SGPRs per group, as
      // k_spmv_vibm's scalar path
#pragma unroll
      for (int t = 0; t < 3; t++) {
#pragma unroll
        for (int q = 0; q < 8; q++) av[t * 9 + q] = coef[(g9 * 3 + t) * VIB_STRIDE + q];
        av[t * 9 + 8] = s9[g9 * 3 + t];
      }
      const int ra = ((k + dz - k0 + 1) & 3) * PLANE + (ly + 1 + dy) * RL + 3 * lx;
      const int rb = ((k + 1 + dz - k0 + 1) & 3) * PLANE + (ly + 1 + dy) * RL + 3 * lx;
#pragma unroll
      for (int q = 0; q < 9; q++) {
        xa[q] = xsv[ra + q];
        xb[q] = xsv[rb + q];
      }
      __builtin_amdgcn_sched_barrier(0);
      if (g9 == 4) {  // (uniform) block 13: the node's own x
        ca0 = xa[3], ca1 = xa[4], ca2 = xa[5];
        cb0 = xb[3], cb1 = xb[4], cb2 = xb[5];
      }
#pragma unroll
      for (int t = 0; t < 3; t++) {
#pragma unroll
        for (int q = 0; q < 9; q++) {
          const int r = q / 3, cc = q % 3;
          const double a = av[t * 9 + q];
          double& ya = r == 0 ? ya0 : (r == 1 ? ya1 : ya2);
          double& yb = r == 0 ? yb0 : (r == 1 ? yb1 : yb2);
          ya = __builtin_fma(a, xa[3 * t + cc], ya);
          yb = __builtin_fma(a, xb[3 * t + cc], yb);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    {  // y of both nodes: branch-free buffer stores, a node the march leaves at an out-of-range offset
      const bool la = inxy && !((m0 >> ln) & 1ull), lb = two && inxy && !((m1 >> ln) & 1ull);
      const int64_t pls = 3 * (int64_t)g.nx * g.ny;
      const __amdgpu_buffer_rsrc_t ra = sp_rsrc(y + pls * k, pls * 8), rb = sp_rsrc(y + pls * min(k + 1, g.nz - 1), pls * 8);
      const unsigned o = 24u * (unsigned)(i + g.nx * j), oa = la ? o : SP_OOB, ob = lb ? o : SP_OOB;
      typedef unsigned u32x2v __attribute__((ext_vector_type(2)));
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2v, ya0), ra, oa, 0, 2);
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2v, ya1), ra, oa + 8, 0, 2);
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2v, ya2), ra, oa + 16, 0, 2);
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2v, yb0), rb, ob, 0, 2);
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2v, yb1), rb, ob + 8, 0, 2);
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2v, yb2), rb, ob + 16, 0, 2);
      if (DOT && la) dot += ca0 * ya0 + ca1 * ya1 + ca2 * ya2;
      if (DOT && lb) dot += cb0 * yb0 + cb1 * yb1 + cb2 * yb2;
    }
    if (more && !NOSTAGE) {  // (uniform) planes k+3, k+4 replace k-1, k (no longer read); NOSTAGE: timing-only
      __syncthreads();
#pragma unroll
      for (int m = 0; m < NL; m++) {
        const int e = me + m * T;
        if (e < PLANE) {
          xs[(k + 3 - k0 + 1) & 3][e] = PF2 ? cur[0][m] : xr[0][m];
          xs[(k + 4 - k0 + 1) & 3][e] = PF2 ? cur[1][m] : xr[1][m];
        }
      }
      __syncthreads();
    }
  };
  if (PF2) {
    for (int k = k0; k < k1; k += 4) {
      step(k, pfa, pfb);
      if (k + 2 < k1) step(k + 2, pfb, pfa);
    }
  } else {
    for (int k = k0; k < k1; k += 2) step(k, pfa, pfb);
  }
  if (TAIL) {
    __syncthreads();  // every wave is done with the ring: it holds the face patches' x, then the dictionary
    st_faces(g, sf, coef, slot, x, y, dot, &xs[0][0]);
    st_tail<T>(g, list, (int64_t)b * cnt / gridDim.x, (int64_t)(b + 1) * cnt / gridDim.x, I, bdict, exc, x, y,
               reinterpret_cast<double2*>(&xs[0][0]), dot);
  }
  if (DOT) {
    const double s = block_sum<T>(dot, sh);
    if (threadIdx.x == 0) part[blockIdx.x] = s;
  }
}

// the face phase and the listed rows as a kernel of their own (vi_st_tail 0): SFP_T listed rows per
// block (the dictionary staged in the patch's LDS), then one face patch per block
template <bool DOT, bool GATED, bool L16 = true>
__global__ __launch_bounds__(SFP_T) void k_spmv_face(Geo g, StFaces sf, const double* __restrict__ coef,
                                                   const unsigned* __restrict__ slot, const double* __restrict__ x,
                                                   double* __restrict__ y, double* __restrict__ part,
                                                   const CgState* __restrict__ cg, const int* __restrict__ list,
                                                   int64_t cnt, const u32x4* __restrict__ I,
                                                   const double* __restrict__ bdict, const double* __restrict__ exc,
                                                   int nd = VI_MAX) {
  static_assert(SFP_N >= VI_MAX * VIB_STRIDE, "the dictionary fits the patch's LDS");
  __shared__ __attribute__((aligned(16))) double S[SFP_N];
  __shared__ double sh[SFP_T / 64];
  if (GATED && cg->reason) return;
  double dot = 0.;
  // the listed rows' blocks first (their gathers are the launch's longest chains: nine dependent
  // rounds per node before round 6's st_tail16, one now), started before the patches
  constexpr int LPB = L16 ? SFP_T / ST16 : SFP_T;  // listed rows per block (L16: 16 lanes each, st_tail16)
  const int64_t NLB = (cnt + LPB - 1) / LPB;
  if ((int64_t)blockIdx.x >= NLB) {
    const SfPatch q = sf_patch(g, sf, blockIdx.x - NLB);
    sf_stage(g, q, x, S, threadIdx.x);
    __syncthreads();
    sf_rows(g, q, coef, slot, S, y, dot, threadIdx.x);
  } else {
    const int64_t lo = (int64_t)blockIdx.x * LPB;
    if (L16) st_tail16<SFP_T>(g, list, lo, min(cnt, lo + LPB), I, bdict, exc, x, y, reinterpret_cast<double2*>(S), dot, nd);
    else st_tail<SFP_T>(g, list, lo, min(cnt, lo + LPB), I, bdict, exc, x, y, reinterpret_cast<double2*>(S), dot, nd);
  }
  if (DOT) {
    const double sm = block_sum<SFP_T>(dot, sh);
    if (threadIdx.x == 0) part[blockIdx.x] = sm;
  }
}

// ------------------------------------------------------- default-stencil SpMV, x-pair lanes (round 6)
// k_spmv_st (one node per lane, nodes k and k+1) read each node's 81 x values from LDS as 8-B reads.
// k_spmv_sp: every lane computes two x-adjacent nodes of ONE plane; the x row (dy, dz) both need is
// 4 nodes = 12 doubles, six 16-B LDS reads (the pair's 48-B lane stride keeps them 16-B aligned; a
// wave row is 32 lanes = 64 nodes, so every 16-lane group of a ds_read_b128 lies in one staged row
// and covers the 16 bank slots 3 l mod 16: conflict-free for any row pitch).  The block marches a
// 64 x TY tile two planes per step with a 4-slot x ring and k_spmv_st's blocks -> tiles map (z-chunks,
// XCD slabs): the first TY/2 waves compute plane k, the others plane k+1, a wave two tile rows.
// Loads and stores are buffer instructions whose out-of-range offsets the hardware drops (a load
// returns 0): staging and the masked y stores carry no branches, so the compiler counts them and the
// step's wait for its loads (vmcnt counts loads and stores in issue order) leaves the just-issued y
// stores in flight.  With branchy global loads and stores that wait was vmcnt(0): every step waited
// for its y stores' round trip to HBM before refilling the ring (profiles/r06r_*).
// The rows are the fused multiply-adds of k_spmv_st / k_spmv_vibm / k_spmv_face in (nb, c) order, so y
// is bitwise theirs; face and listed nodes (k_st_mask's 16 x 4 patch masks) are left to k_spmv_face.
// TY = 8 (512 threads, two blocks per CU with independent barriers) or 16 (option vi_st_ty).
constexpr int SP_RLP = 198;
// FP (the CG's p update fused into the march, option cg_fusep; single rank, no exception nodes, as
// k_spmv_vibm's FP): the ring is staged from r, the Jacobi index byte and p(i-1) instead of x,
// p(i) = z + beta p(i-1) with z = D^-1 r (k_cg_pupdate's expression, so p is bitwise the
// unfused update's), written to p's buffer i & 1 for the tile's own nodes and multiplied in the
// same step; k_spmv_face then reads that buffer.

template <bool DOT, bool GATED, int TY = 8, bool FP = false, int DBG = 0>
__global__ __launch_bounds__(64 * TY) __attribute__((amdgpu_waves_per_eu(4))) void k_spmv_sp(
    Geo g, const double* __restrict__ coef, const unsigned long long* __restrict__ mask, int npx, int npy,
    const double* __restrict__ x, double* __restrict__ y, double* __restrict__ part, const CgState* __restrict__ cg,
    ZTiling zt, FusedP fp = {}) {
  static_assert(TY == 8 || TY == 16, "64 x 8 tiles (two blocks per CU) or 64 x 16 (one)");
  constexpr int TX = 64, T = 64 * TY, WP = TY / 2, RW = 3 * (TX + 2), RLP = SP_RLP, PR = TY + 2, PLANE = PR * RLP;
  constexpr int SR = T / RW, NL = (PR + SR - 1) / SR;  // staged rows per pass, passes
  static_assert(RLP >= RW && RLP % 2 == 0, "ring rows: 198 doubles, 16-B aligned");
  __shared__ __attribute__((aligned(16))) double xs[4 * PLANE];
  __shared__ double sh[T / 64];
  __shared__ double s9[27];  // value 8 of the default stencil's blocks
  __shared__ double s_jdd[FP ? 3 * VI_MAX : 1];
  if (GATED && cg->reason) return;
  const int b = blockIdx.x;
  const int xcd = b & 7, t8 = b >> 3;
  const int slab = (zt.nty + 7) >> 3;
  const int ty0 = xcd * slab;
  const int nty_here = min(slab, zt.nty - ty0);
  const int per = max(nty_here, 0) * zt.ntx * zt.nzc;
  const int me = threadIdx.x;
  double dot = 0.;
  if (t8 >= per) {  // whole block idle (uniform): its partial only
    if (DOT) {
      const double s = block_sum<T>(dot, sh);
      if (threadIdx.x == 0) part[blockIdx.x] = s;
    }
    return;
  }
  const int txi = t8 % zt.ntx, r8 = t8 / zt.ntx;
  const int tyi = ty0 + r8 % nty_here, zc = r8 / nty_here;
  const int i0 = txi * TX, j0 = tyi * TY;
  const int k0 = zc * zt.kc, k1 = min(g.nz, k0 + zt.kc);
  if (me < 27) s9[me] = coef[me * VIB_STRIDE + 8];
  // FP: the CG step's scalars and p's buffers of this iteration
  const int cgi = FP ? cg->i : 0;
  const double cb = FP ? cg->bcoef : 0.;
  const double* psrc = FP ? fp.pb[(cgi & 1) ^ 1] : x;
  double* pdst = FP ? fp.pb[cgi & 1] : nullptr;
  if (FP)
    for (int t = me; t < 3 * VI_MAX; t += T) s_jdd[t] = fp.jdd[t];
  const int wv = me >> 6, ln = me & 63;
  const int h = __builtin_amdgcn_readfirstlane(wv / WP), w8 = __builtin_amdgcn_readfirstlane(wv % WP);
  const int rw = ln >> 5;          // the lane's row of the wave's two (plane k + h, tile rows 2 w8, 2 w8 + 1)
  const int ix = 2 * (ln & 31);    // tile x of the lane's first node
  const int ly = 2 * w8 + rw;
  // k_st_mask's 16 x 4 patches of the wave's rows: patch row gpy, patch columns gpx0 .. gpx0 + 3;
  // bits 16 q .. 16 q + 15 of a row's patch word: the row's nodes in patch row position q
  const int gpx0 = i0 >> 4, gpy = (j0 >> 2) + (w8 >> 1), q0 = (2 * w8) & 3;  // (uniform)
  const int PX = g.PX, PXY = g.PX * g.PY;
  const int len = 3 * min(TX + 2, g.nx + 2 - i0);
  const int rows = min(TY + 2, g.ny + 2 - j0);
  // Staging map (plane-invariant): threads 0 .. SR RW - 1 stage, thread t the column so = t % RW of
  // the rows sr0 + SR m (sr0 = t / RW, m = 0 .. NL-1): every element's addresses are affine in m and
  // in the plane, so staging costs a few adds per element instead of a division chain
  const bool stg = me < SR * RW;
  const int so = me % RW, sr0 = me / RW;
  const bool sx = stg && so < len;                     // the column exists in the padded box
  const int spo = 3 * (i0 + (j0 + sr0) * PX) + so;     // padded offset of element 0 within its plane
  const int sro = sr0 * RLP + so;                      // its ring offset
  const int64_t PXY3 = 3 * (int64_t)PXY;
  auto srow = [&](int m) { return sx && sr0 + SR * m < rows; };
  auto xload = [&](int p, int m) -> double {  // x of padded plane p + 1 (p = -1 .. nz): 0 outside the box
    if (DBG & 1024) {  // (diagnostic) branchy global loads
      if (!srow(m) || p > g.nz) return 0.;
      return x[(int64_t)(p + 1) * PXY3 + spo + 3 * SR * m * PX];
    }
    const __amdgpu_buffer_rsrc_t rx = sp_rsrc(x + (int64_t)(p + 1) * PXY3, p > g.nz ? 0 : PXY3 * 8);
    const unsigned off = srow(m) ? 8u * (unsigned)(spo + 3 * SR * m * PX) : SP_OOB;
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rx, off, 0, 0));
  };
  auto xstore = [&](int slot, int m, double v) {
    if (stg && sr0 + SR * m < PR) xs[slot * PLANE + sro + SR * m * RLP] = v;
  };
  // FP: the element's owned node (else the zero ghost layer); jx carries 0x100 = owned node,
  // 0x200 = one of this tile's own nodes (its p is written)
  const int sgi = i0 - 1 + so / 3, sd = so - 3 * (so / 3);
  const bool sox = sgi >= 0 && sgi < g.nx, stx = sgi >= i0 && sgi < i0 + TX;
  struct Fe {
    double po, rv;
    unsigned jx;
  };
  // (buffer loads and stores, out-of-range offsets for elements off the owned nodes: no branches)
  const int64_t NXY = (int64_t)g.nx * g.ny;
  auto fload = [&](int p, int m, Fe& f) {
    const int gj = j0 - 1 + sr0 + SR * m;
    const bool own = srow(m) && sox && gj >= 0 && gj < g.ny && p >= 0 && p < g.nz;
    const bool pl_ok = p >= 0 && p < g.nz;  // (uniform)
    const __amdgpu_buffer_rsrc_t rr_ = sp_rsrc(fp.r + 3 * NXY * (pl_ok ? p : 0), pl_ok ? 24 * NXY : 0);
    const __amdgpu_buffer_rsrc_t rj = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<unsigned char*>(fp.jix) + NXY * (pl_ok ? p : 0), (short)0, (int)(pl_ok ? NXY : 0), 0x00020000);
    const __amdgpu_buffer_rsrc_t rp = sp_rsrc(psrc + (int64_t)(p + 1) * PXY3, cgi > 0 && p <= g.nz ? PXY3 * 8 : 0);
    const unsigned nn = (unsigned)(sgi + g.nx * gj);
    typedef unsigned u32x2v __attribute__((ext_vector_type(2)));
    f.rv = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rr_, own ? 8u * (3u * nn + sd) : SP_OOB, 0, 0));
    f.jx = (unsigned)__builtin_amdgcn_raw_buffer_load_b8(rj, own ? nn : SP_OOB, 0, 0) | (own ? 0x100u : 0u) |
           (own && stx && gj >= j0 && gj < j0 + TY && p >= k0 && p < k1 ? 0x200u : 0u);
    f.po = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(
                                          rp, own ? 8u * (unsigned)(spo + 3 * SR * m * PX) : SP_OOB, 0, 0));
  };
  // p(i) of a staged element (k_cg_pupdate's expression: z = D^-1 r, p = z (i = 0) or z + beta p(i-1));
  // a tile's own node's p goes to p's buffer of this iteration
  auto fpn = [&](int p, int m, const Fe& f) -> double {
    const double z = f.rv * s_jdd[3 * (f.jx & 255u) + sd];
    const double pn = cgi == 0 ? z : z + cb * f.po;
    typedef unsigned u32x2v __attribute__((ext_vector_type(2)));
    const __amdgpu_buffer_rsrc_t rd = sp_rsrc(pdst + (int64_t)(p + 1) * PXY3, p <= g.nz ? PXY3 * 8 : 0);
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2v, pn), rd,
                                          (f.jx & 0x200u) ? 8u * (unsigned)(spo + 3 * SR * m * PX) : SP_OOB, 0, 0);
    return (f.jx & 0x100u) ? pn : 0.;
  };
  // prologue: planes k0-1 .. k0+2 in ring slots 0 .. 3, every load issued before the first store
  if (FP) {
    __syncthreads();  // s_jdd
#pragma unroll
    for (int s2 = 0; s2 < 2; s2++) {
      Fe fe[2][NL];
#pragma unroll
      for (int s = 0; s < 2; s++)
#pragma unroll
        for (int m = 0; m < NL; m++) fload(k0 - 1 + 2 * s2 + s, m, fe[s][m]);
#pragma unroll
      for (int s = 0; s < 2; s++)
#pragma unroll
        for (int m = 0; m < NL; m++) xstore(2 * s2 + s, m, fpn(k0 - 1 + 2 * s2 + s, m, fe[s][m]));
    }
  } else {
    double v[4][NL];
#pragma unroll
    for (int s = 0; s < 4; s++)
#pragma unroll
      for (int m = 0; m < NL; m++) v[s][m] = xload(k0 - 1 + s, m);
#pragma unroll
    for (int s = 0; s < 4; s++)
#pragma unroll
      for (int m = 0; m < NL; m++) xstore(s, m, v[s][m]);
  }
  __syncthreads();
  typedef double d2v __attribute__((ext_vector_type(2)));
  typedef unsigned u32x4v __attribute__((ext_vector_type(4)));
  typedef unsigned u32x2v __attribute__((ext_vector_type(2)));
  typedef const __attribute__((address_space(3))) d2v lds_d2v;
  lds_d2v* xs2 = (lds_d2v*)&xs[0];
  // DBG (timing-only diagnostics, option split_dbg; wrong products): 1 = one row's coefficients
  // loaded once before the march (no scalar loads in the row loop), 2 = no x reads in the row loop,
  // 4 = no staging loads, 8 = no rows, 32 = no y stores; 1024 = branchy global loads and stores
  double dav[(DBG & 1) ? 27 : 1], dxw[(DBG & 2) ? 12 : 1];
  if constexpr ((DBG & 1) != 0) {
#pragma unroll
    for (int q = 0; q < 27; q++) dav[q] = coef[(q / 9) * VIB_STRIDE + q % 9];
  }
  if constexpr ((DBG & 2) != 0) {
#pragma unroll
    for (int q = 0; q < 12; q++) dxw[q] = xs[q + ln];
  }
  for (int k = k0; k < k1; k += 2) {
    const bool more = k + 2 < k1;
    const int kk = k + h;
    const bool act = kk < k1;  // (uniform per wave) an odd last plane: the second half's waves idle
    double xr[2][NL];
    Fe fe[2][FP ? NL : 1];
    if (more && !(DBG & 4)) {  // planes k+3 and k+4, in flight during the step
#pragma unroll
      for (int m = 0; m < NL; m++) {
        if (FP) {
          fload(k + 3, m, fe[0][m]);
          fload(k + 4, m, fe[1][m]);
        } else {
          xr[0][m] = xload(k + 3, m);
          xr[1][m] = xload(k + 4, m);
        }
      }
    }
    if ((DBG & 4) && more) {
#pragma unroll
      for (int m = 0; m < NL; m++) xr[0][m] = xr[1][m] = 0.;
    }
    double y00 = 0., y01 = 0., y02 = 0., y10 = 0., y11 = 0., y12 = 0.;
    bool live0 = false, live1 = false;
    if (act) {
      // the live nodes of the wave's two rows (bit x: node i0 + x is marched; faces, listed rows and
      // nodes outside the domain are not): from the 4 patch masks, scalar
      unsigned long long lv[2] = {0ull, 0ull};
#pragma unroll
      for (int p4 = 0; p4 < 4; p4++) {
        unsigned long long mk = ~0ull;
        if (gpx0 + p4 < npx && gpy < npy) mk = mask[((int64_t)kk * npy + gpy) * npx + gpx0 + p4];
#pragma unroll
        for (int r2 = 0; r2 < 2; r2++) lv[r2] |= ((~mk >> (16 * (q0 + r2))) & 0xffffull) << (16 * p4);
      }
      const unsigned long long lvr = rw ? lv[1] : lv[0];
      live0 = (lvr >> ix) & 1ull, live1 = (lvr >> (ix + 1)) & 1ull;
      // a rolled loop over the 9 stencil rows (see k_spmv_st: unrolled, the compiler hoists the
      // rows' scalar loads and spills)
#pragma unroll 1
      for (int g9 = 0; g9 < ((DBG & 8) ? 0 : 9); g9++) {  // stencil row (dy, dz): blocks nb = 3 g9 .. 3 g9 + 2
        const int dy = g9 % 3 - 1, dz = g9 / 3 - 1;
        double av[27], xw[12];
        if constexpr ((DBG & 1) != 0) {
#pragma unroll
          for (int q = 0; q < 27; q++) av[q] = dav[q];
        } else {
#pragma unroll
          for (int t = 0; t < 3; t++) {
#pragma unroll
            for (int q = 0; q < 8; q++) av[t * 9 + q] = coef[(g9 * 3 + t) * VIB_STRIDE + q];
            av[t * 9 + 8] = s9[g9 * 3 + t];
          }
        }
        // nodes ix-1 .. ix+2 of the row: 12 doubles, six 16-B reads
        const int ro = (((kk + dz - k0 + 1) & 3) * PLANE + (ly + 1 + dy) * RLP + 3 * ix) >> 1;
        if constexpr ((DBG & 2) != 0) {
#pragma unroll
          for (int q = 0; q < 12; q++) xw[q] = dxw[q] + (double)g9;
        } else {
#pragma unroll
          for (int q = 0; q < 6; q++) {
            const d2v v = xs2[ro + q];
            xw[2 * q] = v.x;
            xw[2 * q + 1] = v.y;
          }
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int t = 0; t < 3; t++) {
#pragma unroll
          for (int q = 0; q < 9; q++) {
            const int r = q / 3, cc = q % 3;
            const double a = av[t * 9 + q];
            double& ya = r == 0 ? y00 : (r == 1 ? y01 : y02);
            double& yb = r == 0 ? y10 : (r == 1 ? y11 : y12);
            ya = __builtin_fma(a, xw[3 * t + cc], ya);
            yb = __builtin_fma(a, xw[3 * t + 3 + cc], yb);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      if (DOT) {  // p.w with the nodes' own x from the ring (block 13 of the rows: not kept live)
        const int rc = (((kk - k0 + 1) & 3) * PLANE + (ly + 1) * RLP + 3 * ix) >> 1;
        const d2v c0 = xs2[rc + 1], c1 = xs2[rc + 2], c2 = xs2[rc + 3], c3 = xs2[rc + 4];
        // c0 = (x[2], x[3]) ... : node 0's x at doubles 3..5, node 1's at 6..8 of the row segment
        if (live0) dot += c0.y * y00 + c1.x * y01 + c1.y * y02;
        if (live1) dot += c2.x * y10 + c2.y * y11 + c3.x * y12;
      }
    }
    {
      // y: the pair's 6 doubles (48 B), per node (a node's doubles at an out-of-range offset when it is
      // not marched; the compiler merges each node's three 8-B stores into a 16-B and an 8-B one).
      // Outside `act`: every wave issues the same stores (the idle half's all dropped)
      const int64_t pl = 3 * (int64_t)g.nx * g.ny * min(kk, g.nz - 1);  // (uniform) the plane's first double
      const unsigned o0 = 24u * (unsigned)(i0 + ix + g.nx * (j0 + ly));
      if (DBG & 32) {
      } else if (DBG & 1024) {  // (diagnostic) branchy global stores
        double* yp = y + pl + o0 / 8;
        if (live0 && live1) {
          __builtin_nontemporal_store(y00, yp + 0), __builtin_nontemporal_store(y01, yp + 1);
          __builtin_nontemporal_store(y02, yp + 2), __builtin_nontemporal_store(y10, yp + 3);
          __builtin_nontemporal_store(y11, yp + 4), __builtin_nontemporal_store(y12, yp + 5);
        } else {
          if (live0)
            __builtin_nontemporal_store(y00, yp + 0), __builtin_nontemporal_store(y01, yp + 1),
                __builtin_nontemporal_store(y02, yp + 2);
          if (live1)
            __builtin_nontemporal_store(y10, yp + 3), __builtin_nontemporal_store(y11, yp + 4),
                __builtin_nontemporal_store(y12, yp + 5);
        }
      } else {
        // no branch: every lane issues the same stores (the compiler then counts them, and the
        // step's wait for its loads leaves them in flight); an unmarched node's at an out-of-range offset
        const __amdgpu_buffer_rsrc_t ry = sp_rsrc(y + pl, 24 * (int64_t)g.nx * g.ny);
        {
          const unsigned a0 = live0 ? o0 : SP_OOB, a1 = live1 ? o0 + 24 : SP_OOB;
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2v, y00), ry, a0, 0, 2);
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2v, y01), ry, a0 + 8, 0, 2);
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2v, y02), ry, a0 + 16, 0, 2);
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2v, y10), ry, a1, 0, 2);
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2v, y11), ry, a1 + 8, 0, 2);
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2v, y12), ry, a1 + 16, 0, 2);
        }
      }
    }
    if (more) {  // (uniform) planes k+3, k+4 replace k-1, k (no longer read)
      if (FP) {  // their p before the barrier (the loads landed during the rows): off the barrier's path
#pragma unroll
        for (int m = 0; m < NL; m++) {
          xr[0][m] = fpn(k + 3, m, fe[0][m]);
          xr[1][m] = fpn(k + 4, m, fe[1][m]);
        }
      }
      __syncthreads();
#pragma unroll
      for (int m = 0; m < NL; m++) {
        xstore((k + 3 - k0 + 1) & 3, m, xr[0][m]);
        xstore((k + 4 - k0 + 1) & 3, m, xr[1][m]);
      }
      __syncthreads();
    }
  }
  if (DOT) {
    const double s = block_sum<T>(dot, sh);
    if (threadIdx.x == 0) part[blockIdx.x] = s;
  }
}

// Stencil classes of the default-stencil SpMV: 0 the interior (marched), 1/2 the x-lo/x-hi domain
// face, 3/4 y-lo/y-hi, 5/6 z-lo/z-hi (an owned node on exactly one face of the GLOBAL domain: the
// face phase st_faces; a node on two or three is an edge / corner node and always listed).  On the
// uniform grid almost every node of a face has the same 27 block indices (its far-side blocks the
// zero block the DMDA's clipping leaves).
__device__ __forceinline__ int st_class(const Geo& g, int i, int j, int k, int& nf) {
  const bool xl = g.xs == 0 && i == 0, xh = g.xs + g.nx == g.NX && i == g.nx - 1;
  const bool yl = g.ys == 0 && j == 0, yh = g.ys + g.ny == g.NY && j == g.ny - 1;
  const bool zl = g.zs == 0 && k == 0, zh = g.zs + g.nz == g.NZ && k == g.nz - 1;
  nf = (int)(xl || xh) + (int)(yl || yh) + (int)(zl || zh) + (int)(xl && xh) + (int)(yl && yh) + (int)(zl && zh);
  return xl ? 1 : xh ? 2 : yl ? 3 : yh ? 4 : zl ? 5 : zh ? 6 : 0;
}

// block nb's index byte in the node's index words
__device__ __forceinline__ unsigned st_byte(const unsigned* w, int nb) { return (w[nb >> 2] >> (8 * (nb & 3))) & 255u; }

// default-stencil build, pass 0 (one block per class c): the class's representative node -- of up to
// 5 candidates spread over the class's nodes (not exception nodes, on exactly the class's face), the
// one whose index words the most candidates share (the interior: the middle node first; a face: its
// middle and 2 nodes in from its corners, away from Dirichlet edges and load patches) -- its 27 blocks
// as coef[c][27][VIB_STRIDE], its 7 index words as ids[8 c + 0..6] and ids[8 c + 7] = 1 when the
// class is usable: it has a representative (a face: and option vi_st_faces is on).  ids[7] = 0: no
// default stencil at all.
__global__ __launch_bounds__(320) void k_st_setup(Geo g, const u32x4* __restrict__ I, const double* __restrict__ bdict,
                                                  double* __restrict__ coef, unsigned* __restrict__ ids, int faces) {
  __shared__ unsigned wsel[2][8];  // [0] the interior's words, [1] this class's; [.][7] = found
  const int c = blockIdx.x, t = threadIdx.x;
  if (t == 0) {
    for (int pass = 0; pass < (c ? 2 : 1); pass++) {
      const int cc = pass ? c : 0;
      int cand[5][3];
      auto pos = [](int n, int a) { return max(0, min(n - 1, a)); };
      if (cc == 0) {
        const int xs[5] = {g.nx / 2, 2, g.nx - 3, 2, g.nx - 3}, ys[5] = {g.ny / 2, 2, g.ny - 3, g.ny - 3, 2},
                  zs[5] = {g.nz / 2, 2, g.nz - 3, g.nz / 2, g.nz / 2};
        for (int q = 0; q < 5; q++) cand[q][0] = pos(g.nx, xs[q]), cand[q][1] = pos(g.ny, ys[q]), cand[q][2] = pos(g.nz, zs[q]);
      } else {
        const int ax = (cc - 1) >> 1, hi = (cc - 1) & 1;  // face normal 0/1/2, high side
        const int n3[3] = {g.nx, g.ny, g.nz};
        const int ua = ax == 0 ? 1 : 0, va = ax == 2 ? 1 : 2;  // the in-face axes
        const int us[5] = {n3[ua] / 2, 2, n3[ua] - 3, 2, n3[ua] - 3}, vs[5] = {n3[va] / 2, 2, 2, n3[va] - 3, n3[va] - 3};
        for (int q = 0; q < 5; q++) {
          cand[q][ax] = hi ? n3[ax] - 1 : 0;
          cand[q][ua] = pos(n3[ua], us[q]);
          cand[q][va] = pos(n3[va], vs[q]);
        }
      }
      unsigned w[5][7];
      bool ok[5];
      for (int q = 0; q < 5; q++) {
        int nf = 0;
        const int cl = st_class(g, cand[q][0], cand[q][1], cand[q][2], nf);
        const int n = cand[q][0] + g.nx * (cand[q][1] + g.ny * cand[q][2]);
        const u32x4* ip = I + (int64_t)(n >> 6) * (2 * 64) + (n & 63);
        const u32x4 w0 = ip[0], w1 = ip[64];
        for (int r = 0; r < 7; r++) w[q][r] = r < 4 ? w0[r] : w1[r - 4];
        ok[q] = g.nown > 0 && cl == cc && (cc ? nf == 1 : nf == 0) && w1[3] == 0u;
      }
      int best = -1, bestv = 0;
      for (int q = 0; q < 5; q++) {
        if (!ok[q]) continue;
        int v = 0;
        for (int p = 0; p < 5; p++) {
          bool same = ok[p];
          for (int r = 0; r < 7; r++) same = same && w[p][r] == w[q][r];
          v += same;
        }
        if (v > bestv) best = q, bestv = v;
      }
      for (int r = 0; r < 7; r++) wsel[pass][r] = best >= 0 ? w[best][r] : 0u;
      wsel[pass][7] = best >= 0;
    }
    wsel[1][7] = c ? wsel[0][7] && wsel[1][7] && ((faces >> c) & 1) : wsel[0][7];
  }
  __syncthreads();
  const unsigned* w = wsel[c ? 1 : 0];
  if (t < 27 * VIB_STRIDE) {  // rows of VIB_STRIDE doubles like the dictionary's (zeros: class unused)
    const int nb = t / VIB_STRIDE, q = t % VIB_STRIDE;
    coef[c * 27 * VIB_STRIDE + t] = q < 9 && wsel[1][7] ? bdict[st_byte(w, nb) * VIB_STRIDE + q] : 0.;
  }
  if (t < 7) ids[8 * c + t] = w[t];
  if (t == 7) ids[8 * c + 7] = wsel[1][7];
}

// pass 1: flag[n] = 1 for a listed node: an exception node, an edge / corner node, a node of an
// unusable class, or one whose index words differ from its class representative's; cnt[block] =
// the block's count (then k_exc_scan / k_exc_assign: list in owned-node order, flag -> slot + 1)
__global__ __launch_bounds__(TPB) void k_st_flag(Geo g, const u32x4* __restrict__ I, const unsigned* __restrict__ ids,
                                                 unsigned* __restrict__ flag, unsigned* __restrict__ cnt) {
  const int n = blockIdx.x * TPB + threadIdx.x;
  bool nd = false;
  if (n < g.nown) {
    int i, j, k, nf;
    node_ijk(g, n, i, j, k);
    const int cl = st_class(g, i, j, k, nf);
    const unsigned* id = ids + 8 * cl;
    const u32x4* ip = I + (int64_t)(n >> 6) * (2 * 64) + (n & 63);
    const u32x4 w0 = ip[0], w1 = ip[64];
    unsigned diff = w1[3] | (nf > 1) | (id[7] ^ 1u);
#pragma unroll
    for (int q = 0; q < 7; q++) diff |= (q < 4 ? w0[q] : w1[q - 4]) ^ id[q];
    nd = diff != 0u;
    flag[n] = nd ? 1u : 0u;
  }
  const int c = __syncthreads_count(nd);
  if (threadIdx.x == 0) cnt[blockIdx.x] = (unsigned)c;
}

// pass 2: one 64-bit mask per 16 x 4 patch and plane (k_spmv_st's wave layout): bit = the lane's
// node is not marched: on a domain face (the face phase), listed (slot != 0), or outside the domain
__global__ __launch_bounds__(TPB) void k_st_mask(Geo g, const unsigned* __restrict__ slot,
                                                 unsigned long long* __restrict__ mask, int npx, int npy) {
  const int64_t w = (int64_t)blockIdx.x * (TPB / 64) + (threadIdx.x >> 6);
  const int ln = threadIdx.x & 63;
  if (w >= (int64_t)npx * npy * g.nz) return;  // (whole wave)
  const int px = (int)(w % npx);
  const int64_t r = w / npx;
  const int py = (int)(r % npy), k = (int)(r / npy);
  const int i = px * 16 + (ln & 15), j = py * 4 + (ln >> 4);
  bool skip = true;
  if (i < g.nx && j < g.ny) {
    int nf;
    st_class(g, i, j, k, nf);
    skip = nf > 0 || slot[i + g.nx * (j + (int64_t)g.ny * k)] != 0u;  // a face node: the face phase's or listed
  }
  const unsigned long long m = __ballot(skip);
  if (ln == 0) mask[w] = m;
}

// Owned nodes on the global domain boundary (faces whose stencil the DMDA clips), enumerated
// without repetition: the z-face planes (whole nx x ny planes), then in the remaining planes the
// y-face rows (whole nx rows), then in the remaining rows the x-face columns.
struct FaceEnum {
  int kz[2], nkz;      // z-face planes (0 and/or nz-1), count
  int jy[2], njy;      // y-face rows
  int ix[2], nix;      // x-face columns
  int k0, kn, j0, jn;  // the other planes [k0, k0+kn), the other rows [j0, j0+jn)
  int64_t nA, nB, n;   // nodes in the z planes, + the y rows, total
};

static FaceEnum face_enum(const Geo& g) {
  FaceEnum f{};
  auto sides = [](int lo_at_boundary, int hi_at_boundary, int w, int (&v)[2], int& cnt, int& o0, int& on) {
    cnt = 0;
    if (lo_at_boundary) v[cnt++] = 0;
    if (hi_at_boundary && !(cnt && w - 1 == 0)) v[cnt++] = w - 1;
    o0 = lo_at_boundary ? 1 : 0;
    on = std::max(0, w - cnt);
  };
  int dummy0 = 0, dummy1 = 0;
  sides(g.zs == 0, g.zs + g.nz == g.NZ, g.nz, f.kz, f.nkz, f.k0, f.kn);
  sides(g.ys == 0, g.ys + g.ny == g.NY, g.ny, f.jy, f.njy, f.j0, f.jn);
  sides(g.xs == 0, g.xs + g.nx == g.NX, g.nx, f.ix, f.nix, dummy0, dummy1);
  f.nA = (int64_t)f.nkz * g.nx * g.ny;
  f.nB = f.nA + (int64_t)f.kn * f.njy * g.nx;
  f.n = f.nB + (int64_t)f.kn * f.jn * f.nix;
  return f;
}

__device__ __forceinline__ void face_node(const Geo& g, const FaceEnum& f, int64_t t, int& i, int& j, int& k) {
  if (t < f.nA) {
    const int64_t pl = (int64_t)g.nx * g.ny;
    k = f.kz[t / pl];
    j = (int)((t % pl) / g.nx);
    i = (int)(t % g.nx);
  } else if (t < f.nB) {
    t -= f.nA;
    const int64_t rows = (int64_t)f.njy * g.nx;
    k = f.k0 + (int)(t / rows);
    j = f.jy[(t % rows) / g.nx];
    i = (int)(t % g.nx);
  } else {
    t -= f.nB;
    const int64_t cols = (int64_t)f.jn * f.nix;
    k = f.k0 + (int)(t / cols);
    j = f.j0 + (int)((t % cols) / f.nix);
    i = f.ix[t % f.nix];
  }
}

// Exact rows (-mat_vi_fma 0) of the value-indexed block storage on the global domain boundary:
// the z-marching kernel leaves them out (their inode pairing follows the present columns, a
// per-node pattern, which would put runtime pairing on every wave touching the boundary).  One
// node per thread, x gathered from the padded vector, blocks from the dictionary in global memory
// (20 KB, cached) or from the exception array, InodeRows with the node's presence mask; the block
// p.w partial goes after the z-march's partials (part[blockIdx.x] of this grid).
template <bool DOT, bool GATED, bool EXC>
__global__ __launch_bounds__(TPB) void k_spmv_vib_faces(Geo g, const u32x4* __restrict__ I,
                                                        const double* __restrict__ bdict,
                                                        const double* __restrict__ x, double* __restrict__ y,
                                                        double* __restrict__ part, const CgState* __restrict__ cg,
                                                        FaceEnum fe, const double* __restrict__ exc) {
  __shared__ double sh[TPB / 64];
  if (GATED && cg->reason) return;
  const int64_t t = (int64_t)blockIdx.x * TPB + threadIdx.x;
  double dot = 0.;
  if (t < fe.n) {
    int i, j, k;
    face_node(g, fe, t, i, j, k);
    const int64_t n = i + g.nx * (j + (int64_t)g.ny * k);
    const int PX = g.PX, PXY = g.PX * g.PY;
    const int pc = (i + 1) + (j + 1) * PX + (k + 1) * PXY;
    const u32x4* ip = I + (n >> 6) * (2 * 64) + (n & 63);
    const u32x4 w0 = ip[0], w1 = ip[64];
    const unsigned slot = EXC ? w1[3] : 0u;
    InodeRows<false> acc;
    acc.pres = present_mask(g, i, j, k);
    double xc0 = 0., xc1 = 0., xc2 = 0.;
#pragma unroll
    for (int nb = 0; nb < 27; nb++) {
      if (!((acc.pres >> nb) & 1u)) continue;
      const int off = (nb % 3 - 1) + ((nb / 3) % 3 - 1) * PX + (nb / 9 - 1) * PXY;
      const double* xp = x + 3 * (int64_t)(pc + off);
      const double xv[3] = {xp[0], xp[1], xp[2]};
      if (nb == 13) {
        xc0 = xv[0];
        xc1 = xv[1];
        xc2 = xv[2];
      }
      const double* e;
      int es = 1;  // stride of the block's values: the dictionary's 1, the exception array's 64
      if (EXC && slot) {
        e = exc + exc_base(slot - 1) + nb * 9 * 64;
        es = 64;
      } else {
        const unsigned word = nb < 16 ? w0[nb >> 2] : w1[(nb - 16) >> 2];
        e = bdict + ((word >> (8 * (nb & 3))) & 255u) * VIB_STRIDE;
      }
#pragma unroll
      for (int q = 0; q < 9; q++) acc.term(nb, q / 3, q % 3, e[q * es] * xv[q % 3]);
    }
    const double y0 = acc.row(0), y1 = acc.row(1), y2 = acc.row(2);
    y[3 * n + 0] = y0;
    y[3 * n + 1] = y1;
    y[3 * n + 2] = y2;
    if (DOT) dot = xc0 * y0 + xc1 * y1 + xc2 * y2;
  }
  if (DOT) {
    const double sm = block_sum<TPB>(dot, sh);
    if (threadIdx.x == 0) part[blockIdx.x] = sm;
  }
}

// The exception rows of the block-indexed storage: after the z-march (which
// leaves them out, vi_exc_kernel), one thread per exception slot over the whole device instead of a
// block-wide pass in the tail of the tile that owns them.  Slots are in owned-node order (ordered
// compaction) and exc is slot fastest, so the 243 value loads of a wave are whole lines; x is
// gathered from the padded vector.  Each row adds its 27 blocks' terms in the order and with the
// products of the z-march's rows (FMA: one fused multiply-add per term in (nb, c) order; exact:
// the inode pairs of a node with all 27 neighbours — exact rows of boundary nodes are the faces
// kernel's), so y is bitwise what the in-tile pass computed.  The block's p.w partial goes after
// the z-march's and the faces kernel's partials.
template <bool DOT, bool GATED, bool FMA>
__global__ __launch_bounds__(TPB) void k_spmv_exc(Geo g, const int* __restrict__ xlist, int64_t nexc,
                                                  const double* __restrict__ exc, const double* __restrict__ x,
                                                  double* __restrict__ y, double* __restrict__ part,
                                                  const CgState* __restrict__ cg) {
  __shared__ double sh[TPB / 64];
  if (GATED && cg->reason) return;
  const int64_t t = (int64_t)blockIdx.x * TPB + threadIdx.x;
  double dot = 0.;
  int n = -1, i = 0, j = 0, k = 0;
  if (t < nexc) {
    n = xlist[t];
    node_ijk(g, n, i, j, k);
    if (!FMA && present_mask(g, i, j, k) != PRES_ALL) n = -1;  // k_spmv_vib_faces' row
  }
  if (n >= 0) {
    const int PX = g.PX, PXY = g.PX * g.PY;
    const double* eb = exc + exc_base(t);  // value v at eb[v * 64]
    double y0 = 0., y1 = 0., y2 = 0., xc0 = 0., xc1 = 0., xc2 = 0.;
    InodeRows<true> acc;
#pragma unroll 1
    for (int nb0 = 0; nb0 < 27; nb0 += 3) {  // one dy row of the stencil: 27 values, 9 x
      double av[27];
#pragma unroll
      for (int q = 0; q < 27; q++) av[q] = eb[(nb0 * 9 + q) * 64];
      const int dy = (nb0 / 3) % 3 - 1, dz = nb0 / 9 - 1;
      const double* xr = x + 3 * ((int64_t)i + (j + 1 + dy) * (int64_t)PX + (k + 1 + dz) * (int64_t)PXY);
      double xw[9];
#pragma unroll
      for (int q = 0; q < 9; q++) xw[q] = xr[q];  // nodes i-1, i, i+1 of the row (padded i = node i + 1)
#pragma unroll
      for (int t3 = 0; t3 < 3; t3++) {
        const double xv[3] = {xw[3 * t3], xw[3 * t3 + 1], xw[3 * t3 + 2]};
        if (nb0 + t3 == 13) {
          xc0 = xv[0];
          xc1 = xv[1];
          xc2 = xv[2];
        }
#pragma unroll
        for (int q = 0; q < 9; q++) {
          const int r = q / 3, cc = q % 3;
          double& yr = r == 0 ? y0 : (r == 1 ? y1 : y2);
          if constexpr (FMA) yr = __builtin_fma(av[t3 * 9 + q], xv[cc], yr);
          else acc.term(nb0 + t3, r, cc, av[t3 * 9 + q] * xv[cc]);
        }
      }
    }
    if constexpr (!FMA) y0 = acc.row(0), y1 = acc.row(1), y2 = acc.row(2);
    __builtin_nontemporal_store(y0, &y[3 * (int64_t)n + 0]);
    __builtin_nontemporal_store(y1, &y[3 * (int64_t)n + 1]);
    __builtin_nontemporal_store(y2, &y[3 * (int64_t)n + 2]);
    if (DOT) dot = xc0 * y0 + xc1 * y1 + xc2 * y2;
  }
  if (DOT) {
    const double sm = block_sum<TPB>(dot, sh);
    if (threadIdx.x == 0) part[blockIdx.x] = sm;
  }
}

// y = A x on FMT_VI with x staged in LDS, z-marching.  k_spmv_vi's 81 x gathers per node (8 B
// at a 24-B lane stride: a third of every fetched line used) are a third of its time
// (profiles/old/r02_vi_dbg.log: 1.14 ms, 0.78 without them); staging one plane per block and launch
// was slower still (1.39 ms: one 113-KB block per CU waits on its own staging,
// profiles/old/r02_ab_vis_*.log).  Here a 1024-thread block owns a TX x TY node tile and marches it
// up a z-chunk: LDS holds a ring of three x planes (rows j0-1 .. j0+TY, TX+2 nodes each, as
// contiguous in the padded box), and while plane k is computed the registers already carry plane
// k+2's x (coalesced 8-B loads, 1.5 x per owned node at TY = 4) and plane k+1's index chunks,
// written to the ring after the step's barrier.  Same slot order and products as k_spmv:
// bit-identical to the reference's AIJ MatMult (inode order, oracle/oracle.c row_part).
template <bool DOT, bool GATED, int TX, int TY, int NIB>
__global__ __launch_bounds__(TX * TY) void k_spmv_vim(Geo g, const u32x4* __restrict__ I,
                                                      const double* __restrict__ dict, const double* __restrict__ x,
                                                      double* __restrict__ y, double* __restrict__ part,
                                                      const CgState* __restrict__ cg, ZTiling zt) {
  constexpr int T = TX * TY, RL = 3 * (TX + 2), PR = TY + 2, PLANE = PR * RL;  // doubles per staged plane
  constexpr int NL = (PLANE + T - 1) / T;                                      // x loads per thread per plane
  constexpr int CH = vi_chunks<NIB>(), NT = NIB == 8 ? VI_MAX : NSLOT * 16;
  __shared__ double xs[3][PLANE];
  __shared__ double tab[NT];
  __shared__ double sh[T / 64];
  if (GATED && cg->reason) return;
  const int b = blockIdx.x;
  const int xcd = b & 7, t8 = b >> 3;
  const int slab = (zt.nty + 7) >> 3;
  const int ty0 = xcd * slab;
  const int nty_here = min(slab, zt.nty - ty0);
  const int per = max(nty_here, 0) * zt.ntx * zt.nzc;
  if (t8 >= per) {  // whole block idle (uniform): still write the partial
    if (DOT && threadIdx.x == 0) part[blockIdx.x] = 0.;
    return;
  }
  const int txi = t8 % zt.ntx, r8 = t8 / zt.ntx;  // x tiles fastest, then the slab's tile rows, then z-chunks
  const int tyi = ty0 + r8 % nty_here, zc = r8 / nty_here;
  const int i0 = txi * TX, j0 = tyi * TY;
  const int k0 = zc * zt.kc, k1 = min(g.nz, k0 + zt.kc);
  const int me = threadIdx.x, lx = me % TX, ly = me / TX;
  const int i = i0 + lx, j = j0 + ly;
  const bool inxy = i < g.nx && j < g.ny;
  const int PX = g.PX, PXY = g.PX * g.PY;
  const int len = 3 * min(TX + 2, g.nx + 2 - i0);  // doubles of a staged row that exist in the padded box
  const int rows = min(TY + 2, g.ny + 2 - j0);      // staged rows (j0-1 ..) that exist (padded j <= ny)
  // x of node plane p (-1 .. nz): staged element e = rr * RL + o of padded row j0+rr, plane p+1
  auto xload = [&](int p, int m) -> double {
    const int e = me + m * T;
    const int rr = e / RL, o = e - rr * RL;
    if (e >= PLANE || o >= len || rr >= rows) return 0.;
    return x[3 * (int64_t)(i0 + (j0 + rr) * PX + (p + 1) * PXY) + o];
  };
  auto xstore = [&](int slot, int m, double v) {
    const int e = me + m * T;
    if (e < PLANE) xs[slot][e] = v;
  };
  auto iload = [&](int k, u32x4 (&w)[CH]) {
    if (inxy) {
      const int n = i + g.nx * (j + g.ny * k);
      const u32x4* ip = I + (int64_t)(n >> 6) * (CH * 64) + (n & 63);
#pragma unroll
      for (int q = 0; q < CH; q++) w[q] = __builtin_nontemporal_load(ip + q * 64);
    }
  };
  for (int t = me; t < NT; t += T) tab[t] = dict[t];
  // prologue: planes k0-1, k0, k0+1 in ring slots 0, 1, 2 (plane p in slot (p - k0 + 1) % 3)
#pragma unroll
  for (int s = 0; s < 3; s++)
#pragma unroll
    for (int m = 0; m < NL; m++) xstore(s, m, xload(k0 - 1 + s, m));
  u32x4 cur[CH], nxt[CH];
  iload(k0, cur);
  __syncthreads();
  double dot = 0.;
  for (int k = k0; k < k1; k++) {
    const bool more = k + 1 < k1;
    double xr[NL];
    if (more) {  // in flight during this plane: x of plane k+2 (the padded ghost plane at most), indices of k+1
#pragma unroll
      for (int m = 0; m < NL; m++) xr[m] = xload(k + 2, m);
      iload(k + 1, nxt);
    }
    if (inxy) {
      double xc0 = 0., xc1 = 0., xc2 = 0.;
      InodeRows<false> acc;
      acc.pres = present_mask(g, i, j, k);
#pragma unroll
      for (int nb = 0; nb < 27; nb++) {
        const int dx = nb % 3 - 1, dy = (nb / 3) % 3 - 1, dz = nb / 9 - 1;
        const double* xp = xs[(k + dz - k0 + 1) % 3] + (ly + 1 + dy) * RL + 3 * (lx + 1 + dx);
        const double xv[3] = {xp[0], xp[1], xp[2]};
        if (nb == 13) {
          xc0 = xv[0];
          xc1 = xv[1];
          xc2 = xv[2];
        }
#pragma unroll
        for (int q = 0; q < 9; q++) {
          const int S = nb * 9 + q, r = q / 3, cc = q % 3;
          const double v = tab[vi_entry<NIB>(S, vi_index<NIB>(cur, S))];
          acc.term(nb, r, cc, v * xv[cc]);
        }
      }
      const double y0 = acc.row(0), y1 = acc.row(1), y2 = acc.row(2);
      const int64_t n = i + g.nx * (j + (int64_t)g.ny * k);
      __builtin_nontemporal_store(y0, &y[3 * n + 0]);
      __builtin_nontemporal_store(y1, &y[3 * n + 1]);
      __builtin_nontemporal_store(y2, &y[3 * n + 2]);
      if (DOT) dot += xc0 * y0 + xc1 * y1 + xc2 * y2;
    }
    if (more) {  // uniform
      __syncthreads();  // plane k-1's slot is free
#pragma unroll
      for (int m = 0; m < NL; m++) xstore((k + 2 - k0 + 1) % 3, m, xr[m]);
#pragma unroll
      for (int q = 0; q < CH; q++) cur[q] = nxt[q];
      __syncthreads();
    }
  }
  if (DOT) {
    double s = block_sum<T>(dot, sh);
    if (threadIdx.x == 0) part[blockIdx.x] = s;
  }
}

static void z_shape(int kern, int& ztx, int& zty) {
  switch (kern) {
    case 2: ztx = 32; zty = 4; break;
    case 3: ztx = 64; zty = 2; break;
    case 4: ztx = 128; zty = 2; break;
    case 5: ztx = 128; zty = 4; break;
    case 6: ztx = 256; zty = 2; break;
    case 7: ztx = 128; zty = 4; break;  // phased (k_spmv_symp) from here on
    case 8: ztx = 64; zty = 4; break;
    case 9: ztx = 64; zty = 8; break;
    case 10: ztx = 256; zty = 2; break;
    case 11: ztx = 256; zty = 4; break;
    default: ztx = 64; zty = 4; break;
  }
}

template <int ZTX, int ZTY, bool AIJS = false>
static void launch_symp(Ctx& c, const double* xpad, double* y, bool dot, bool gated, const ZTiling& zt, int nb) {
  const uint16_t* Dq = c.D;
  DSlots dl = c.dsl;
  if (AIJS && dl.dense) {  // the z-march without corrections, then the dense pass (with the dot)
    DSlots none = dl;
    none.L = 0;
    none.Lq = 0;
    if (gated)
      hipLaunchKernelGGL((k_spmv_symp<false, true, ZTX, ZTY, AIJS>), dim3(nb), dim3(ZTX * ZTY), 0, c.stream, c.g, c.U,
                         xpad, y, c.partials, c.cg, zt, Dq, none);
    else
      hipLaunchKernelGGL((k_spmv_symp<false, false, ZTX, ZTY, AIJS>), dim3(nb), dim3(ZTX * ZTY), 0, c.stream, c.g,
                         c.U, xpad, y, c.partials, c.cg, zt, Dq, none);
    const dim3 gd((unsigned)((c.g.nown + TPB - 1) / TPB));
    const unsigned* en = dl.esc && dl.nesc ? c.esc_node : nullptr;
    const double* er = c.esc_res;
    const unsigned char* es = c.esc_slot;
    if (dot && gated && dl.wide)
      hipLaunchKernelGGL((k_split_dense<true, true, true>), gd, dim3(TPB), 0, c.stream, c.g, Dq, dl.Lq, xpad, y,
                         c.partials, c.cg);
    else if (dot && gated)
      hipLaunchKernelGGL((k_split_dense<true, true, false>), gd, dim3(TPB), 0, c.stream, c.g, Dq, dl.Lq, xpad, y,
                         c.partials, c.cg, en, er, es);
    else if (dot && dl.wide)
      hipLaunchKernelGGL((k_split_dense<true, false, true>), gd, dim3(TPB), 0, c.stream, c.g, Dq, dl.Lq, xpad, y,
                         c.partials, c.cg);
    else if (dot)
      hipLaunchKernelGGL((k_split_dense<true, false, false>), gd, dim3(TPB), 0, c.stream, c.g, Dq, dl.Lq, xpad, y,
                         c.partials, c.cg, en, er, es);
    else if (dl.wide)
      hipLaunchKernelGGL((k_split_dense<false, false, true>), gd, dim3(TPB), 0, c.stream, c.g, Dq, dl.Lq, xpad, y,
                         c.partials, c.cg);
    else
      hipLaunchKernelGGL((k_split_dense<false, false, false>), gd, dim3(TPB), 0, c.stream, c.g, Dq, dl.Lq, xpad, y,
                         c.partials, c.cg, en, er, es);
    return;
  }
  if (c.split_dbg) {  // timing-only diagnostics (wrong products): 1 = loads, no corrections; 2 = neither
    dl.L = 0;
    if (c.split_dbg == 2) dl.Lq = 0;
  }
  if (dot && gated)
    hipLaunchKernelGGL((k_spmv_symp<true, true, ZTX, ZTY, AIJS>), dim3(nb), dim3(ZTX * ZTY), 0, c.stream, c.g, c.U,
                       xpad, y, c.partials, c.cg, zt, Dq, dl);
  else if (dot)
    hipLaunchKernelGGL((k_spmv_symp<true, false, ZTX, ZTY, AIJS>), dim3(nb), dim3(ZTX * ZTY), 0, c.stream, c.g, c.U,
                       xpad, y, c.partials, c.cg, zt, Dq, dl);
  else
    hipLaunchKernelGGL((k_spmv_symp<false, false, ZTX, ZTY, AIJS>), dim3(nb), dim3(ZTX * ZTY), 0, c.stream, c.g, c.U,
                       xpad, y, c.partials, c.cg, zt, Dq, dl);
}

template <int ZTX, int ZTY>
static void launch_symz(Ctx& c, const double* xpad, double* y, bool dot, bool gated, const ZTiling& zt, int nb) {
  if (dot && gated)
    hipLaunchKernelGGL((k_spmv_symz<true, true, ZTX, ZTY>), dim3(nb), dim3(ZTX * ZTY), 0, c.stream, c.g, c.U, xpad, y,
                       c.partials, c.cg, zt);
  else if (dot)
    hipLaunchKernelGGL((k_spmv_symz<true, false, ZTX, ZTY>), dim3(nb), dim3(ZTX * ZTY), 0, c.stream, c.g, c.U, xpad, y,
                       c.partials, c.cg, zt);
  else
    hipLaunchKernelGGL((k_spmv_symz<false, false, ZTX, ZTY>), dim3(nb), dim3(ZTX * ZTY), 0, c.stream, c.g, c.U, xpad,
                       y, c.partials, c.cg, zt);
}

// ---------------------------------------------------------------------------- CG vectors
// KSPSolve_CG (PETSc, KSP_NORM_PRECONDITIONED, zero guess) + PCApply_Jacobi, with the scalar
// recurrences kept on the device (CgState) so the host only polls every few iterations.
__device__ __forceinline__ int converged_default(const CgState* s, double rn) {
  if (isnan(rn) || isinf(rn)) return MCX_KSP_DIVERGED_NANORINF;
  if (rn <= s->ttol) return rn < s->abstol ? MCX_KSP_CONVERGED_ATOL : MCX_KSP_CONVERGED_RTOL;
  if (rn >= s->dtol * s->rnorm0) return MCX_KSP_DIVERGED_DTOL;
  return 0;
}

// r <- b; x <- 0; z <- D^-1 r; partials z.z, z.r
__global__ __launch_bounds__(TPB) void k_cg_init(Geo g, const double* __restrict__ bvec, const double* __restrict__ dinv,
                                                 double* __restrict__ x, double* __restrict__ r,
                                                 double* __restrict__ z, double* __restrict__ part, int nparts) {
  __shared__ double sh[TPB / 64];
  int n = blockIdx.x * TPB + threadIdx.x;
  double zz = 0., zr = 0.;
  if (n < g.nown) {
#pragma unroll
    for (int d = 0; d < 3; d++) {
      const int q = 3 * n + d;
      const double rv = bvec[q];
      const double zv = rv * dinv[q];
      x[q] = 0.;
      r[q] = rv;
      z[q] = zv;
      zz += zv * zv;
      zr += zv * rv;
    }
  }
  double s0 = block_sum<TPB>(zz, sh);
  double s1 = block_sum<TPB>(zr, sh);
  if (threadIdx.x == 0) {
    part[blockIdx.x] = s0;
    part[nparts + blockIdx.x] = s1;
  }
}

// p <- z (i == 0) or z + (beta/betaold) p   (VecCopy / VecAYPX).  The previous iteration's
// VecAXPY(x, alpha, p) is applied here, where p is read anyway (same operation and rounding as
// in KSPSolve_CG, one iteration later; k_cg_xfinal applies the last one): the update kernel
// then reads neither x nor p.
template <bool NT>
__device__ __forceinline__ void st(double* p, double v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// Jacobi inverse diagonal of DOF 3n+d.  DIX (block-indexed value storage): dinv is the
// dictionary's inverse diagonals [VI_MAX][3] and jix the owned nodes' diagonal-block index (one
// byte per node instead of 24 B of dinv); the values are k_jacobi_vib's, so z = r * dinv is
// bit-identical either way.  jix 255 (an exception node, or dictionary block 255): the node's
// own entry of the Jacobi vector, which the context keeps right behind the dictionary's
// (c.dinv = c.jdd + 3 VI_MAX) — the same value for a dictionary block, the only one for an
// exception node; a branch no lane of an exception-free wave takes.
template <bool DIX>
__device__ __forceinline__ double jac_inv(const double* __restrict__ dinv, const unsigned char* __restrict__ jix,
                                          int n, int d) {
  if constexpr (DIX) {
    const unsigned jx = jix[n];
    if (jx == 255u) return dinv[3 * VI_MAX + 3 * n + d];
    return dinv[3 * jx + d];
  } else {
    return dinv[3 * n + d];
  }
}

// z of DOF q = 3n+d: stored z, or (DIX) recomputed from r (the update kernel then writes no z)
template <bool DIX>
__device__ __forceinline__ double z_of(const double* __restrict__ z, const double* __restrict__ dinv,
                                       const unsigned char* __restrict__ jix, int n, int d) {
  if constexpr (DIX) return z[3 * n + d] * jac_inv<true>(dinv, jix, n, d);
  else return z[3 * n + d];
}

template <bool NT, bool DIX>
__device__ __forceinline__ void pupdate_node(const Geo& g, int n, const double* __restrict__ z,
                                             const double* __restrict__ dinv, const unsigned char* __restrict__ jix,
                                             double* __restrict__ ppad, double* __restrict__ x,
                                             const CgState* __restrict__ cg) {
  int i, j, k;
  node_ijk(g, n, i, j, k);
  const int pc = pad_of(g, i, j, k);
  if (cg->i == 0) {
#pragma unroll
    for (int d = 0; d < 3; d++) st<NT>(&ppad[3 * pc + d], z_of<DIX>(z, dinv, jix, n, d));
  } else {
    const double bc = cg->bcoef, a = cg->alpha;
#pragma unroll
    for (int d = 0; d < 3; d++) {
      const int q = 3 * n + d;
      const double pv = ppad[3 * pc + d];
      st<NT>(&x[q], x[q] + a * pv);
      st<NT>(&ppad[3 * pc + d], z_of<DIX>(z, dinv, jix, n, d) + bc * pv);
    }
  }
}

// a node some neighbour rank receives: on a subdomain face that has a neighbour (width-1 halo)
__device__ __forceinline__ bool sent_node(const Geo& g, int i, int j, int k) {
  return (i == 0 && g.xs > 0) || (i == g.nx - 1 && g.xs + g.nx < g.NX) || (j == 0 && g.ys > 0) ||
         (j == g.ny - 1 && g.ys + g.ny < g.NY) || (k == 0 && g.zs > 0) || (k == g.nz - 1 && g.zs + g.nz < g.NZ);
}

// PDB (option cg_pdb): p double-buffered, p(i) in pb[i & 1].  Iteration i reads p(i-1) from the
// other buffer and writes p(i) = z + (beta/betaold) p(i-1); VecAXPY(x) runs on odd iterations
// only, both owed terms in PETSc's order: x = (x + a(i-2) p(i-2)) + a(i-1) p(i-1), p(i-2) being
// read from p(i)'s buffer before it is overwritten (i = 1: the one term a(0) p(0)).  Even
// iterations move 73 B per node instead of 121, odd ones 145.  xdone = the last odd iteration
// (every term j < xdone applied); k_cg_xfinal applies the rest.
template <bool NT, bool DIX>
__device__ __forceinline__ void pupdate_node_db(const Geo& g, int n, const double* __restrict__ z,
                                                const double* __restrict__ dinv, const unsigned char* __restrict__ jix,
                                                double* __restrict__ pb0, double* __restrict__ pb1,
                                                double* __restrict__ x, const CgState* __restrict__ cg) {
  int i, j, k;
  node_ijk(g, n, i, j, k);
  const int pc = pad_of(g, i, j, k);
  const int it = cg->i;
  double* pn = (it & 1) ? pb1 : pb0;
  const double* po = (it & 1) ? pb0 : pb1;
  if (it == 0) {
#pragma unroll
    for (int d = 0; d < 3; d++) st<NT>(&pn[3 * pc + d], z_of<DIX>(z, dinv, jix, n, d));
    return;
  }
  // every load before any store (pn / po are selected at run time: the compiler cannot tell
  // them apart, and would otherwise order each load after the previous component's stores)
  const double bc = cg->bcoef, a = cg->alpha;
  double pv[3], zv[3], xv[3], pp[3];
#pragma unroll
  for (int d = 0; d < 3; d++) {
    pv[d] = po[3 * pc + d];
    zv[d] = z_of<DIX>(z, dinv, jix, n, d);
  }
  if (it & 1) {
    const double ap = cg->alpha_prev;
#pragma unroll
    for (int d = 0; d < 3; d++) {
      xv[d] = x[3 * n + d];
      pp[d] = it >= 3 ? pn[3 * pc + d] : 0.;
    }
#pragma unroll
    for (int d = 0; d < 3; d++) {
      if (it >= 3) xv[d] = xv[d] + ap * pp[d];
      st<NT>(&x[3 * n + d], xv[d] + a * pv[d]);
    }
  }
#pragma unroll
  for (int d = 0; d < 3; d++) st<NT>(&pn[3 * pc + d], zv[d] + bc * pv[d]);
}

// PAR (option cg_par): the iteration's parity as the host counts it, so one kernel holds one
// straight path with every load issued before the first use: 1 = an even iteration >= 2 (73 B
// per node), 2 = an odd one >= 3 (145 B); 0 = the parity read from cg->i (also the fallback
// should the device's count ever differ from the host's)
template <bool NT, bool DIX, int PAR>
__device__ __forceinline__ void pupdate_node_par(const Geo& g, int n, const double* __restrict__ z,
                                                 const double* __restrict__ dinv,
                                                 const unsigned char* __restrict__ jix, double* __restrict__ pb0,
                                                 double* __restrict__ pb1, double* __restrict__ x,
                                                 const CgState* __restrict__ cg) {
  int i, j, k;
  node_ijk(g, n, i, j, k);
  const int pc = pad_of(g, i, j, k);
  double* pn = PAR == 2 ? pb1 : pb0;
  const double* po = PAR == 2 ? pb0 : pb1;
  const double bc = cg->bcoef, a = cg->alpha;
  double pv[3], zv[3], xv[3], pp[3];
#pragma unroll
  for (int d = 0; d < 3; d++) {
    pv[d] = po[3 * pc + d];
    if (PAR == 2) {
      xv[d] = x[3 * n + d];
      pp[d] = pn[3 * pc + d];
    }
    zv[d] = z_of<DIX>(z, dinv, jix, n, d);
  }
  if (PAR == 2) {
    const double ap = cg->alpha_prev;
#pragma unroll
    for (int d = 0; d < 3; d++) st<NT>(&x[3 * n + d], (xv[d] + ap * pp[d]) + a * pv[d]);
  }
#pragma unroll
  for (int d = 0; d < 3; d++) st<NT>(&pn[3 * pc + d], zv[d] + bc * pv[d]);
}

template <bool NT, bool DIX, bool SKIP_SENT = false, int PAR = 0>
__global__ void k_cg_pupdate_db(Geo g, const double* __restrict__ z, const double* __restrict__ dinv,
                                const unsigned char* __restrict__ jix, double* __restrict__ pb0,
                                double* __restrict__ pb1, double* __restrict__ x, const CgState* __restrict__ cg,
                                int* __restrict__ xdone, const int* __restrict__ list, int64_t cnt,
                                int rev = 0) {
  if (cg->reason) return;
  const int64_t t = (int64_t)blockIdx.x * TPB + threadIdx.x;
  const int it = cg->i;
  if (t == 0 && (it & 1)) *xdone = it;
  if (t >= cnt) return;
  // rev (option cg_rev): nodes from the last one down (no reduction here: same results)
  const int n = list ? list[t] : (int)(rev ? cnt - 1 - t : t);
  if (SKIP_SENT) {
    int i, j, k;
    node_ijk(g, n, i, j, k);
    if (sent_node(g, i, j, k)) return;
  }
  if constexpr (PAR != 0) {
    if (it >= 2 && (it & 1) == (PAR == 2 ? 1 : 0)) {
      pupdate_node_par<NT, DIX, PAR>(g, n, z, dinv, jix, pb0, pb1, x, cg);
      return;
    }
  }
  pupdate_node_db<NT, DIX>(g, n, z, dinv, jix, pb0, pb1, x, cg);
}

// PQB (option cg_pdb 4): p in four buffers, p(i) in pq[i & 3], and VecAXPY(x) on every fourth
// iteration only: at i = 4m (m >= 1) the four owed terms in PETSc's order,
// x = (((x + a(i-4) p(i-4)) + a(i-3) p(i-3)) + a(i-2) p(i-2)) + a(i-1) p(i-1), p(i-4) read from
// p(i)'s buffer before it is overwritten, the alphas from CgState::ah.  x then costs
// (48 + 3 x 24) / 4 = 30 B per node and iteration instead of PDB's 36.  xdone = the last such i;
// k_cg_xfinal_qb applies the (at most four) terms still owed.
// PAR: 1 = an iteration >= 1 without the x terms, 2 = one with them (i = 4m >= 4), 0 = from cg->i
// XS (option cg_xs): p in eight buffers, p(i) in pq[i & 7], and the four owed x terms left to
// k_cg_xwin on a side stream (this kernel only marks the window: xdone = i)
struct PQ {
  double* p[8];
};
// P2D (option cg_p2d): grid (ny nz rows, x chunks), the node's row from the block index, so the
// row / plane split is scalar work instead of two vector integer divisions per node
template <bool NT, bool DIX, bool SKIP_SENT = false, int PAR = 0, bool XS = false, bool P2D = false>
__global__ void k_cg_pupdate_qb(Geo g, const double* __restrict__ z, const double* __restrict__ dinv,
                                const unsigned char* __restrict__ jix, PQ pq, double* __restrict__ x,
                                const CgState* __restrict__ cg, int* __restrict__ xdone,
                                const int* __restrict__ list, int64_t cnt, int rev = 0) {
  constexpr int M = XS ? 7 : 3;  // buffer ring mask
  if (cg->reason) return;
  const int64_t t = P2D ? (int64_t)blockIdx.y * TPB + threadIdx.x : (int64_t)blockIdx.x * TPB + threadIdx.x;
  const int it = cg->i;
  const bool dox = it >= 4 && (it & 3) == 0;
  if (t == 0 && dox && (!P2D || blockIdx.x == 0)) *xdone = it;
  int n, i, j, k;
  if (P2D) {
    const int row = blockIdx.x;  // (uniform)
    i = (int)t;
    if (i >= g.nx) return;
    j = row % g.ny;
    k = row / g.ny;
    n = i + g.nx * row;
  } else {
    if (t >= cnt) return;
    n = list ? list[t] : (int)(rev ? cnt - 1 - t : t);
    node_ijk(g, n, i, j, k);
  }
  if (SKIP_SENT && sent_node(g, i, j, k)) return;
  const int pc = pad_of(g, i, j, k);
  double* pn = pq.p[it & M];
  if (it == 0) {
#pragma unroll
    for (int d = 0; d < 3; d++) st<NT>(&pn[3 * pc + d], z_of<DIX>(z, dinv, jix, n, d));
    return;
  }
  // the x terms follow the device's count (dox), whatever the host's parity hint PAR: a wrong
  // hint costs a kernel built for the other branch, never an x term (a PAR 1 launch
  // at i = 4m used to mark xdone without applying the four owed terms).  cg_par 2 skews the hint
  // on purpose (test_cg_par_hint_mismatch_bitwise).
  const double* po = pq.p[(it - 1) & M];
  const double bc = cg->bcoef;
  double pv[3], zv[3];
  if (!XS && dox) {
    const double* p3 = pq.p[(it - 3) & 3];
    const double* p2 = pq.p[(it - 2) & 3];
    const double a4 = cg->ah[(it - 4) & 7], a3 = cg->ah[(it - 3) & 7], a2 = cg->ah[(it - 2) & 7],
                 a1 = cg->ah[(it - 1) & 7];
    double xv[3], q4[3], q3[3], q2[3];
#pragma unroll
    for (int d = 0; d < 3; d++) {  // every load before any store
      pv[d] = po[3 * pc + d];
      zv[d] = z_of<DIX>(z, dinv, jix, n, d);
      xv[d] = x[3 * n + d];
      q4[d] = pn[3 * pc + d];
      q3[d] = p3[3 * pc + d];
      q2[d] = p2[3 * pc + d];
    }
#pragma unroll
    for (int d = 0; d < 3; d++) st<NT>(&x[3 * n + d], (((xv[d] + a4 * q4[d]) + a3 * q3[d]) + a2 * q2[d]) + a1 * pv[d]);
  } else {
#pragma unroll
    for (int d = 0; d < 3; d++) {
      pv[d] = po[3 * pc + d];
      zv[d] = z_of<DIX>(z, dinv, jix, n, d);
    }
  }
#pragma unroll
  for (int d = 0; d < 3; d++) st<NT>(&pn[3 * pc + d], zv[d] + bc * pv[d]);
}

// XS: the window i0-4 .. i0-1 of VecAXPY(x) terms, on the side stream while the main stream runs
// the next iterations (it waits for this kernel before p(i0+4) overwrites p(i0-4)'s buffer);
// skipped unless iteration i0's p update ran (xdone == i0), so a finished solve's window is left
// to k_cg_xfinal_qb.  The same terms in the same order as k_cg_pupdate_qb's: bitwise the same x.
__global__ __launch_bounds__(TPB) void k_cg_xwin(Geo g, PQ pq, double* __restrict__ x,
                                                 const CgState* __restrict__ cg, const int* __restrict__ xdone,
                                                 int i0) {
  if (*xdone != i0) return;
  const int n = blockIdx.x * TPB + threadIdx.x;
  if (n >= g.nown) return;
  int i, j, k;
  node_ijk(g, n, i, j, k);
  const int pc = pad_of(g, i, j, k);
  const double a4 = cg->ah[(i0 - 4) & 7], a3 = cg->ah[(i0 - 3) & 7], a2 = cg->ah[(i0 - 2) & 7],
               a1 = cg->ah[(i0 - 1) & 7];
  const double* q4 = pq.p[(i0 - 4) & 7];
  const double* q3 = pq.p[(i0 - 3) & 7];
  const double* q2 = pq.p[(i0 - 2) & 7];
  const double* q1 = pq.p[(i0 - 1) & 7];
  double xv[3], v4[3], v3[3], v2[3], v1[3];
#pragma unroll
  for (int d = 0; d < 3; d++) {
    xv[d] = x[3 * n + d];
    v4[d] = q4[3 * pc + d];
    v3[d] = q3[3 * pc + d];
    v2[d] = q2[3 * pc + d];
    v1[d] = q1[3 * pc + d];
  }
#pragma unroll
  for (int d = 0; d < 3; d++) x[3 * n + d] = (((xv[d] + a4 * v4[d]) + a3 * v3[d]) + a2 * v2[d]) + a1 * v1[d];
}

// PQB: the terms j = xdone .. xp still owed after the loop (at most four), in order (m: the
// buffer ring's mask, 3 or 7)
__global__ void k_cg_xfinal_qb(Geo g, PQ pq, double* __restrict__ x, const CgState* __restrict__ cg,
                               const int* __restrict__ xdone, int m) {
  const int xd = *xdone, xp = cg->xp;
  if (xp < xd) return;
  const int n = blockIdx.x * TPB + threadIdx.x;
  if (n >= g.nown) return;
  int i, j, k;
  node_ijk(g, n, i, j, k);
  const int pc = pad_of(g, i, j, k);
#pragma unroll
  for (int d = 0; d < 3; d++) {
    double xv = x[3 * n + d];
    for (int jj = xd; jj <= xp; jj++) xv = xv + cg->ah[jj & 7] * pq.p[jj & m][3 * pc + d];
    x[3 * n + d] = xv;
  }
}

// SKIP_SENT: the sent nodes were updated before the halo exchange (k_cg_pupdate_list)
template <bool NT, bool DIX, bool SKIP_SENT = false>
__global__ void k_cg_pupdate(Geo g, const double* __restrict__ z, const double* __restrict__ dinv,
                             const unsigned char* __restrict__ jix, double* __restrict__ ppad,
                             double* __restrict__ x, const CgState* __restrict__ cg) {
  if (cg->reason) return;
  int n = blockIdx.x * TPB + threadIdx.x;
  if (n >= g.nown) return;
  if (SKIP_SENT) {
    int i, j, k;
    node_ijk(g, n, i, j, k);
    if (sent_node(g, i, j, k)) return;
  }
  pupdate_node<NT, DIX>(g, n, z, dinv, jix, ppad, x, cg);
}

template <bool NT, bool DIX>
__global__ void k_cg_pupdate_list(Geo g, const double* __restrict__ z, const double* __restrict__ dinv,
                                  const unsigned char* __restrict__ jix, double* __restrict__ ppad,
                                  double* __restrict__ x, const CgState* __restrict__ cg,
                                  const int* __restrict__ list, int64_t cnt) {
  if (cg->reason) return;
  const int64_t t = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (t >= cnt) return;
  pupdate_node<NT, DIX>(g, list[t], z, dinv, jix, ppad, x, cg);
}

// the last iteration's x += alpha p (when that iteration reached its update); ppad2: the fused
// path's second p buffer (p of iteration i in buffer i & 1)
__global__ void k_cg_xfinal(Geo g, const double* __restrict__ ppad, const double* __restrict__ ppad2,
                            double* __restrict__ x, const CgState* __restrict__ cg, const int* __restrict__ xdone) {
  if (xdone) {  // PDB: the terms j = xdone .. xp still owed (at most two), in order
    const int xd = *xdone, xp = cg->xp;
    if (xp < xd) return;
    int n = blockIdx.x * TPB + threadIdx.x;
    if (n >= g.nown) return;
    int i, j, k;
    node_ijk(g, n, i, j, k);
    const int pc = pad_of(g, i, j, k);
    const double* pl = (xp & 1) ? ppad2 : ppad;
    const double* pp = (xp & 1) ? ppad : ppad2;
#pragma unroll
    for (int d = 0; d < 3; d++) {
      double xv = x[3 * n + d];
      if (xp - 1 >= xd) xv = xv + cg->alpha_prev * pp[3 * pc + d];
      x[3 * n + d] = xv + cg->alpha * pl[3 * pc + d];
    }
    return;
  }
  if (ppad2) {
    // fused path: odd iterations' updates applied x through them, so only an even last
    // successful iteration xp (whose update ran, but applies no x) leaves a(xp) p(xp) pending;
    // an indefinite matrix stops before the update of xp + 1, cg->alpha is still a(xp)
    if (cg->xp < 0 || (cg->xp & 1)) return;
  } else if (!cg->xpend) {
    return;
  }
  int n = blockIdx.x * TPB + threadIdx.x;
  if (n >= g.nown) return;
  int i, j, k;
  node_ijk(g, n, i, j, k);
  const int pc = pad_of(g, i, j, k);
  const double a = cg->alpha;
#pragma unroll
  for (int d = 0; d < 3; d++) x[3 * n + d] = x[3 * n + d] + a * ppad[3 * pc + d];
}

// r += (-a) w; z = D^-1 r; partials z.z, z.r   (x += a p: deferred to k_cg_pupdate)
// 1024-thread blocks: a quarter of the partials for k_reduce (one block reads them all).  Option
// cg_ublocks caps the grid (grid-stride: a thread's nodes n, n + grid, ... summed in that order)
// so that k_reduce sums fewer partials: 0.8676 (2,048 blocks) / 0.8708 (512) against 0.8492 ms
// per CG iteration uncapped at 256^3 (profiles/old/r04_cg_ab_ublocks256.log): the update kernel
// loses more than the reduction saves
static constexpr int UTPB = 1024;

template <bool NT, bool DIX>
__global__ __launch_bounds__(UTPB) void k_cg_update(Geo g, const double* __restrict__ w,
                                                   const double* __restrict__ dinv,
                                                   const unsigned char* __restrict__ jix,
                                                   double* __restrict__ r, double* __restrict__ z,
                                                   double* __restrict__ part, int nparts,
                                                   const CgState* __restrict__ cg) {
  __shared__ double sh[UTPB / 64];
  if (cg->reason) return;
  const double ma = -cg->alpha;
  double zz = 0., zr = 0.;
  for (int n = blockIdx.x * UTPB + threadIdx.x; n < g.nown; n += gridDim.x * UTPB) {
#pragma unroll
    for (int d = 0; d < 3; d++) {
      const int q = 3 * n + d;
      const double rv = r[q] + ma * w[q];
      st<NT>(&r[q], rv);
      const double zv = rv * jac_inv<DIX>(dinv, jix, n, d);
      if (!DIX) st<NT>(&z[q], zv);
      zz += zv * zv;
      zr += zv * rv;
    }
  }
  double s0 = block_sum<UTPB>(zz, sh);
  double s1 = block_sum<UTPB>(zr, sh);
  if (threadIdx.x == 0) {
    part[blockIdx.x] = s0;
    part[nparts + blockIdx.x] = s1;
  }
}

// the fused p-update path's update (FusedP): r += (-a) w; z = D^-1 r; partials z.z, z.r; and on
// odd iterations i the two VecAXPYs of x that iterations i-1 and i owe, x = (x + a(i-1) p(i-1))
// + a(i) p(i), from the two p buffers (p(i) in pb[i&1]) — the same operations, in the same
// order, as KSPSolve_CG's VecAXPY(x) per iteration
template <bool NT>
__global__ __launch_bounds__(UTPB) void k_cg_update_x(Geo g, const double* __restrict__ w,
                                                     const double* __restrict__ jdd,
                                                     const unsigned char* __restrict__ jix, double* __restrict__ r,
                                                     double* __restrict__ x, const double* __restrict__ pb0,
                                                     const double* __restrict__ pb1, double* __restrict__ part,
                                                     int nparts, const CgState* __restrict__ cg) {
  __shared__ double sh[UTPB / 64];
  if (cg->reason) return;
  const double a = cg->alpha, ma = -a;
  const int it = cg->i;
  int n = blockIdx.x * UTPB + threadIdx.x;
  double zz = 0., zr = 0.;
  if (n < g.nown) {
    const unsigned jx = jix[n];
#pragma unroll
    for (int d = 0; d < 3; d++) {
      const int q = 3 * n + d;
      const double rv = r[q] + ma * w[q];
      st<NT>(&r[q], rv);
      // jix 255: the node's entry of the Jacobi vector behind the dictionary's (jac_inv<true>)
      const double zv = rv * (jx == 255u ? jdd[3 * VI_MAX + q] : jdd[3 * jx + d]);
      zz += zv * zv;
      zr += zv * rv;
    }
    if (it & 1) {  // uniform
      int i, j, k;
      node_ijk(g, n, i, j, k);
      const int pc = pad_of(g, i, j, k);
      const double ap = cg->alpha_prev;
      const double* pp = (it & 1) ? pb0 : pb1;  // p(i-1) (i odd: buffer 0)
      const double* pi = (it & 1) ? pb1 : pb0;  // p(i)
#pragma unroll
      for (int d = 0; d < 3; d++) {
        const int q = 3 * n + d;
        const double x1 = x[q] + ap * pp[3 * pc + d];
        st<NT>(&x[q], x1 + a * pi[3 * pc + d]);
      }
    }
  }
  double s0 = block_sum<UTPB>(zz, sh);
  double s1 = block_sum<UTPB>(zr, sh);
  if (threadIdx.x == 0) {
    part[blockIdx.x] = s0;
    part[nparts + blockIdx.x] = s1;
  }
}

// ---- single rank: the CG scalar steps folded into the vector kernels (no k_reduce launch) ----
// Two device CgState buffers alternate between kernels: the update reads B and writes A, the
// fused p update reads A and writes B.  Every block reduces the partial sums it needs itself,
// in one fixed order (so all blocks compute the same scalars), runs the PETSc CG step on a
// private copy of the state, and block 0 stores it.  A finished solve's state is copied on
// unchanged, so gated kernels keep seeing its reason.
__device__ void cg_logic_alpha(CgState* s, double dpi);
__device__ void cg_logic_beta(CgState* s, double zz, double zr, double* hist);

// r += (-a) w; z = D^-1 r; partials z.z, z.r — with alpha from the SpMV's p.w partials
// (k_reduce's RED_ALPHA step, same summation tree for npw <= UTPB)
template <bool NT, bool DIX>
__global__ __launch_bounds__(UTPB) void k_cg_update_fa(Geo g, const double* __restrict__ w,
                                                      const double* __restrict__ dinv,
                                                      const unsigned char* __restrict__ jix, double* __restrict__ r,
                                                      double* __restrict__ z, double* __restrict__ part, int nparts,
                                                      const double* __restrict__ part_pw, int npw,
                                                      const CgState* __restrict__ cg_in, CgState* __restrict__ cg_out) {
  __shared__ double sh[UTPB / 64];
  __shared__ double s_alpha;
  __shared__ int s_reason;
  double v = 0.;
  for (int q = threadIdx.x; q < npw; q += UTPB) v += part_pw[q];
  const double pw = block_sum<UTPB>(v, sh);
  if (threadIdx.x == 0) {
    CgState st = *cg_in;
    cg_logic_alpha(&st, pw);
    if (blockIdx.x == 0) *cg_out = st;
    s_alpha = st.alpha;
    s_reason = st.reason;
  }
  __syncthreads();
  if (s_reason) return;
  const double ma = -s_alpha;
  int n = blockIdx.x * UTPB + threadIdx.x;
  double zz = 0., zr = 0.;
  if (n < g.nown) {
#pragma unroll
    for (int d = 0; d < 3; d++) {
      const int q = 3 * n + d;
      const double rv = r[q] + ma * w[q];
      st<NT>(&r[q], rv);
      const double zv = rv * jac_inv<DIX>(dinv, jix, n, d);
      if (!DIX) st<NT>(&z[q], zv);
      zz += zv * zv;
      zr += zv * rv;
    }
  }
  double s0 = block_sum<UTPB>(zz, sh);
  double s1 = block_sum<UTPB>(zr, sh);
  if (threadIdx.x == 0) {
    part[blockIdx.x] = s0;
    part[nparts + blockIdx.x] = s1;
  }
}

// the sum k_reduce forms over n <= 1024 values (block_sum<1024>: one value per thread, a
// shuffle tree per 64-value group, the 16 group sums added in order), with 256 threads, so the
// fused steps compute the same scalars bit for bit
__device__ __forceinline__ double sum1024_by256(const double* __restrict__ v, int n, double* sh) {
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
#pragma unroll
  for (int gq = 0; gq < 4; gq++) {
    const int q = (w * 4 + gq) * 64 + l;
    const double x = wave_sum(q < n ? v[q] : 0.);
    if (l == 0) sh[w * 4 + gq] = x;
  }
  __syncthreads();
  double r = 0.;
  if (threadIdx.x == 0)
    for (int q = 0; q < 16; q++) r += sh[q];
  __syncthreads();
  return r;
}

// p update with beta from the update's z.z / z.r partials (k_reduce's RED_BETA step)
template <bool NT, bool DIX>
__global__ __launch_bounds__(TPB) void k_cg_pupdate_fb(Geo g, const double* __restrict__ z,
                                                      const double* __restrict__ dinv,
                                                      const unsigned char* __restrict__ jix,
                                                      double* __restrict__ ppad, double* __restrict__ x,
                                                      const double* __restrict__ part, int nparts,
                                                      const CgState* __restrict__ cg_in, CgState* __restrict__ cg_out,
                                                      double* __restrict__ hist) {
  __shared__ double sh[16];
  __shared__ CgState s_st;
  const double zz = sum1024_by256(part, nparts, sh);
  const double zr = sum1024_by256(part + nparts, nparts, sh);
  if (threadIdx.x == 0) {
    CgState st = *cg_in;
    cg_logic_beta(&st, zz, zr, blockIdx.x == 0 ? hist : nullptr);
    if (blockIdx.x == 0) *cg_out = st;
    s_st = st;
  }
  __syncthreads();
  if (s_st.reason) return;
  const int n = blockIdx.x * TPB + threadIdx.x;
  if (n >= g.nown) return;
  int i, j, k;
  node_ijk(g, n, i, j, k);
  const int pc = pad_of(g, i, j, k);
  const double bc = s_st.bcoef, a = s_st.alpha;
#pragma unroll
  for (int d = 0; d < 3; d++) {
    const int q = 3 * n + d;
    const double pv = ppad[3 * pc + d];
    st<NT>(&x[q], x[q] + a * pv);
    st<NT>(&ppad[3 * pc + d], z_of<DIX>(z, dinv, jix, n, d) + bc * pv);
  }
}

// CG scalar steps (thread 0 of the reduction block)
__device__ void cg_logic_init(CgState* s, double zz, double zr, double* hist) {
  const double dp = sqrt(zz);
  s->dp = dp;
  if (s->hist_on) hist[0] = dp;
  s->ttol = fmax(s->rtol * dp, s->abstol);
  s->rnorm0 = dp;
  s->i = 0;
  s->its = 0;
  s->dpi = 0.;
  s->betaold = 0.;
  s->xpend = 0;
  s->reason = converged_default(s, dp);
  if (s->reason) return;
  s->beta = zr;
  s->its = 1;
  if (zr == 0.0) s->reason = MCX_KSP_CONVERGED_ATOL;
}

__device__ void cg_logic_alpha(CgState* s, double dpi) {
  if (s->reason) return;
  const double dpiold = s->dpi;
  s->dpiold = dpiold;
  s->dpi = dpi;
  s->betaold = s->beta;
  if (dpi == 0.0 || (s->i > 0 && dpi * dpiold <= 0.0)) {
    s->reason = MCX_KSP_DIVERGED_INDEFINITE_MAT;  // before VecAXPY: the pending x update is none
    s->xpend = 0;
    return;
  }
  s->alpha_prev = s->alpha;
  s->alpha = s->beta / dpi;
  s->ah[s->i & 7] = s->alpha;
  s->xpend = 1;
  s->xp = s->i;
}

__device__ void cg_logic_beta(CgState* s, double zz, double zr, double* hist) {
  if (s->reason) return;
  const double dp = sqrt(zz);
  s->dp = dp;
  if (s->hist_on && hist) hist[s->i + 1] = dp;
  int rs = converged_default(s, dp);
  if (rs) {
    s->reason = rs;
    return;
  }
  s->beta = zr;
  s->i += 1;
  if (s->i >= s->maxits) {
    s->reason = MCX_KSP_DIVERGED_ITS;
    return;
  }
  s->its = s->i + 1;
  if (zr == 0.0) {
    s->reason = MCX_KSP_CONVERGED_ATOL;
    return;
  }
  if (zr * s->betaold < 0.0) {
    s->reason = MCX_KSP_DIVERGED_INDEFINITE_PC;
    return;
  }
  s->bcoef = zr / s->betaold;
}

enum { RED_STORE = 0, RED_INIT = 1, RED_ALPHA = 2, RED_BETA = 3, RED_NORM = 4 };

// res[v] = sum_i part[v*nparts + i], v < nvals <= 2, by one 1024-thread block (thread 0's
// result): k_reduce's fixed summation tree
__device__ __forceinline__ void reduce_parts(const double* part, int nparts, int nvals, double* sh, double res[2]) {
  for (int v = 0; v < nvals; v++) {
    // 8 independent accumulators per thread keep 8 loads in flight; fixed combination order
    const double* pv = part + (int64_t)v * nparts;
    double a[8] = {0., 0., 0., 0., 0., 0., 0., 0.};
    int q = threadIdx.x;
    for (; q + 7 * 1024 < nparts; q += 8 * 1024) {
#pragma unroll
      for (int u = 0; u < 8; u++) a[u] += pv[q + u * 1024];
    }
    for (; q < nparts; q += 1024) a[0] += pv[q];
    const double acc = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
    res[v] = block_sum<1024>(acc, sh);
  }
}

// one block: out[v] = sum_i part[v*nparts + i] (fixed order); then optional CG logic.
// mode RED_STORE writes the local sums only (an all-reduce + k_cg_logic follows).
// cg_src: the state the step starts from (copied to cg first when it is the other buffer)
__global__ __launch_bounds__(1024) void k_reduce(const double* __restrict__ part, int nparts, int nvals,
                                                 double* __restrict__ out, int mode, CgState* cg,
                                                 double* __restrict__ hist, int gated, const CgState* cg_src) {
  __shared__ double sh[16];
  // the gate and the partials are loaded together, one round trip: the partials are read even by a
  // finished solve's launch (nothing is written then)
  // the gate as a vector (buffer) load: waited for with the partials' loads (vmcnt, in order), where a
  // scalar load's wait (lgkmcnt(0)) would come first, with the kernel arguments'
  const int reason = (int)__builtin_amdgcn_raw_buffer_load_b32(
      __builtin_amdgcn_make_buffer_rsrc(const_cast<CgState*>(cg_src), (short)0, (int)sizeof(CgState), 0x00020000),
      (unsigned)offsetof(CgState, reason), 0, 0);
  if (cg_src != cg && threadIdx.x == 0) *cg = *cg_src;  // read by thread 0 only below
  double res[2] = {0., 0.};
  reduce_parts(part, nparts, nvals, sh, res);
  if (threadIdx.x || (gated && reason)) return;
  for (int v = 0; v < nvals; v++) out[v] = res[v];
  if (mode == RED_INIT) cg_logic_init(cg, res[0], res[1], hist);
  else if (mode == RED_ALPHA) cg_logic_alpha(cg, res[0]);
  else if (mode == RED_BETA) cg_logic_beta(cg, res[0], res[1], hist);
  else if (mode == RED_NORM) out[0] = sqrt(res[0]);
}

__global__ void k_cg_logic(const double* __restrict__ red, int mode, CgState* cg, double* __restrict__ hist,
                           double* __restrict__ out) {
  if (threadIdx.x) return;
  if (mode == RED_INIT) cg_logic_init(cg, red[0], red[1], hist);
  else if (mode == RED_ALPHA) cg_logic_alpha(cg, red[0]);
  else if (mode == RED_BETA) cg_logic_beta(cg, red[0], red[1], hist);
  else if (mode == RED_NORM) out[0] = sqrt(red[0]);
}

// in-process all-reduce: out[v] = sum over ranks (rank order) of ptrs[r][v]
// in-process all-reduce over the group members' buffers, in rank order (op 0 sum, 1 max)
__global__ void k_group_sum(const double* const* __restrict__ ptrs, int nranks, int count, double* __restrict__ out,
                            int op) {
  int v = threadIdx.x;
  if (v >= count) return;
  double s = op ? ptrs[0][v] : 0.;
  for (int r = op ? 1 : 0; r < nranks; r++) s = op ? fmax(s, ptrs[r][v]) : s + ptrs[r][v];
  out[v] = s;
}

// reaction-force post-processing (src/forces.c:82-91, :145-155): per element of one boundary
// layer, the plain sum over its 8 Gauss points of stress component `comp`, in GP order.
// The layer is global element index `fixed` along axis `fa`; (a, b) = the other two axes in
// the reference's loop order (outer a over [a0, a0+na), inner b over [b0, b0+nb)).
__global__ void k_force_layer(Geo g, const double* __restrict__ sig, int comp, int fa, int fixed, int a0, int na,
                              int b0, int nb, double* __restrict__ out) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= na * nb) return;
  const int ia = t / nb, ib = t % nb;
  int e[3];
  e[fa] = fixed;
  e[fa == 0 ? 1 : 0] = a0 + ia;
  e[2] = b0 + ib;
  const int64_t le = (e[0] - g.ex0) + (int64_t)(e[1] - g.ey0) * g.nex + (int64_t)(e[2] - g.ez0) * g.nex * g.ney;
  double s = 0.;
#pragma unroll
  for (int gp = 0; gp < 8; gp++) s += sig[((int64_t)comp * 8 + gp) * g.nelem + le];
  out[t] = s;
}

// ---------------------------------------------------------------------------- misc vectors
__global__ void k_update_u(Geo g, double* __restrict__ u, const double* __restrict__ du) {
  int n = blockIdx.x * TPB + threadIdx.x;
  if (n >= g.nown) return;
  int i, j, k;
  node_ijk(g, n, i, j, k);
  const int pc = pad_of(g, i, j, k);
#pragma unroll
  for (int d = 0; d < 3; d++) u[3 * pc + d] = u[3 * pc + d] + 1. * du[3 * n + d];
}

__global__ void k_owned_to_pad(Geo g, const double* __restrict__ src, double* __restrict__ pad) {
  int n = blockIdx.x * TPB + threadIdx.x;
  if (n >= g.nown) return;
  int i, j, k;
  node_ijk(g, n, i, j, k);
  const int pc = pad_of(g, i, j, k);
#pragma unroll
  for (int d = 0; d < 3; d++) pad[3 * pc + d] = src[3 * n + d];
}

__global__ void k_pad_to_owned(Geo g, const double* __restrict__ pad, double* __restrict__ dst) {
  int n = blockIdx.x * TPB + threadIdx.x;
  if (n >= g.nown) return;
  int i, j, k;
  node_ijk(g, n, i, j, k);
  const int pc = pad_of(g, i, j, k);
#pragma unroll
  for (int d = 0; d < 3; d++) dst[3 * n + d] = pad[3 * pc + d];
}

__global__ void k_pack(const int* __restrict__ idx, int64_t cnt, const double* __restrict__ pad, double* __restrict__ buf) {
  int64_t t = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (t >= cnt) return;
  const int p = idx[t];
#pragma unroll
  for (int d = 0; d < 3; d++) buf[3 * t + d] = pad[3 * (int64_t)p + d];
}

__global__ void k_unpack(const int* __restrict__ idx, int64_t cnt, const double* __restrict__ buf, double* __restrict__ pad) {
  int64_t t = (int64_t)blockIdx.x * TPB + threadIdx.x;
  if (t >= cnt) return;
  const int p = idx[t];
#pragma unroll
  for (int d = 0; d < 3; d++) pad[3 * (int64_t)p + d] = buf[3 * t + d];
}

// ============================================================================ launchers
static inline unsigned nblk(int64_t n) { return (unsigned)((n + TPB - 1) / TPB); }

int dirichlet_mask_host(const Geo& g, int gi, int gj, int gk) { return dirichlet_mask(g, gi, gj, gk); }

int64_t node_blocks(const Ctx& c) { return nblk(c.g.nown); }
// AIJ-split SpMV tile: the phased z-marching kernel, 128x4 where the subdomain is wide enough
static void split_shape(const Ctx& c, int& ztx, int& zty) {
  ztx = c.split_tx ? c.split_tx : (c.g.nx >= 256 ? 256 : (c.g.nx >= 128 ? 128 : 64));
  // tiles 256x4 (1 block / CU), 128x4 (2), 64x4 (4); 256x2, 128x8, 64x16.  Defaults by subdomain
  // width: 256x4, 128x8 (128^3: 0.478 vs 0.496 ms for 128x4), 64x4 (64^3: 0.0716 ms, best of
  // six shapes / chunkings), profiles/old/r02_ab_{64,128}.log
  zty = c.split_ty ? c.split_ty : (ztx == 128 && !c.split_tx ? 8 : 4);
  const bool built = (ztx == 256 && (zty == 2 || zty == 4)) || (ztx == 128 && (zty == 4 || zty == 8)) ||
                     (ztx == 64 && (zty == 4 || zty == 16));
  if (!built) zty = 4;  // the launcher instantiates only these shapes
}

// FMT_VI with x staged in LDS (k_spmv_vim): 1024-thread tiles TX x TY marching z-chunks, one
// resident round of blocks (one per CU: the ring and the dictionaries fill the LDS)
// 64x16 tiles: with the scalar-dictionary 16x4 patches, 256^3 0.358 vs 0.419 ms (256x4) and
// 128^3 0.0563 vs 0.0589 ms (128x8) per SpMV (profiles/old/r03_ab_tx{256b,128}.log): a third less
// halo than 256x4 (66x18 staged nodes per 1024 instead of 258x6), and tiles away from the x
// faces have no wave that reads the dictionary from LDS.  Option vi_tx selects 256x4 / 128x8.
static void vis_shape(const Ctx& c, int& tx, int& ty) {
  tx = 64;
  if (c.vi_tx == 256 || c.vi_tx == 128 || c.vi_tx == 64) tx = c.vi_tx;
  ty = 1024 / tx;
}

static ZTiling vis_tiling(const Ctx& c) {
  int tx, ty;
  vis_shape(c, tx, ty);
  ZTiling t;
  t.ntx = (c.g.nx + tx - 1) / tx;
  t.nty = (c.g.ny + ty - 1) / ty;
  const int tiles = t.ntx * t.nty, want = c.spmv_zblocks > 0 ? c.spmv_zblocks : c.g.ncu;
  t.nzc = std::max(1, std::min(c.g.nz, (want + tiles - 1) / tiles));
  t.kc = (c.g.nz + t.nzc - 1) / t.nzc;
  t.nzc = (c.g.nz + t.kc - 1) / t.kc;
  return t;
}

// staged (z-marching) value-indexed SpMV: forced by option vi_stage 0 / 1, else where a block
// marches at least 4 planes (256^3: 0.49 vs 0.66 ms gathered, 128^3 0.073 vs 0.090; 64^3, one
// plane per block: 0.024 vs 0.012; profiles/old/r02_vibm_ab*.log)
bool vi_staged(const Ctx& c) {
  if (c.vi_stage >= 0) return c.vi_stage != 0;
  return vis_tiling(c).kc >= 4;
}

static bool sp_used(const Ctx& c);
static ZTiling sp_tiling(const Ctx& c);

int64_t spmv_grid_blocks(const Ctx& c) {
  if (sp_used(c)) {
    const ZTiling t = sp_tiling(c);
    return 8 * (int64_t)(((t.nty + 7) / 8) * t.ntx * t.nzc);
  }
  if (c.fmt == FMT_VI && vi_staged(c) && (c.vi_bits == 4 || c.vi_block)) {  // launch_spmv's staged kernels
    const ZTiling t = vis_tiling(c);
    return 8 * (int64_t)(((t.nty + 7) / 8) * t.ntx * t.nzc);
  }
  if (c.fmt == FMT_SPLIT || (c.fmt == FMT_U && c.spmv_kernel >= 1)) {
    int ztx, zty;
    if (c.fmt == FMT_SPLIT) split_shape(c, ztx, zty);
    else z_shape(c.spmv_kernel, ztx, zty);
    const ZTiling zt = z_tiling(c.g, ztx, zty, c.spmv_zblocks);
    return 8 * (int64_t)(((zt.nty + 7) / 8) * zt.ntx * zt.nzc);
  }
  const SpmvTiling t = spmv_tiling(c.g, c.spmv_subl);
  if (c.spmv_subl < 0) return (int64_t)c.g.nz * t.jgroups * t.nxc;
  return 8 * (int64_t)t.per_xcd;
}
void spmv_tile(const Ctx& c, int* tx, int* ty, int* kc) {
  *tx = *ty = *kc = 0;
  if (sp_used(c)) {
    *tx = 64;
    *ty = c.vi_st_ty;
    *kc = sp_tiling(c).kc;
  } else if (c.fmt == FMT_VI && vi_staged(c) && (c.vi_bits == 4 || c.vi_block)) {
    vis_shape(c, *tx, *ty);
    *kc = vis_tiling(c).kc;
  } else if (c.fmt == FMT_SPLIT || (c.fmt == FMT_U && c.spmv_kernel >= 1)) {
    if (c.fmt == FMT_SPLIT) split_shape(c, *tx, *ty);
    else z_shape(c.spmv_kernel, *tx, *ty);
    *kc = z_tiling(c.g, *tx, *ty, c.spmv_zblocks).kc;
  }
}

// exact value-indexed rows on the staged kernel: the boundary-face pass's blocks (their p.w
// partials follow the z-march's)
static int64_t faces_blocks(const Ctx& c) {
  if (!(c.fmt == FMT_VI && c.vi_block && vi_staged(c) && !c.vi_fma)) return 0;
  return (face_enum(c.g).n + TPB - 1) / TPB;
}

bool fusep(const Ctx& c);
bool st_fusep(const Ctx& c);

// the default-stencil SpMV (k_spmv_st + k_spmv_face): FMA rows on the 64 x 16 staged tiles with the
// scalar-dictionary patches, not the fused p update
// vi_st -1: from ST_MIN_NODES owned nodes, or with exception nodes up to a tenth of the owned nodes
// (their rows are listed rows there; the z-march's exception instantiations cost every wave:
// config 5 226.7 vs 236.7 ms per Newton iteration, 128^3 sweep 0.1511 / 0.1689 / 0.2018 vs
// 0.1604 / 0.1671 / 0.2128 ms per CG iteration at 1.6 / 3.1 / 7.0 % exception nodes, 0.3567 vs
// 0.3362 at 25.8 %: profiles/r05s_*, r05t_exc_sweep128.log)
static bool st_auto(const Ctx& c) {
  return c.g.nown >= ST_MIN_NODES || (c.vi_nexc > 0 && c.vi_nexc * 10 <= (int64_t)c.g.nown);
}

bool st_used(const Ctx& c) {
  int tx, ty;
  vis_shape(c, tx, ty);
  return st_wanted(c) && c.st_ok && c.fmt == FMT_VI && c.vi_block && vi_staged(c) && c.vi_fma && c.vi_uni && c.vi_patch &&
         tx == 64 && (!fusep(c) || st_fusep(c));
}

// the fused p update on the default-stencil path: k_spmv_sp's FP instantiation (not k_spmv_st, not the tail)
bool st_fusep(const Ctx& c) { return c.vi_st_pair && !c.vi_st_tail; }

// the default-stencil march is k_spmv_sp (x-pair lanes, 64 x vi_st_ty tiles)
static bool sp_used(const Ctx& c) { return st_used(c) && c.vi_st_pair && !c.vi_st_tail; }

// k_spmv_sp's tiling: 64 x vi_st_ty tiles, z-chunks for one resident round (1024 / (64 ty) blocks per CU)
static ZTiling sp_tiling(const Ctx& c) {
  const int ty = c.vi_st_ty;
  ZTiling t;
  t.ntx = (c.g.nx + 63) / 64;
  t.nty = (c.g.ny + ty - 1) / ty;
  const int tiles = t.ntx * t.nty, want = c.spmv_zblocks > 0 ? c.spmv_zblocks : c.g.ncu * (16 / ty);
  t.nzc = std::max(1, std::min(c.g.nz, (want + tiles - 1) / tiles));
  t.kc = (c.g.nz + t.nzc - 1) / t.nzc;
  t.nzc = (c.g.nz + t.kc - 1) / t.kc;
  return t;
}

// the listed rows 16 lanes per node (st_tail16) while they fill at most half a resident round of the
// device (1,024 threads per CU: 8,192 rows on 256 CUs); beyond that one thread per node (st_tail):
// 16 lanes issue every row's 27 FMAs nine times over, which a long list pays in VALU time.  Measured:
// config 5's few thousand listed rows at 128^3, face kernel 12.0 vs 24.4 us (profiles/r06zb_*);
// 256^3's 6,370, SpMV 0.2635 vs 0.2666 ms, CG iteration 0.7704 vs 0.7735 ms (r06h2_*); 32,768 or
// more exception nodes at 128^3, CG iteration 0.159-0.184 vs 0.142-0.175 ms (r06zc_*, r06zd_*,
// r06h2_*).  Option vi_st_l16: 1 / 0 force, -1 = this rule
static bool st_l16(const Ctx& c) {
  return c.vi_st_l16 > 0 || (c.vi_st_l16 < 0 && (int64_t)ST16 * c.st_n * 2 <= (int64_t)c.g.ncu * 1024);
}

// k_spmv_face's blocks (the face phase and the listed rows as a kernel of their own: vi_st_tail 0)
static int64_t stface_blocks(const Ctx& c) {
  const int lpb = st_l16(c) ? SFP_T / ST16 : SFP_T;
  return st_used(c) && !c.vi_st_tail ? c.st_faces.u[6] + (c.st_n + lpb - 1) / lpb : 0;
}

// the exception rows' kernel (staged block-indexed storage with exception nodes, vi_exc_kernel)
static int64_t exc_blocks(const Ctx& c) {
  if (!(c.fmt == FMT_VI && c.vi_block && c.vi_nexc && vi_staged(c) && c.vi_exc_kernel) || st_used(c)) return 0;
  return (c.vi_nexc + TPB - 1) / TPB;
}

int64_t spmv_nparts(const Ctx& c) {
  if (c.fmt == FMT_SPLIT && c.dsl.dense) return node_blocks(c);
  return spmv_grid_blocks(c) + faces_blocks(c) + exc_blocks(c) + stface_blocks(c);
}

// the SpMV's partial sums (every kernel of one SpMV, the face / listed / exception blocks included)
// and the node-block partials fit one half of the partials buffer: the fused update kernels read
// the SpMV's half while they write the other (partials2), so an SpMV spilling past the half would
// corrupt the p.Ap / z.r sums
bool partials_fit(const Ctx& c) {
  return std::max(spmv_nparts(c), node_blocks(c)) + 32 <= c.partials_cap / 2;
}

bool st_wanted(const Ctx& c) { return c.vi_st == 1 || (c.vi_st < 0 && st_auto(c)); }

int upload_constants(Ctx& c) {
  double B[8][6][24];
  compute_B_table(B);
  MCX_HIP(hipMemcpyToSymbol(HIP_SYMBOL(cB), B, sizeof(B)));
  return 0;
}

void launch_apply_bc_u(Ctx& c, double U) {
  hipLaunchKernelGGL(k_apply_bc_u, dim3(nblk(c.g.nown)), dim3(TPB), 0, c.stream, c.g, c.u_pad, U);
}

void launch_strains(Ctx& c) {
  hipLaunchKernelGGL(k_strains, dim3(nblk(c.g.nelem)), dim3(TPB), 0, c.stream, c.g, c.u_pad, c.eps);
}

void launch_homogenize(Ctx& c) {
  int64_t ngp = 8 * c.g.nelem;
  if (c.mat.law == MCX_LAW_PLASTIC)
    hipLaunchKernelGGL(k_homogenize_plastic, dim3(nblk(ngp)), dim3(TPB), 0, c.stream, ngp, c.mat, c.eps, c.hist_old,
                       c.sig, c.ctan, c.hist_new, c.ftrial);
  else if (c.mat.law == MCX_LAW_ELASTIC)
    hipLaunchKernelGGL(k_homogenize_elastic, dim3(nblk(ngp)), dim3(TPB), 0, c.stream, ngp, c.mat, c.eps, c.sig);
}

void launch_residual(Ctx& c) {
  hipLaunchKernelGGL(k_residual, dim3(nblk(c.g.nown)), dim3(TPB), 0, c.stream, c.g, c.sig, c.b, c.partials);
}

// every law but the isotropic elastic one hands over a per-GP tangent (ctan)
static bool table_law(const Ctx& c) { return c.mat.law != MCX_LAW_ELASTIC; }
// the element matrices matrix_block reads: per element (table laws) or the elastic law's one
static const double* ke_src(const Ctx& c) { return table_law(c) ? c.Ke : c.ke_uni; }

void launch_elastic_ke(Ctx& c) { hipLaunchKernelGGL(k_elastic_ke, dim3(1), dim3(64), 0, c.stream, c.g, c.mat, c.ke_uni); }

// element matrices of a per-GP-tangent law (k_element_ke), read by the gathers below
void launch_element_ke(Ctx& c) {
  const int64_t ngroups = nblk(c.g.nelem);
  const int64_t blocks = pad8(ngroups) * 16;
  hipLaunchKernelGGL(k_element_ke, dim3((unsigned)blocks), dim3(TPB), 0, c.stream, c.g, c.ctan, c.Ke, ngroups,
                     (const unsigned char*)nullptr);
}

// a per-GP-tangent law headed for the value-indexed storage with exception nodes: the plain
// elements (every tangent = the reference tangent), the reference element matrix kref, and the
// element matrices of the other elements only
int launch_plain_ke(Ctx& c) {
  if (!c.elem_plain) {
    MCX_HIP(hipMalloc(&c.elem_plain, c.g.nelem));
    MCX_HIP(hipMalloc(&c.cref, (36 + 36 * 8 + 576) * sizeof(double)));  // cref, cref8, kref
    MCX_HIP(hipMalloc(&c.vi_xslot, c.g.nown * sizeof(unsigned)));
    MCX_HIP(hipMalloc(&c.vi_xlist, c.g.nown * sizeof(int)));
    MCX_HIP(hipMalloc(&c.vi_xcnt, (node_blocks(c) + 1) * sizeof(unsigned)));
    c.device_bytes += c.g.nelem + (36 + 288 + 576) * 8 + c.g.nown * 8 + (node_blocks(c) + 1) * 4;
  }
  double* kref = c.cref + 36 + 288;
  hipLaunchKernelGGL(k_cref, dim3(1), dim3(64), 0, c.stream, c.mat, c.ctan, (int64_t)8 * c.g.nelem, c.cref);
  hipLaunchKernelGGL(k_ref_ke, dim3(1), dim3(64), 0, c.stream, c.g, c.cref + 36, kref);
  hipLaunchKernelGGL(k_elem_plain, dim3(nblk(c.g.nelem)), dim3(TPB), 0, c.stream, c.g, c.ctan, c.cref, c.elem_plain);
  const int64_t ngroups = nblk(c.g.nelem);
  const int64_t blocks = pad8(ngroups) * 16;
  hipLaunchKernelGGL(k_element_ke, dim3((unsigned)blocks), dim3(TPB), 0, c.stream, c.g, c.ctan, c.Ke, ngroups,
                     (const unsigned char*)c.elem_plain);
  c.plain_ke = true;
  return 0;
}

void launch_gather_matrix(Ctx& c) {
  if (table_law(c))
    hipLaunchKernelGGL(k_gather_matrix<true>, dim3(nblk(c.g.nown), 27), dim3(TPB), 0, c.stream, c.g, c.mat, ke_src(c),
                       c.V);
  else
    hipLaunchKernelGGL(k_gather_matrix<false>, dim3(nblk(c.g.nown), 27), dim3(TPB), 0, c.stream, c.g, c.mat, ke_src(c),
                       c.V);
}

void launch_gather_matrix_sym(Ctx& c) {
  const int npad = c.g.PX * c.g.PY * c.g.PZ;
  if (table_law(c))
    hipLaunchKernelGGL(k_gather_matrix_sym<true>, dim3(nblk(npad), 14), dim3(TPB), 0, c.stream, c.g, c.mat, ke_src(c),
                       c.U, npad);
  else
    hipLaunchKernelGGL(k_gather_matrix_sym<false>, dim3(nblk(npad), 14), dim3(TPB), 0, c.stream, c.g, c.mat, ke_src(c),
                       c.U, npad);
}

// exact = the split storage is used (every correction exact and at most split_maxq quads).
// Pass 1 (k_split_mask) finds the active slots and exactness; pass 2 (k_split_pack) recomputes
// the corrections and writes the packed ones, so no per-slot scratch array exists.
int build_split(Ctx& c, bool* exact) {
  MCX_HIP(hipMemsetAsync(c.d_mask, 0, 16 * sizeof(unsigned), c.stream));
  if (c.split_esc && !c.esc_node) {  // per owned node: escape flag, then count << 24 | first + 1
    MCX_HIP(hipMalloc(&c.esc_node, std::max<int64_t>(1, c.g.nown) * sizeof(unsigned)));
    c.device_bytes += c.g.nown * (int64_t)sizeof(unsigned);
  }
  if (c.esc_node) MCX_HIP(hipMemsetAsync(c.esc_node, 0, c.g.nown * sizeof(unsigned), c.stream));
  unsigned* eflag = c.split_esc ? c.esc_node : nullptr;
  const dim3 grid(nblk(c.g.nown), 14);
  if (table_law(c))
    hipLaunchKernelGGL(k_split_mask<true>, grid, dim3(TPB), 0, c.stream, c.g, c.mat, ke_src(c), c.U, c.d_mask, eflag);
  else
    hipLaunchKernelGGL(k_split_mask<false>, grid, dim3(TPB), 0, c.stream, c.g, c.mat, ke_src(c), c.U, c.d_mask, eflag);
  unsigned hm[16];
  MCX_HIP(hipMemcpyAsync(hm, c.d_mask, sizeof(hm), hipMemcpyDeviceToHost, c.stream));
  MCX_HIP(hipStreamSynchronize(c.stream));
  DSlots dl;
  // dense bf16 corrections with escapes: every correction not exact in bf16 is escapable (its
  // truncated bf16 hi plus an exact double residual reconstruct it), dense storage is needed,
  // and the escapes are few (at most one per 16 owned nodes, < 2^24 entries)
  int lbf = 0;
  for (int b = 0; b < 14; b++) lbf += __builtin_popcount(hm[b] & 511u);
  const bool esc = eflag && (hm[14] & 1u) && !(hm[14] & 4u) && !c.split_wide && c.split_dense &&
                   (lbf + 7) / 8 > c.split_maxq && (int64_t)hm[15] <= std::min<int64_t>(c.g.nown / 16 + 64, (1 << 24) - 2);
  *exact = (hm[14] & 2u) == 0 || esc;  // f32 always suffices when bf16 does
  if (!*exact) return 0;
  dl.wide = !esc && ((hm[14] & 1u) || c.split_wide) ? 1 : 0;
  dl.esc = esc ? 1 : 0;
  dl.nesc = esc ? (int)hm[15] : 0;
  for (int b = 0; b < 14; b++) {
    dl.m9[b] = (unsigned short)(hm[b] & 511u);
    dl.pos[b] = (unsigned char)dl.L;
    for (int q = 0; q < 9; q++)
      if (hm[b] >> q & 1) dl.s[dl.L++] = (unsigned char)(b * 9 + q);
  }
  dl.Lq = dl.wide ? (dl.L + 3) / 4 : (dl.L + 7) / 8;
  for (int p = 0; p < std::min(dl.L, 24); p++) {  // the walk's x gather offsets (k_spmv_symp)
    const int s = dl.s[p], nb = s / 9, rc = s - 9 * nb;
    const int off = (nb % 3 - 1) + ((nb / 3) % 3 - 1) * c.g.PX + (nb / 9 - 1) * c.g.PX * c.g.PY;
    dl.xc[p] = (3 * off + rc % 3) * 4 + rc / 3;
  }
  if (dl.Lq > c.split_maxq) {
    // many corrections: the in-kernel walk would take one round trip per slot.  Either store all
    // 120 slots in canonical order and add them in a second streaming pass (k_split_dense), or
    // use the AIJ blocks
    if (!c.split_dense) {
      *exact = false;
      return 0;
    }
    dl.dense = 1;
    dl.L = 0;
    for (int b = 0; b < 14; b++) {
      dl.m9[b] = b < 13 ? 511 : (unsigned short)((1u << 3) | (1u << 6) | (1u << 7));
      dl.pos[b] = (unsigned char)dl.L;
      for (int q = 0; q < 9; q++)
        if (dl.m9[b] >> q & 1) dl.s[dl.L++] = (unsigned char)(b * 9 + q);
    }
    dl.Lq = dl.wide ? (dl.L + 3) / 4 : (dl.L + 7) / 8;
  }
  const int64_t need = std::max<int64_t>(1, c.npgroups * dl.Lq) * 64 * 16;  // bytes of [u/64][Lq][64] x 16 B
  if (need > c.D_bytes) {
    if (c.D) {
      MCX_HIP(hipStreamSynchronize(c.stream));
      MCX_HIP(hipFree(c.D));
      c.device_bytes -= c.D_bytes;
      c.D = nullptr;
    }
    MCX_HIP(hipMalloc(&c.D, need));
    c.D_bytes = need;
    c.device_bytes += need;
  }
  c.dsl = dl;
  if (dl.L) {
    MCX_HIP(hipMemsetAsync(c.D, 0, (size_t)c.npgroups * dl.Lq * 64 * 16, c.stream));
    if (table_law(c))
      hipLaunchKernelGGL(k_split_pack<true>, grid, dim3(TPB), 0, c.stream, c.g, c.mat, ke_src(c), c.U, c.D, dl);
    else
      hipLaunchKernelGGL(k_split_pack<false>, grid, dim3(TPB), 0, c.stream, c.g, c.mat, ke_src(c), c.U, c.D, dl);
  }
  if (dl.esc && dl.nesc) {  // the escapes' residuals, a node's entries contiguous in slot order
    if (dl.nesc > c.esc_cap) {
      if (c.esc_res) {
        MCX_HIP(hipStreamSynchronize(c.stream));
        MCX_HIP(hipFree(c.esc_res));
        MCX_HIP(hipFree(c.esc_slot));
        c.device_bytes -= c.esc_cap * 9;
      }
      c.esc_cap = std::max<int64_t>(dl.nesc, 1024);
      MCX_HIP(hipMalloc(&c.esc_res, c.esc_cap * sizeof(double)));
      MCX_HIP(hipMalloc(&c.esc_slot, c.esc_cap));
      c.device_bytes += c.esc_cap * 9;
    }
    MCX_HIP(hipMemsetAsync(c.d_mask + 15, 0, sizeof(unsigned), c.stream));  // the entries' allocation counter
    if (table_law(c))
      hipLaunchKernelGGL(k_split_esc<true>, dim3(nblk(c.g.nown)), dim3(TPB), 0, c.stream, c.g, c.mat, ke_src(c), c.U,
                         c.esc_node, c.d_mask + 15, (unsigned)c.esc_cap, c.esc_res, c.esc_slot);
    else
      hipLaunchKernelGGL(k_split_esc<false>, dim3(nblk(c.g.nown)), dim3(TPB), 0, c.stream, c.g, c.mat, ke_src(c), c.U,
                         c.esc_node, c.d_mask + 15, (unsigned)c.esc_cap, c.esc_res, c.esc_slot);
    // the escape pass must have placed exactly the escapes the mask pass counted (an
    // overflow leaves a sentinel k_split_dense would misread); otherwise this matrix goes to AIJ
    // blocks (*exact = false)
    unsigned placed = 0;
    MCX_HIP(hipMemcpyAsync(&placed, c.d_mask + 15, sizeof(unsigned), hipMemcpyDeviceToHost, c.stream));
    MCX_HIP(hipStreamSynchronize(c.stream));
    if ((int64_t)placed != dl.nesc) {
      c.dsl.nesc = 0;
      *exact = false;
    }
  }
  return 0;
}

// FMT_VI assembly (see k_vi_collect).  ok = the matrix has at most VI_MAX distinct values; the
// dictionary is the sorted set of their bit patterns, so indices do not depend on the order
// the set was filled in.
// the index array at bytes_per_node x the owned node groups (grown, never shrunk)
static int ensure_vi_idx(Ctx& c, int64_t bytes_per_node) {
  const int64_t need = c.ngroups * 64 * bytes_per_node;
  if (need <= c.vi_idx_bytes) return 0;
  if (c.vi_idx) {
    MCX_HIP(hipStreamSynchronize(c.stream));
    MCX_HIP(hipFree(c.vi_idx));
    c.device_bytes -= c.vi_idx_bytes;
    c.vi_idx = nullptr;
  }
  MCX_HIP(hipMalloc(&c.vi_idx, need));
  c.vi_idx_bytes = need;
  c.device_bytes += need;
  return 0;
}

// single-pass block build (k_vib_build / k_vib_remap); ok = at most VI_MAX distinct blocks and no
// set overflowed.  One host round trip: the sets come back, the dictionary and the position map
// go up from pinned buffers that stay untouched until the next build's readback has synchronised.
static int build_vib(Ctx& c, bool* ok) {
  *ok = false;
  const int64_t nsv = (int64_t)NSLOT * VB_GSV;
  unsigned long long* gsv = c.vib_keys;
  unsigned long long* gbk = c.vib_keys + nsv;
  const int64_t need = (int64_t)27 * c.g.nown * sizeof(unsigned short);
  if (need > c.vib_pos_bytes) {
    if (c.vib_pos) {
      MCX_HIP(hipStreamSynchronize(c.stream));
      MCX_HIP(hipFree(c.vib_pos));
      c.device_bytes -= c.vib_pos_bytes;
      c.vib_pos = nullptr;
    }
    MCX_HIP(hipMalloc(&c.vib_pos, need));
    c.vib_pos_bytes = need;
    c.device_bytes += need;
  }
  MCX_HIP(hipMemsetAsync(c.vib_keys, 0xff, (nsv + VI_HASH) * sizeof(unsigned long long), c.stream));
  MCX_HIP(hipMemsetAsync(c.vib_ctl, 0, 4 * sizeof(unsigned), c.stream));
  const dim3 grid(nblk(c.g.nown), 27);
  // a per-GP-tangent law: the nodes touching a non-plain element become exceptions
  // a per-GP-tangent law (launch_plain_ke ran): the nodes touching a non-plain element become
  // exceptions; every other node's blocks are sums of kref blocks
  const bool exc = table_law(c) && c.plain_ke;
  c.vi_nexc = 0;
  if (exc) {  // ordered compaction: slots in owned-node order
    const unsigned nbn = nblk(c.g.nown);
    hipLaunchKernelGGL(k_exc_flag, dim3(nbn), dim3(TPB), 0, c.stream, c.g, c.elem_plain, c.vi_xslot, c.vi_xcnt);
    hipLaunchKernelGGL(k_exc_scan, dim3(1), dim3(1024), 0, c.stream, c.vi_xcnt, (int)nbn, c.vib_ctl + 2);
    hipLaunchKernelGGL(k_exc_assign, dim3(nbn), dim3(TPB), 0, c.stream, c.g, c.vi_xslot, c.vi_xlist, c.vi_xcnt);
  }
  const unsigned* xslot = exc ? c.vi_xslot : nullptr;
  const double* kref = exc ? c.cref + 36 + 288 : nullptr;
  if (exc)
    hipLaunchKernelGGL(k_vib_build<false>, grid, dim3(TPB), 0, c.stream, c.g, c.mat, kref, gsv, gbk, c.vib_pos,
                       c.vib_ctl, xslot);
  else if (table_law(c))
    hipLaunchKernelGGL(k_vib_build<true>, grid, dim3(TPB), 0, c.stream, c.g, c.mat, ke_src(c), gsv, gbk, c.vib_pos,
                       c.vib_ctl, xslot);
  else
    hipLaunchKernelGGL(k_vib_build<false>, grid, dim3(TPB), 0, c.stream, c.g, c.mat, ke_src(c), gsv, gbk, c.vib_pos,
                       c.vib_ctl, xslot);
  unsigned long long* hk = c.h_vib_keys;
  unsigned* hctl = reinterpret_cast<unsigned*>(hk + nsv + VI_HASH);
  MCX_HIP(hipMemcpyAsync(hk, c.vib_keys, (nsv + VI_HASH) * sizeof(unsigned long long), hipMemcpyDeviceToHost,
                         c.stream));
  MCX_HIP(hipMemcpyAsync(hctl, c.vib_ctl, 4 * sizeof(unsigned), hipMemcpyDeviceToHost, c.stream));
  MCX_HIP(hipStreamSynchronize(c.stream));
  if (hctl[1] || hctl[0] > (unsigned)VI_MAX) return 0;
  const int64_t nexc = exc ? (int64_t)hctl[2] : 0;
  if (nexc * 1000 > (int64_t)c.vi_exc_max * c.g.nown) return 0;  // too many: AIJ-split
  if (nexc > c.g.xld) {
    if (c.vi_exc) {
      MCX_HIP(hipFree(c.vi_exc));
      c.device_bytes -= c.vi_exc_bytes;
      c.vi_exc = nullptr;
    }
    // AoSoA groups of 64 slots (exc_base); grown with headroom (the plastic zone spreads over the
    // time steps)
    c.g.xld = (std::min<int64_t>(2 * nexc + 1024, c.g.nown) + 63) / 64 * 64;
    c.vi_exc_bytes = c.g.xld * 27 * 9 * (int64_t)sizeof(double);
    MCX_HIP(hipMalloc(&c.vi_exc, c.vi_exc_bytes));
    c.device_bytes += c.vi_exc_bytes;
  }
  // each slot's values sorted by bit pattern; rank of every set position
  std::vector<unsigned char> rank(nsv, 0);
  std::vector<unsigned long long> all;
  int maxper = 0;
  for (int S = 0; S < NSLOT; S++) {
    const unsigned long long* ks = hk + (int64_t)S * VB_GSV;
    std::vector<unsigned long long> v;
    for (int h = 0; h < VB_GSV; h++)
      if (ks[h] != VI_EMPTY) v.push_back(ks[h]);
    std::sort(v.begin(), v.end());
    maxper = std::max(maxper, (int)v.size());
    for (int h = 0; h < VB_GSV; h++)
      if (ks[h] != VI_EMPTY) rank[(int64_t)S * VB_GSV + h] = (unsigned char)(std::lower_bound(v.begin(), v.end(), ks[h]) - v.begin());
    all.insert(all.end(), v.begin(), v.end());
  }
  std::sort(all.begin(), all.end());
  const int nvals = (int)(std::unique(all.begin(), all.end()) - all.begin());
  // blocks ordered by (position nb, the 9 values' ranks from slot 8 down to slot 0): with <= 16
  // values per slot this is round 2's key order (nb << 36 | rank nibbles)
  std::vector<std::pair<unsigned long long, int>> blk;  // (order key, set position)
  for (int h = 0; h < VI_HASH; h++) {
    const unsigned long long code = hk[nsv + h];
    if (code == VI_EMPTY) continue;
    const int nb = (int)(code >> 54);
    unsigned long long key = (unsigned long long)nb << 54;
    for (int q = 0; q < 9; q++) {
      const int gp = (int)((code >> (6 * q)) & 63);
      key |= (unsigned long long)rank[(int64_t)(nb * 9 + q) * VB_GSV + gp] << (6 * q);
    }
    blk.push_back({key, h});
  }
  std::sort(blk.begin(), blk.end());
  std::memset(c.h_vib_map, 0, VI_HASH);
  std::memset(c.h_vib_dict, 0, VI_MAX * VIB_STRIDE * sizeof(double));
  for (size_t b = 0; b < blk.size(); b++) {
    const unsigned long long code = hk[nsv + blk[b].second];
    const int nb = (int)(code >> 54);
    c.h_vib_map[blk[b].second] = (unsigned char)b;
    for (int q = 0; q < 9; q++) {
      const unsigned long long bits = hk[(int64_t)(nb * 9 + q) * VB_GSV + ((code >> (6 * q)) & 63)];
      std::memcpy(&c.h_vib_dict[b * VIB_STRIDE + q], &bits, sizeof(double));
    }
  }
  unsigned char* bmap = c.vi_slot + NSLOT * 32;
  MCX_HIP(hipMemcpyAsync(bmap, c.h_vib_map, VI_HASH, hipMemcpyHostToDevice, c.stream));
  MCX_HIP(hipMemcpyAsync(c.vi_bdict, c.h_vib_dict, VI_MAX * VIB_STRIDE * sizeof(double), hipMemcpyHostToDevice,
                         c.stream));
  if (int rc = ensure_vi_idx(c, 32)) return rc;
  hipLaunchKernelGGL(k_vib_remap, dim3(nblk(c.g.nown)), dim3(TPB), 0, c.stream, c.g, c.vib_pos, bmap,
                     reinterpret_cast<u32x4*>(c.vi_idx), xslot);
  if (nexc) {
    const dim3 eg((unsigned)((nexc + TPB - 1) / TPB), 27);
    hipLaunchKernelGGL(k_exc_fill, eg, dim3(TPB), 0, c.stream, c.g, c.mat, ke_src(c), kref, c.elem_plain,
                       c.vi_xlist, nexc, c.vi_exc);
  }
  c.vi_nexc = nexc;
  c.vi_n = nvals;
  c.vi_bits = maxper <= 16 ? 4 : 8;
  c.vi_nblocks = (int)blk.size();
  c.vi_block = true;
  *ok = true;
  return 0;
}

// Wave descriptors of the block-indexed storage (k_spmv_vibm WD): one per 16 x 4 node patch and
// plane (the node set of one wave of the staged SpMV, whatever the tile shape), 32 words: flags
// (bit 0: the 64 nodes are in the domain, not exception nodes, with the same 27 block indices;
// bit 1: each has all 27 neighbours; bit 2: not uniform, but every node holds one of two index
// sets), the patch's first node's 7 index words (set A), set B's 7 words, and the lane mask of
// set B.  Such a wave then reads its block indices from this descriptor (one coalesced 128-B load,
// scalar registers by v_readlane) instead of 32 B per node: a uniform wave runs the
// scalar-dictionary pass once, a two-set wave (an x- or y-face column or row in a patch: FMA
// rows) once per set under the set's exec mask; the others load their nodes' words as before.
// ctr[0..2] count the present blocks of the nodes in waves that still read per-lane words (FMA
// rows with uniform waves only / exact rows / FMA rows with two-set waves).
__global__ __launch_bounds__(TPB) void k_vi_wdesc(Geo g, const u32x4* __restrict__ I, unsigned* __restrict__ D,
                                                  int npx, int npy, unsigned long long* __restrict__ ctr) {
  const int64_t w = (int64_t)blockIdx.x * (TPB / 64) + (threadIdx.x >> 6);
  const int ln = threadIdx.x & 63;
  if (w >= (int64_t)npx * npy * g.nz) return;  // (whole wave)
  const int px = (int)(w % npx);
  const int64_t r = w / npx;
  const int py = (int)(r % npy), k = (int)(r / npy);
  const int i = px * 16 + (ln & 15), j = py * 4 + (ln >> 4);
  const bool inxy = i < g.nx && j < g.ny;
  u32x4 w0 = {0u, 0u, 0u, 0u}, w1 = w0;
  unsigned pres = 0u;
  if (inxy) {
    const int64_t n = i + g.nx * (j + (int64_t)g.ny * k);
    const u32x4* ip = I + (n >> 6) * (2 * 64) + (n & 63);
    w0 = ip[0];
    w1 = ip[64];
    pres = present_mask(g, i, j, k);
  }
  unsigned sw[7], sb[7], diff = 0u;
#pragma unroll
  for (int q = 0; q < 7; q++) {
    const unsigned v = q < 4 ? w0[q] : w1[q - 4];
    sw[q] = __builtin_amdgcn_readfirstlane(v);
    diff |= v ^ sw[q];
  }
  const bool ina = inxy && diff == 0u && w1[3] == 0u;
  const bool uni = __all(ina);
  const bool full = __all(inxy && pres == PRES_ALL);
  // set B: the first lane outside set A
  const unsigned long long oa = __ballot(!ina);
  const int lb = oa ? __builtin_ctzll(oa) : 0;
  unsigned db = 0u;
#pragma unroll
  for (int q = 0; q < 7; q++) {
    const unsigned v = q < 4 ? w0[q] : w1[q - 4];
    sb[q] = (unsigned)__builtin_amdgcn_readlane((int)v, lb);
    db |= v ^ sb[q];
  }
  const bool inb = !ina && inxy && db == 0u && w1[3] == 0u;
  const bool two = !uni && __all(ina || inb);
  const unsigned long long mb = __ballot(inb);
  if (ln < 32) {
    unsigned v = (uni ? 1u : 0u) | (full ? 2u : 0u) | (two ? 4u : 0u);
#pragma unroll
    for (int q = 0; q < 7; q++) {
      if (ln == q + 1) v = sw[q];
      if (ln == q + 8) v = two ? sb[q] : 0u;
    }
    if (ln == 15) v = 0u;
    if (ln == 16) v = two ? (unsigned)mb : 0u;
    if (ln == 17) v = two ? (unsigned)(mb >> 32) : 0u;
    if (ln > 17) v = 0u;
    D[(w << 5) + ln] = v;
  }
  const double nbl = wave_sum((double)__popc(pres));
  if (ln == 0) {
    if (!uni) atomicAdd(&ctr[0], (unsigned long long)nbl);
    if (!(uni && full)) atomicAdd(&ctr[1], (unsigned long long)nbl);
    if (!uni && !two) atomicAdd(&ctr[2], (unsigned long long)nbl);
  }
}

int build_wdesc(Ctx& c) {
  c.wd_ok = false;
  if (!(c.fmt == FMT_VI && c.vi_block)) return 0;
  const int npx = (c.g.nx + 15) / 16, npy = (c.g.ny + 3) / 4;
  const int64_t nw = (int64_t)npx * npy * c.g.nz;
  const int64_t bytes = nw * 32 * sizeof(unsigned) + 3 * sizeof(unsigned long long);
  if (bytes > c.wd_bytes) {
    if (c.wd) {
      MCX_HIP(hipFree(c.wd));
      c.device_bytes -= c.wd_bytes;
      c.wd = nullptr;
    }
    MCX_HIP(hipMalloc(&c.wd, bytes));
    c.wd_bytes = bytes;
    c.device_bytes += bytes;
  }
  unsigned long long* ctr = reinterpret_cast<unsigned long long*>(c.wd + nw * 32);
  MCX_HIP(hipMemsetAsync(ctr, 0, 3 * sizeof(unsigned long long), c.stream));
  hipLaunchKernelGGL(k_vi_wdesc, dim3((unsigned)((nw + TPB / 64 - 1) / (TPB / 64))), dim3(TPB), 0, c.stream, c.g,
                     reinterpret_cast<const u32x4*>(c.vi_idx), c.wd, npx, npy, ctr);
  unsigned long long h[3];
  MCX_HIP(hipMemcpyAsync(h, ctr, sizeof(h), hipMemcpyDeviceToHost, c.stream));
  MCX_HIP(hipStreamSynchronize(c.stream));
  c.wd_npx = npx;
  c.wd_npy = npy;
  c.wd_blocks_fma = (int64_t)h[0];
  c.wd_blocks_exact = (int64_t)h[1];
  c.wd_blocks_two = (int64_t)h[2];
  c.wd_ok = true;
  return 0;
}

// default-stencil structures (k_spmv_st): the stencil of the middle node, the list of the other
// nodes (ordered compaction), the patch masks; one host round trip for the list's length
// Built lazily: only when the SpMV would take the path (vi_st 1, or -1 by size); else
// marked pending, and the vi_st option handler builds them when it turns the path on.
int build_st(Ctx& c) {
  c.st_ok = false;
  c.st_pending = false;
  if (!(c.fmt == FMT_VI && c.vi_block && vi_staged(c) && c.g.nown > 0)) return 0;
  if (!st_wanted(c)) {
    c.st_pending = true;
    return 0;
  }
  const int npx = (c.g.nx + 15) / 16, npy = (c.g.ny + 3) / 4;
  const int64_t nwp = (int64_t)npx * npy * c.g.nz;
  if (!c.st_coef) {
    MCX_HIP(hipMalloc(&c.st_coef, ST_CLASSES * 27 * VIB_STRIDE * sizeof(double)));
    MCX_HIP(hipMalloc(&c.st_ids, ST_CLASSES * 8 * sizeof(unsigned)));
    MCX_HIP(hipMalloc(&c.st_slot, c.g.nown * sizeof(unsigned)));
    MCX_HIP(hipMalloc(&c.st_list, c.g.nown * sizeof(int)));
    MCX_HIP(hipMalloc(&c.st_cnt, (node_blocks(c) + 1) * sizeof(unsigned)));
    c.device_bytes += ST_CLASSES * (27 * VIB_STRIDE * 8 + 32) + c.g.nown * 8 + (node_blocks(c) + 1) * 4;
  }
  if (nwp * 8 > c.st_mask_bytes) {
    if (c.st_mask) {
      MCX_HIP(hipFree(c.st_mask));
      c.device_bytes -= c.st_mask_bytes;
    }
    MCX_HIP(hipMalloc(&c.st_mask, nwp * 8));
    c.st_mask_bytes = nwp * 8;
    c.device_bytes += c.st_mask_bytes;
  }
  const u32x4* I = reinterpret_cast<const u32x4*>(c.vi_idx);
  const unsigned nbn = nblk(c.g.nown);
  hipLaunchKernelGGL(k_st_setup, dim3(ST_CLASSES), dim3(320), 0, c.stream, c.g, I, c.vi_bdict, c.st_coef, c.st_ids,
                     c.vi_st_faces == 1 ? 0x7e : c.vi_st_faces);
  hipLaunchKernelGGL(k_st_flag, dim3(nbn), dim3(TPB), 0, c.stream, c.g, I, c.st_ids, c.st_slot, c.st_cnt);
  hipLaunchKernelGGL(k_exc_scan, dim3(1), dim3(1024), 0, c.stream, c.st_cnt, (int)nbn, c.st_cnt + nbn);
  hipLaunchKernelGGL(k_exc_assign, dim3(nbn), dim3(TPB), 0, c.stream, c.g, c.st_slot, c.st_list, c.st_cnt);
  hipLaunchKernelGGL(k_st_mask, dim3((unsigned)((nwp + TPB / 64 - 1) / (TPB / 64))), dim3(TPB), 0, c.stream, c.g,
                     c.st_slot, c.st_mask, npx, npy);
  unsigned h[1 + 8 * ST_CLASSES] = {};
  MCX_HIP(hipMemcpyAsync(&h[0], c.st_cnt + nbn, sizeof(unsigned), hipMemcpyDeviceToHost, c.stream));
  MCX_HIP(hipMemcpyAsync(&h[1], c.st_ids, 8 * ST_CLASSES * sizeof(unsigned), hipMemcpyDeviceToHost, c.stream));
  MCX_HIP(hipStreamSynchronize(c.stream));
  c.st_n = h[0];
  c.st_npx = npx;
  c.st_npy = npy;
  c.st_fm = 0;
  for (int k = 0; k < ST_CLASSES; k++) c.st_fm |= (h[1 + 8 * k + 7] != 0u) << k;
  c.st_ok = c.st_fm & 1u;  // no interior representative (exception nodes): no default stencil
  // the face phase's patches: class q's face (if usable) in patches of 64 x SFP_S nodes (fast x slow axis)
  const Geo& g = c.g;
  const bool on[7] = {false, g.xs == 0, g.xs + g.nx == g.NX, g.ys == 0, g.ys + g.ny == g.NY, g.zs == 0, g.zs + g.nz == g.NZ};
  c.st_faces.u[0] = 0;
  for (int q = 1; q < ST_CLASSES; q++) {
    const int ax = (q - 1) >> 1;
    const int nfast = ax == 0 ? g.ny : g.nx, nslow = ax == 2 ? g.ny : g.nz;
    const bool use = on[q] && ((c.st_fm >> q) & 1u) && !(ax == 0 && g.nx == 1 && q == 2) &&
                     !(ax == 1 && g.ny == 1 && q == 4) && !(ax == 2 && g.nz == 1 && q == 6);
    c.st_faces.u[q] = c.st_faces.u[q - 1] + (use ? (int64_t)((nfast + 63) / 64) * ((nslow + SFP_S - 1) / SFP_S) : 0);
  }
  if (c.st_ok && !partials_fit(c)) c.st_ok = false;  // its partials would spill into partials2: k_spmv_vibm
  return 0;
}

// the staged SpMV reads the wave descriptors (option vi_wdesc): block-indexed storage without
// exception nodes, scalar-dictionary patches, not the fused p update
bool wd_used(const Ctx& c) {
  return c.vi_wdesc && c.wd_ok && c.fmt == FMT_VI && c.vi_block && !c.vi_nexc && c.vi_uni && c.vi_patch &&
         vi_staged(c) && !fusep(c);
}

int build_vi(Ctx& c, bool* ok) {
  *ok = false;
  if (c.vi_block_on && c.vi_bits_max == 4 && c.vib_onepass) {
    if (int rc = build_vib(c, ok)) return rc;
    if (*ok || c.plain_ke) return 0;  // (plain_ke: Ke holds the non-plain elements only)
  }
  const bool table = table_law(c);
  MCX_HIP(hipMemsetAsync(c.vi_keys, 0xff, (VI_HASH + NSLOT * 32) * sizeof(unsigned long long), c.stream));
  MCX_HIP(hipMemsetAsync(c.vi_ctl, 0, (3 + NSLOT) * sizeof(unsigned), c.stream));
  unsigned long long* skeys = c.vi_keys + VI_HASH;
  const dim3 grid(nblk(c.g.nown), 27);
  if (table)
    hipLaunchKernelGGL(k_vi_collect<true>, grid, dim3(TPB), 0, c.stream, c.g, c.mat, ke_src(c), c.vi_keys, skeys, c.vi_ctl);
  else
    hipLaunchKernelGGL(k_vi_collect<false>, grid, dim3(TPB), 0, c.stream, c.g, c.mat, ke_src(c), c.vi_keys, skeys, c.vi_ctl);
  std::vector<unsigned> ctl(3 + NSLOT);
  std::vector<unsigned long long> keys(VI_HASH + NSLOT * 32);
  MCX_HIP(hipMemcpyAsync(ctl.data(), c.vi_ctl, ctl.size() * sizeof(unsigned), hipMemcpyDeviceToHost, c.stream));
  MCX_HIP(hipMemcpyAsync(keys.data(), c.vi_keys, keys.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost,
                         c.stream));
  MCX_HIP(hipStreamSynchronize(c.stream));
  if (ctl[1] || ctl[0] > (unsigned)VI_MAX) return 0;
  const int bits = (!ctl[2] && c.vi_bits_max == 4) ? 4 : 8;
  // dictionaries: sorted bit patterns (the whole matrix's, or each slot's), and the index of
  // every occupied set entry
  const int nsets = bits == 8 ? 1 : NSLOT, ssize = bits == 8 ? VI_HASH : 32, dsize = bits == 8 ? VI_MAX : 16;
  const unsigned long long* kk = bits == 8 ? keys.data() : keys.data() + VI_HASH;
  std::vector<unsigned char> slot(nsets * ssize, 0);
  std::vector<double> dict(nsets * dsize, 0.);
  for (int st = 0; st < nsets; st++) {
    std::vector<unsigned long long> vals;
    for (int h = 0; h < ssize; h++)
      if (kk[st * ssize + h] != VI_EMPTY) vals.push_back(kk[st * ssize + h]);
    std::sort(vals.begin(), vals.end());
    for (int h = 0; h < ssize; h++)
      if (kk[st * ssize + h] != VI_EMPTY)
        slot[st * ssize + h] =
            (unsigned char)(std::lower_bound(vals.begin(), vals.end(), kk[st * ssize + h]) - vals.begin());
    for (size_t q = 0; q < vals.size(); q++) std::memcpy(&dict[st * dsize + q], &vals[q], sizeof(double));
  }
  MCX_HIP(hipMemcpyAsync(c.vi_slot, slot.data(), slot.size(), hipMemcpyHostToDevice, c.stream));
  MCX_HIP(hipMemcpyAsync(c.vi_dict, dict.data(), dict.size() * sizeof(double), hipMemcpyHostToDevice, c.stream));
  c.vi_block = false;
  if (bits == 4 && c.vi_block_on && !c.vib_onepass) {  // one byte per 3x3 block when the blocks are few (k_vib_collect)
    unsigned long long* bkeys = c.vi_keys + VI_HASH + NSLOT * 32;
    unsigned char* bmap = c.vi_slot + NSLOT * 32;
    unsigned* bctl = c.vi_ctl + 3 + NSLOT;
    MCX_HIP(hipMemsetAsync(bkeys, 0xff, VI_HASH * sizeof(unsigned long long), c.stream));
    MCX_HIP(hipMemsetAsync(bctl, 0, 2 * sizeof(unsigned), c.stream));
    if (table)
      hipLaunchKernelGGL(k_vib_collect<true>, grid, dim3(TPB), 0, c.stream, c.g, c.mat, ke_src(c), skeys, c.vi_slot, bkeys,
                         bctl);
    else
      hipLaunchKernelGGL(k_vib_collect<false>, grid, dim3(TPB), 0, c.stream, c.g, c.mat, ke_src(c), skeys, c.vi_slot, bkeys,
                         bctl);
    unsigned bc[2];
    std::vector<unsigned long long> bk(VI_HASH);
    MCX_HIP(hipMemcpyAsync(bc, bctl, sizeof(bc), hipMemcpyDeviceToHost, c.stream));
    MCX_HIP(hipMemcpyAsync(bk.data(), bkeys, VI_HASH * sizeof(unsigned long long), hipMemcpyDeviceToHost, c.stream));
    MCX_HIP(hipStreamSynchronize(c.stream));
    if (!bc[1] && bc[0] <= (unsigned)VI_MAX) {
      std::vector<unsigned long long> bv;
      for (unsigned long long k : bk)
        if (k != VI_EMPTY) bv.push_back(k);
      std::sort(bv.begin(), bv.end());
      std::vector<unsigned char> bm(VI_HASH, 0);
      for (int h = 0; h < VI_HASH; h++)
        if (bk[h] != VI_EMPTY) bm[h] = (unsigned char)(std::lower_bound(bv.begin(), bv.end(), bk[h]) - bv.begin());
      std::vector<double> bd((size_t)VI_MAX * VIB_STRIDE, 0.);
      for (size_t b = 0; b < bv.size(); b++) {
        const int nb = (int)(bv[b] >> 36);
        for (int q = 0; q < 9; q++) bd[b * VIB_STRIDE + q] = dict[(nb * 9 + q) * 16 + ((bv[b] >> (4 * q)) & 15)];
      }
      MCX_HIP(hipMemcpyAsync(bmap, bm.data(), VI_HASH, hipMemcpyHostToDevice, c.stream));
      MCX_HIP(hipMemcpyAsync(c.vi_bdict, bd.data(), bd.size() * sizeof(double), hipMemcpyHostToDevice, c.stream));
      if (int rc = ensure_vi_idx(c, 32)) return rc;
      if (table)
        hipLaunchKernelGGL(k_vib_pack<true>, grid, dim3(TPB), 0, c.stream, c.g, c.mat, ke_src(c), skeys, c.vi_slot, bkeys,
                           bmap, c.vi_idx);
      else
        hipLaunchKernelGGL(k_vib_pack<false>, grid, dim3(TPB), 0, c.stream, c.g, c.mat, ke_src(c), skeys, c.vi_slot, bkeys,
                           bmap, c.vi_idx);
      MCX_HIP(hipStreamSynchronize(c.stream));
      c.vi_n = (int)ctl[0];
      c.vi_bits = 4;
      c.vi_nblocks = (int)bv.size();
      c.vi_block = true;
      *ok = true;
      return 0;
    }
  }
  if (int rc = ensure_vi_idx(c, bits == 8 ? 256 : 128)) return rc;
  u32x4* I = reinterpret_cast<u32x4*>(c.vi_idx);
  const dim3 pg(nblk(c.g.nown));
  if (bits == 8 && table)
    hipLaunchKernelGGL((k_vi_pack<true, 8>), pg, dim3(TPB), 0, c.stream, c.g, c.mat, ke_src(c), c.vi_keys, c.vi_slot, I);
  else if (bits == 8)
    hipLaunchKernelGGL((k_vi_pack<false, 8>), pg, dim3(TPB), 0, c.stream, c.g, c.mat, ke_src(c), c.vi_keys, c.vi_slot, I);
  else if (table)
    hipLaunchKernelGGL((k_vi_pack<true, 4>), pg, dim3(TPB), 0, c.stream, c.g, c.mat, ke_src(c), skeys, c.vi_slot, I);
  else
    hipLaunchKernelGGL((k_vi_pack<false, 4>), pg, dim3(TPB), 0, c.stream, c.g, c.mat, ke_src(c), skeys, c.vi_slot, I);
  // the host copies above must outlive the async uploads
  MCX_HIP(hipStreamSynchronize(c.stream));
  c.vi_n = (int)ctl[0];
  c.vi_bits = bits;
  *ok = true;
  return 0;
}

void launch_jacobi(Ctx& c) {
  if (c.fmt == FMT_VI && c.vi_block)
  {
    hipLaunchKernelGGL(k_jacobi_vib, dim3(nblk(c.g.nown)), dim3(TPB), 0, c.stream, c.g, c.vi_idx, c.vi_bdict, c.dinv,
                       c.jix, c.vi_nexc ? c.vi_exc : nullptr);
    hipLaunchKernelGGL(k_jacobi_vib_dict, dim3(nblk(3 * VI_MAX)), dim3(TPB), 0, c.stream, c.vi_bdict, c.jdd);
  } else if (c.fmt == FMT_VI && c.vi_bits == 4)
    hipLaunchKernelGGL(k_jacobi_vi<4>, dim3(nblk(c.g.nown)), dim3(TPB), 0, c.stream, c.g,
                       reinterpret_cast<const u32x4*>(c.vi_idx), c.vi_dict, c.dinv);
  else if (c.fmt == FMT_VI)
    hipLaunchKernelGGL(k_jacobi_vi<8>, dim3(nblk(c.g.nown)), dim3(TPB), 0, c.stream, c.g,
                       reinterpret_cast<const u32x4*>(c.vi_idx), c.vi_dict, c.dinv);
  else if (c.fmt != FMT_V)
    hipLaunchKernelGGL(k_jacobi_sym, dim3(nblk(c.g.nown)), dim3(TPB), 0, c.stream, c.g, c.U, c.dinv);
  else
    hipLaunchKernelGGL(k_jacobi, dim3(nblk(c.g.nown)), dim3(TPB), 0, c.stream, c.g, c.V, c.dinv);
}

template <int NIB>
static void launch_spmv_vi(Ctx& c, const double* xpad, double* y, bool dot, bool gated, int nb, const SpmvTiling& tl) {
  const u32x4* I = reinterpret_cast<const u32x4*>(c.vi_idx);
  if (NIB == 4 && vi_staged(c)) {  // x staged in LDS, 1024-node tiles marching z-chunks
    const ZTiling zt = vis_tiling(c);
    int tx, ty;
    vis_shape(c, tx, ty);
#define MCX_VIS(TXV, TYV)                                                                                            \
  do {                                                                                                              \
    if (dot && gated)                                                                                               \
      hipLaunchKernelGGL((k_spmv_vim<true, true, TXV, TYV, NIB>), dim3(nb), dim3(1024), 0, c.stream, c.g, I,         \
                         c.vi_dict, xpad, y, c.partials, c.cg, zt);                                                 \
    else if (dot)                                                                                                   \
      hipLaunchKernelGGL((k_spmv_vim<true, false, TXV, TYV, NIB>), dim3(nb), dim3(1024), 0, c.stream, c.g, I,        \
                         c.vi_dict, xpad, y, c.partials, c.cg, zt);                                                 \
    else                                                                                                            \
      hipLaunchKernelGGL((k_spmv_vim<false, false, TXV, TYV, NIB>), dim3(nb), dim3(1024), 0, c.stream, c.g, I,       \
                         c.vi_dict, xpad, y, c.partials, c.cg, zt);                                                 \
  } while (0)
    if constexpr (NIB == 4) {
      if (tx == 256) MCX_VIS(256, 4);
      else if (tx == 128) MCX_VIS(128, 8);
      else MCX_VIS(64, 16);
    }
#undef MCX_VIS
    return;
  }
  if (c.split_dbg) {  // timing-only diagnostics of the gathered kernel (wrong products)
    if (c.split_dbg == 1)
      hipLaunchKernelGGL((k_spmv_vi<false, false, NIB, 1>), dim3(nb), dim3(TPB), 0, c.stream, c.g, I, c.vi_dict, xpad,
                         y, c.partials, c.cg, tl);
    else if (c.split_dbg == 2)
      hipLaunchKernelGGL((k_spmv_vi<false, false, NIB, 2>), dim3(nb), dim3(TPB), 0, c.stream, c.g, I, c.vi_dict, xpad,
                         y, c.partials, c.cg, tl);
    else
      hipLaunchKernelGGL((k_spmv_vi<false, false, NIB, 3>), dim3(nb), dim3(TPB), 0, c.stream, c.g, I, c.vi_dict, xpad,
                         y, c.partials, c.cg, tl);
    return;
  }
  if (dot && gated)
    hipLaunchKernelGGL((k_spmv_vi<true, true, NIB>), dim3(nb), dim3(TPB), 0, c.stream, c.g, I, c.vi_dict, xpad, y,
                       c.partials, c.cg, tl);
  else if (dot)
    hipLaunchKernelGGL((k_spmv_vi<true, false, NIB>), dim3(nb), dim3(TPB), 0, c.stream, c.g, I, c.vi_dict, xpad, y,
                       c.partials, c.cg, tl);
  else
    hipLaunchKernelGGL((k_spmv_vi<false, false, NIB>), dim3(nb), dim3(TPB), 0, c.stream, c.g, I, c.vi_dict, xpad, y,
                       c.partials, c.cg, tl);
}

// the CG iteration's p update fused into the value-indexed SpMV (FP, see FusedP): single rank,
// block-indexed storage with x staged, Jacobi from the diagonal index, scalar-dictionary patches
bool fusep(const Ctx& c) {
  return c.cg_fusep && c.vi_fma && c.p_pad2 && c.nranks == 1 && !c.comm && !c.lg && c.fmt == FMT_VI && c.vi_block &&
         !c.vi_nexc && vi_staged(c) && c.cg_dix && c.vi_uni && c.vi_patch;
}

static void launch_spmv_fusep(Ctx& c, double* y) {
  const int nb = (int)spmv_grid_blocks(c);
  const u32x4* I = reinterpret_cast<const u32x4*>(c.vi_idx);
  ZTiling zt = vis_tiling(c);
  int tx, ty;
  vis_shape(c, tx, ty);
  FusedP fp;
  fp.r = c.r;
  fp.jdd = c.jdd;
  fp.jix = c.jix;
  fp.pb[0] = c.p_pad;
  fp.pb[1] = c.p_pad2;
  if (st_used(c)) {  // the default-stencil march with the p update (k_spmv_sp FP), then the faces and
                     // listed rows from p's buffer of this iteration (the host's count cg_it is the
                     // device's cg->i for every iteration that runs; finished ones return at once)
    zt = sp_tiling(c);
    if (c.vi_st_ty == 16)
      hipLaunchKernelGGL((k_spmv_sp<true, true, 16, true>), dim3(nb), dim3(1024), 0, c.stream, c.g, c.st_coef,
                         c.st_mask, c.st_npx, c.st_npy, nullptr, y, c.partials, c.cg, zt, fp);
    else
      hipLaunchKernelGGL((k_spmv_sp<true, true, 8, true>), dim3(nb), dim3(512), 0, c.stream, c.g, c.st_coef,
                         c.st_mask, c.st_npx, c.st_npy, nullptr, y, c.partials, c.cg, zt, fp);
    const int64_t nbfa = stface_blocks(c);
    if (nbfa && !st_l16(c))
      hipLaunchKernelGGL((k_spmv_face<true, true, false>), dim3((unsigned)nbfa), dim3(SFP_T), 0, c.stream, c.g,
                         c.st_faces, c.st_coef, c.st_slot, c.cg_it & 1 ? c.p_pad2 : c.p_pad, y, c.partials + nb, c.cg,
                         c.st_list, c.st_n, I, c.vi_bdict, c.vi_exc);
    else if (nbfa)
      hipLaunchKernelGGL((k_spmv_face<true, true>), dim3((unsigned)nbfa), dim3(SFP_T), 0, c.stream, c.g, c.st_faces,
                         c.st_coef, c.st_slot, c.cg_it & 1 ? c.p_pad2 : c.p_pad, y, c.partials + nb, c.cg, c.st_list,
                         c.st_n, I, c.vi_bdict, c.vi_exc);
    return;
  }
#define MCX_VIBM_FP(TXV, TYV, FV)                                                                                   \
  hipLaunchKernelGGL((k_spmv_vibm<true, true, TXV, TYV, true, true, true, FV, true>), dim3(nb), dim3(1024), 0,        \
                     c.stream, c.g, I, c.vi_bdict, c.p_pad, y, c.partials, c.cg, zt, fp)
  if (c.vi_fma) {
    if (tx == 256) MCX_VIBM_FP(256, 4, true);
    else if (tx == 128) MCX_VIBM_FP(128, 8, true);
    else MCX_VIBM_FP(64, 16, true);
  } else {
    if (tx == 256) MCX_VIBM_FP(256, 4, false);
    else if (tx == 128) MCX_VIBM_FP(128, 8, false);
    else MCX_VIBM_FP(64, 16, false);
  }
#undef MCX_VIBM_FP
}

// the face kernel on a stream of its own beside the march (option vi_st_fstream): the march holds
// one 1,024-thread block per CU at 104 VGPRs and 115 KB of LDS, which leaves room for one
// 256-thread face block (96 VGPRs, 28.5 KB) per CU in the march's idle issue slots.  The stream and
// its two events are made on first use; any failure keeps the faces on the compute stream.
static bool fstream_ok(Ctx& c) {
  if (!c.vi_st_fstream) return false;
  if (!c.f_stream && hipStreamCreateWithFlags(&c.f_stream, hipStreamNonBlocking) != hipSuccess) {
    c.f_stream = nullptr;
    c.vi_st_fstream = 0;
    return false;
  }
  for (hipEvent_t* e : {&c.ev_fx, &c.ev_fd})
    if (!*e && hipEventCreateWithFlags(e, hipEventDisableTiming) != hipSuccess) {
      *e = nullptr;
      c.vi_st_fstream = 0;
      return false;
    }
  return true;
}

// k_spmv_sp's timing-only diagnostic instantiations (option split_dbg; wrong products, see DBG)
template <bool DV, bool GV, int D>
static void sp_dbg1(Ctx& c, int nb, const double* xpad, double* y, const ZTiling& zt) {
  if (c.vi_st_ty == 16)
    hipLaunchKernelGGL((k_spmv_sp<DV, GV, 16, false, D>), dim3(nb), dim3(1024), 0, c.stream, c.g, c.st_coef,
                       c.st_mask, c.st_npx, c.st_npy, xpad, y, c.partials, c.cg, zt);
  else
    hipLaunchKernelGGL((k_spmv_sp<DV, GV, 8, false, D>), dim3(nb), dim3(512), 0, c.stream, c.g, c.st_coef,
                       c.st_mask, c.st_npx, c.st_npy, xpad, y, c.partials, c.cg, zt);
}
template <bool DV, bool GV>
static void sp_dbg(Ctx& c, int nb, const double* xpad, double* y, const ZTiling& zt) {
  switch (zt.dbg) {
    case 1: sp_dbg1<DV, GV, 1>(c, nb, xpad, y, zt); break;
    case 2: sp_dbg1<DV, GV, 2>(c, nb, xpad, y, zt); break;
    case 3: sp_dbg1<DV, GV, 3>(c, nb, xpad, y, zt); break;
    case 4: sp_dbg1<DV, GV, 4>(c, nb, xpad, y, zt); break;
    case 8: sp_dbg1<DV, GV, 8>(c, nb, xpad, y, zt); break;
    case 12: sp_dbg1<DV, GV, 12>(c, nb, xpad, y, zt); break;
    case 44: sp_dbg1<DV, GV, 44>(c, nb, xpad, y, zt); break;
    case 1024: sp_dbg1<DV, GV, 1024>(c, nb, xpad, y, zt); break;
    case 36: sp_dbg1<DV, GV, 36>(c, nb, xpad, y, zt); break;
    case 40: sp_dbg1<DV, GV, 40>(c, nb, xpad, y, zt); break;
    case 32: sp_dbg1<DV, GV, 32>(c, nb, xpad, y, zt); break;
    case 35: sp_dbg1<DV, GV, 35>(c, nb, xpad, y, zt); break;
    default: sp_dbg1<DV, GV, 0>(c, nb, xpad, y, zt); break;
  }
}

void launch_spmv(Ctx& c, const double* xpad, double* y, bool dot, bool gated) {
  const int nb = (int)spmv_grid_blocks(c);
  const SpmvTiling tl = spmv_tiling(c.g, c.spmv_subl);
  if (c.fmt == FMT_VI && c.vi_block) {
    const u32x4* I = reinterpret_cast<const u32x4*>(c.vi_idx);
    if (vi_staged(c)) {  // x staged in LDS, 1024-node tiles marching z-chunks
      ZTiling zt = vis_tiling(c);
      zt.dbg = c.split_dbg;
      zt.wmap = c.vi_wmap;
      zt.xlist = c.vi_exc_list;
      zt.xskip = exc_blocks(c) > 0;
      zt.ypair = c.vi_ypair && (c.g.nx % 2) == 0;
      int tx, ty;
      vis_shape(c, tx, ty);
      if (st_used(c)) {  // default stencil: two planes per step, the listed rows after the march
        if (sp_used(c)) {
          const int dbg = zt.dbg;
          zt = sp_tiling(c);
          zt.dbg = dbg;
        }
        StFaces sfv = c.st_faces;
        int64_t stn = c.st_n, nbfa = stface_blocks(c);
        if (c.face_dbg && nbfa) {  // timing-only (option face_dbg, wrong products): drop listed rows / x / y-z patches
          if (c.face_dbg & 1) stn = 0;
          if (c.face_dbg & 2) {
            const int64_t d = sfv.u[2];
            for (int q = 1; q < 7; q++) sfv.u[q] = std::max<int64_t>(0, sfv.u[q] - d);
          }
          if (c.face_dbg & 4)
            for (int q = 3; q < 7; q++) sfv.u[q] = sfv.u[2];
          const int lpb = st_l16(c) ? SFP_T / ST16 : SFP_T;
          nbfa = sfv.u[6] + (stn + lpb - 1) / lpb;
        }
        double* pf = c.partials + nb;
        const int ndict = c.vi_nblocks > 0 ? c.vi_nblocks : VI_MAX;  // the listed rows stage only the blocks in use
#define MCX_SP_DBG(DV, GV) sp_dbg<DV, GV>(c, nb, xpad, y, zt)
#define MCX_ST(DV, GV)                                                                                             \
  do {                                                                                                            \
    const bool fs = nbfa && !c.vi_st_tail && fstream_ok(c); /* the faces beside the march (vi_st_fstream) */       \
    hipStream_t fst = fs ? c.f_stream : c.stream;                                                                 \
    if (fs) (void)hipEventRecord(c.ev_fx, c.stream);                                                              \
    if (c.vi_st_tail)                                                                                             \
      hipLaunchKernelGGL((k_spmv_st<DV, GV, true>), dim3(nb), dim3(1024), 0, c.stream, c.g, c.st_coef, c.st_mask,   \
                         c.st_npx, c.st_npy, xpad, y, c.partials, c.cg, zt, c.st_list, c.st_n, I, c.vi_bdict,     \
                         c.vi_exc, c.st_slot, c.st_faces);                                                        \
    else if (c.vi_st_pair && zt.dbg > 0)                                                                        \
      MCX_SP_DBG(DV, GV);                                                                                         \
    else if (c.vi_st_pair && c.vi_st_ty == 16)                                                                    \
      hipLaunchKernelGGL((k_spmv_sp<DV, GV, 16>), dim3(nb), dim3(1024), 0, c.stream, c.g, c.st_coef, c.st_mask,     \
                         c.st_npx, c.st_npy, xpad, y, c.partials, c.cg, zt);                                      \
    else if (c.vi_st_pair)                                                                                        \
      hipLaunchKernelGGL((k_spmv_sp<DV, GV, 8>), dim3(nb), dim3(512), 0, c.stream, c.g, c.st_coef, c.st_mask,       \
                         c.st_npx, c.st_npy, xpad, y, c.partials, c.cg, zt);                                      \
    else if (c.vi_st_pf == 3)                                                                                     \
      hipLaunchKernelGGL((k_spmv_st<DV, GV, false, false, true>), dim3(nb), dim3(1024), 0, c.stream, c.g,            \
                         c.st_coef, c.st_mask, c.st_npx, c.st_npy, xpad, y, c.partials, c.cg, zt);                \
    else if (c.vi_st_pf == 2)                                                                                     \
      hipLaunchKernelGGL((k_spmv_st<DV, GV, false, true>), dim3(nb), dim3(1024), 0, c.stream, c.g, c.st_coef,       \
                         c.st_mask, c.st_npx, c.st_npy, xpad, y, c.partials, c.cg, zt);                           \
    else                                                                                                          \
      hipLaunchKernelGGL((k_spmv_st<DV, GV>), dim3(nb), dim3(1024), 0, c.stream, c.g, c.st_coef, c.st_mask,         \
                         c.st_npx, c.st_npy, xpad, y, c.partials, c.cg, zt);                                      \
    if (fs) (void)hipStreamWaitEvent(fst, c.ev_fx, 0);                                                            \
    if (nbfa && st_l16(c))                                                                                        \
      hipLaunchKernelGGL((k_spmv_face<DV, GV>), dim3((unsigned)nbfa), dim3(SFP_T), 0, fst, c.g, sfv,                \
                         c.st_coef, c.st_slot, xpad, y, pf, c.cg, c.st_list, stn, I, c.vi_bdict, c.vi_exc, ndict); \
    else if (nbfa)                                                                                                \
      hipLaunchKernelGGL((k_spmv_face<DV, GV, false>), dim3((unsigned)nbfa), dim3(SFP_T), 0, fst, c.g,              \
                         sfv, c.st_coef, c.st_slot, xpad, y, pf, c.cg, c.st_list, stn, I, c.vi_bdict,   \
                         c.vi_exc, ndict);                                                                        \
    if (fs) {                                                                                                     \
      (void)hipEventRecord(c.ev_fd, fst);                                                                         \
      (void)hipStreamWaitEvent(c.stream, c.ev_fd, 0);                                                             \
    }                                                                                                             \
  } while (0)
        if (dot && gated) MCX_ST(true, true);
        else if (dot) MCX_ST(true, false);
        else MCX_ST(false, false);
#undef MCX_ST
#undef MCX_SP_DBG
        return;
      }
#define MCX_VIBM(TXV, TYV, XVV, UV, PV, ...)                                                                          \
  do {                                                                                                             \
    if (dot && gated)                                                                                              \
      hipLaunchKernelGGL((k_spmv_vibm<true, true, TXV, TYV, XVV, UV, PV, ##__VA_ARGS__>), dim3(nb), dim3(1024), 0,        \
                         c.stream, c.g, I, c.vi_bdict, xpad, y, c.partials, c.cg, zt);                             \
    else if (dot)                                                                                                  \
      hipLaunchKernelGGL((k_spmv_vibm<true, false, TXV, TYV, XVV, UV, PV, ##__VA_ARGS__>), dim3(nb), dim3(1024), 0,       \
                         c.stream, c.g, I, c.vi_bdict, xpad, y, c.partials, c.cg, zt);                             \
    else                                                                                                           \
      hipLaunchKernelGGL((k_spmv_vibm<false, false, TXV, TYV, XVV, UV, PV, ##__VA_ARGS__>), dim3(nb), dim3(1024), 0,      \
                         c.stream, c.g, I, c.vi_bdict, xpad, y, c.partials, c.cg, zt);                             \
  } while (0)
      if (c.vi_nexc) {  // exception nodes: the default (FMA) or exact rows, UNI + PATCH
#define MCX_VIBM_X(TXV, TYV, FV, ...)                                                                               \
  do {                                                                                                             \
    if (dot && gated)                                                                                              \
      hipLaunchKernelGGL((k_spmv_vibm<true, true, TXV, TYV, true, true, true, FV, false, false, true, ##__VA_ARGS__>),  \
                         dim3(nb), dim3(1024), 0, c.stream, c.g, I, c.vi_bdict, xpad, y, c.partials, c.cg, zt,      \
                         FusedP{}, c.vi_exc);                                                                      \
    else if (dot)                                                                                                  \
      hipLaunchKernelGGL((k_spmv_vibm<true, false, TXV, TYV, true, true, true, FV, false, false, true, ##__VA_ARGS__>), \
                         dim3(nb), dim3(1024), 0, c.stream, c.g, I, c.vi_bdict, xpad, y, c.partials, c.cg, zt,      \
                         FusedP{}, c.vi_exc);                                                                      \
    else                                                                                                           \
      hipLaunchKernelGGL((k_spmv_vibm<false, false, TXV, TYV, true, true, true, FV, false, false, true, ##__VA_ARGS__>),\
                         dim3(nb), dim3(1024), 0, c.stream, c.g, I, c.vi_bdict, xpad, y, c.partials, c.cg, zt,      \
                         FusedP{}, c.vi_exc);                                                                      \
  } while (0)
        if (c.vi_fma) {
          if (tx == 256) MCX_VIBM_X(256, 4, true);
          else if (tx == 128) MCX_VIBM_X(128, 8, true);
          else if (c.vi_lg == 2 && c.vi_lg_exc) MCX_VIBM_X(64, 16, true, false, 2);  // grouped LDS-path reads
          else MCX_VIBM_X(64, 16, true);
        } else {
          if (tx == 256) MCX_VIBM_X(256, 4, false);
          else if (tx == 128) MCX_VIBM_X(128, 8, false);
          else MCX_VIBM_X(64, 16, false);
        }
#undef MCX_VIBM_X
      } else if (wd_used(c) && !(c.vi_fma && c.vi_ring3)) {  // wave descriptors
        zt.wd = c.wd;
        zt.wdm = c.vi_wdesc;
        zt.npx = c.wd_npx;
        zt.npy = c.wd_npy;
        if (c.vi_fma) {
          if (tx == 256) MCX_VIBM(256, 4, true, true, true, true, false, false, false, true);
          else if (tx == 128) MCX_VIBM(128, 8, true, true, true, true, false, false, false, true);
          else if (c.vi_lg == 2) MCX_VIBM(64, 16, true, true, true, true, false, false, false, true, 2);
          else MCX_VIBM(64, 16, true, true, true, true, false, false, false, true);
        } else {
          if (tx == 256) MCX_VIBM(256, 4, true, true, true, false, false, false, false, true);
          else if (tx == 128) MCX_VIBM(128, 8, true, true, true, false, false, false, false, true);
          else MCX_VIBM(64, 16, true, true, true, false, false, false, false, true);
        }
      } else if (c.vi_fma && c.vi_ring3 && tx == 64) {
        MCX_VIBM(64, 16, true, true, true, true, false, true);
      } else if (c.vi_fma && tx == 64 && (c.vi_lg == 2 || c.vi_lg == 3)) {
        // LDS-path reads in groups of 2 blocks (default): SpMV 0.3098 vs 0.3228 ms, CG iteration
        // 0.8295 vs 0.8419 ms; groups of 3 spill (0.3866 ms) (profiles/old/r04_cg_ab_lg256.log)
        if (c.vi_lg == 2) MCX_VIBM(64, 16, true, true, true, true, false, false, false, false, 2);
        else MCX_VIBM(64, 16, true, true, true, true, false, false, false, false, 3);
      } else if (!c.vi_fma && c.vi_uni && c.vi_patch && tx == 64 && c.vi_lg == 2) {  // exact rows, the same groups
        MCX_VIBM(64, 16, true, true, true, false, false, false, false, false, 2);
      } else if (c.vi_fma) {
        if (tx == 256) MCX_VIBM(256, 4, true, true, true, true);
        else if (tx == 128) MCX_VIBM(128, 8, true, true, true, true);
        else MCX_VIBM(64, 16, true, true, true, true);
      } else if (c.vi_uni && c.vi_patch) {
        if (tx == 256) MCX_VIBM(256, 4, true, true, true);
        else if (tx == 128) MCX_VIBM(128, 8, true, true, true);
        else MCX_VIBM(64, 16, true, true, true);
      } else if (c.vi_uni) {
        if (tx == 256) MCX_VIBM(256, 4, true, true, false);
        else if (tx == 128) MCX_VIBM(128, 8, true, true, false);
        else MCX_VIBM(64, 16, true, true, false);
      } else if (c.vi_xread) {
        if (tx == 256) MCX_VIBM(256, 4, true, false, false);
        else if (tx == 128) MCX_VIBM(128, 8, true, false, false);
        else MCX_VIBM(64, 16, true, false, false);
      } else {
        if (tx == 256) MCX_VIBM(256, 4, false, false, false);
        else if (tx == 128) MCX_VIBM(128, 8, false, false, false);
        else MCX_VIBM(64, 16, false, false, false);
      }
#undef MCX_VIBM
      const int64_t nbf = faces_blocks(c);
      if (nbf) {  // exact rows: the nodes on the global boundary (skipped by the z-march)
        const FaceEnum fe = face_enum(c.g);
        double* pf = c.partials + nb;
        if (dot && gated && c.vi_nexc)
          hipLaunchKernelGGL((k_spmv_vib_faces<true, true, true>), dim3(nbf), dim3(TPB), 0, c.stream, c.g, I, c.vi_bdict,
                             xpad, y, pf, c.cg, fe, c.vi_exc);
        else if (dot && gated)
          hipLaunchKernelGGL((k_spmv_vib_faces<true, true, false>), dim3(nbf), dim3(TPB), 0, c.stream, c.g, I,
                             c.vi_bdict, xpad, y, pf, c.cg, fe, c.vi_exc);
        else if (dot && c.vi_nexc)
          hipLaunchKernelGGL((k_spmv_vib_faces<true, false, true>), dim3(nbf), dim3(TPB), 0, c.stream, c.g, I,
                             c.vi_bdict, xpad, y, pf, c.cg, fe, c.vi_exc);
        else if (dot)
          hipLaunchKernelGGL((k_spmv_vib_faces<true, false, false>), dim3(nbf), dim3(TPB), 0, c.stream, c.g, I,
                             c.vi_bdict, xpad, y, pf, c.cg, fe, c.vi_exc);
        else if (c.vi_nexc)
          hipLaunchKernelGGL((k_spmv_vib_faces<false, false, true>), dim3(nbf), dim3(TPB), 0, c.stream, c.g, I,
                             c.vi_bdict, xpad, y, pf, c.cg, fe, c.vi_exc);
        else
          hipLaunchKernelGGL((k_spmv_vib_faces<false, false, false>), dim3(nbf), dim3(TPB), 0, c.stream, c.g, I,
                             c.vi_bdict, xpad, y, pf, c.cg, fe, c.vi_exc);
      }
      const int64_t nbx = exc_blocks(c);
      if (nbx) {  // the exception rows the z-march left out
        double* px = c.partials + nb + nbf;
#define MCX_EXCK(DV, GV, FV)                                                                                       \
  hipLaunchKernelGGL((k_spmv_exc<DV, GV, FV>), dim3((unsigned)nbx), dim3(TPB), 0, c.stream, c.g, c.vi_xlist,        \
                     c.vi_nexc, c.vi_exc, xpad, y, px, c.cg)
        if (c.vi_fma) {
          if (dot && gated) MCX_EXCK(true, true, true);
          else if (dot) MCX_EXCK(true, false, true);
          else MCX_EXCK(false, false, true);
        } else {
          if (dot && gated) MCX_EXCK(true, true, false);
          else if (dot) MCX_EXCK(true, false, false);
          else MCX_EXCK(false, false, false);
        }
#undef MCX_EXCK
      }
      return;
    }
    if (c.vi_nexc) {
      if (dot && gated)
        hipLaunchKernelGGL((k_spmv_vib<true, true, true>), dim3(nb), dim3(TPB), 0, c.stream, c.g, I, c.vi_bdict, xpad,
                           y, c.partials, c.cg, tl, c.vi_exc);
      else if (dot)
        hipLaunchKernelGGL((k_spmv_vib<true, false, true>), dim3(nb), dim3(TPB), 0, c.stream, c.g, I, c.vi_bdict, xpad,
                           y, c.partials, c.cg, tl, c.vi_exc);
      else
        hipLaunchKernelGGL((k_spmv_vib<false, false, true>), dim3(nb), dim3(TPB), 0, c.stream, c.g, I, c.vi_bdict,
                           xpad, y, c.partials, c.cg, tl, c.vi_exc);
      return;
    }
    if (dot && gated)
      hipLaunchKernelGGL((k_spmv_vib<true, true>), dim3(nb), dim3(TPB), 0, c.stream, c.g, I, c.vi_bdict, xpad, y,
                         c.partials, c.cg, tl);
    else if (dot)
      hipLaunchKernelGGL((k_spmv_vib<true, false>), dim3(nb), dim3(TPB), 0, c.stream, c.g, I, c.vi_bdict, xpad, y,
                         c.partials, c.cg, tl);
    else
      hipLaunchKernelGGL((k_spmv_vib<false, false>), dim3(nb), dim3(TPB), 0, c.stream, c.g, I, c.vi_bdict, xpad, y,
                         c.partials, c.cg, tl);
    return;
  }
  if (c.fmt == FMT_VI) {
    if (c.vi_bits == 4) launch_spmv_vi<4>(c, xpad, y, dot, gated, nb, tl);
    else launch_spmv_vi<8>(c, xpad, y, dot, gated, nb, tl);  // byte indices: gathered x (the ring spills)
    return;
  }
  if (c.fmt == FMT_SPLIT) {
    int ztx, zty;
    split_shape(c, ztx, zty);
    const ZTiling zt = z_tiling(c.g, ztx, zty, c.spmv_zblocks);
    if (ztx == 256 && zty == 4) launch_symp<256, 4, true>(c, xpad, y, dot, gated, zt, nb);
    else if (ztx == 256) launch_symp<256, 2, true>(c, xpad, y, dot, gated, zt, nb);
    else if (ztx == 128 && zty == 8) launch_symp<128, 8, true>(c, xpad, y, dot, gated, zt, nb);
    else if (ztx == 128) launch_symp<128, 4, true>(c, xpad, y, dot, gated, zt, nb);
    else if (ztx == 64 && zty == 16) launch_symp<64, 16, true>(c, xpad, y, dot, gated, zt, nb);
    else launch_symp<64, 4, true>(c, xpad, y, dot, gated, zt, nb);
    return;
  }
  if (c.fmt == FMT_U && c.spmv_kernel >= 1) {
    int ztx, zty;
    z_shape(c.spmv_kernel, ztx, zty);
    const ZTiling zt = z_tiling(c.g, ztx, zty, c.spmv_zblocks);
    switch (c.spmv_kernel) {
      case 2: launch_symz<32, 4>(c, xpad, y, dot, gated, zt, nb); break;
      case 3: launch_symz<64, 2>(c, xpad, y, dot, gated, zt, nb); break;
      case 4: launch_symz<128, 2>(c, xpad, y, dot, gated, zt, nb); break;
      case 5: launch_symz<128, 4>(c, xpad, y, dot, gated, zt, nb); break;
      case 6: launch_symz<256, 2>(c, xpad, y, dot, gated, zt, nb); break;
      case 7: launch_symp<128, 4>(c, xpad, y, dot, gated, zt, nb); break;
      case 8: launch_symp<64, 4>(c, xpad, y, dot, gated, zt, nb); break;
      case 9: launch_symp<64, 8>(c, xpad, y, dot, gated, zt, nb); break;
      case 10: launch_symp<256, 2>(c, xpad, y, dot, gated, zt, nb); break;
      case 11: launch_symp<256, 4>(c, xpad, y, dot, gated, zt, nb); break;
      default: launch_symz<64, 4>(c, xpad, y, dot, gated, zt, nb); break;
    }
    return;
  }
  if (c.fmt == FMT_U) {
    if (dot && gated)
      hipLaunchKernelGGL((k_spmv_sym<true, true>), dim3(nb), dim3(TPB), 0, c.stream, c.g, c.U, xpad, y, c.partials,
                         c.cg, tl);
    else if (dot)
      hipLaunchKernelGGL((k_spmv_sym<true, false>), dim3(nb), dim3(TPB), 0, c.stream, c.g, c.U, xpad, y, c.partials,
                         c.cg, tl);
    else
      hipLaunchKernelGGL((k_spmv_sym<false, false>), dim3(nb), dim3(TPB), 0, c.stream, c.g, c.U, xpad, y, c.partials,
                         c.cg, tl);
    return;
  }
  const double2* V = reinterpret_cast<const double2*>(c.V);
  if (c.spmv_nt == 2) {
    if (dot && gated)
      hipLaunchKernelGGL((k_spmv<true, true, 2>), dim3(nb), dim3(TPB), 0, c.stream, c.g, V, xpad, y, c.partials, c.cg,
                         tl);
    else
      hipLaunchKernelGGL((k_spmv<true, false, 2>), dim3(nb), dim3(TPB), 0, c.stream, c.g, V, xpad, y, c.partials,
                         c.cg, tl);
    return;
  }
  if (c.spmv_nt) {
    if (dot && gated)
      hipLaunchKernelGGL((k_spmv<true, true, 1>), dim3(nb), dim3(TPB), 0, c.stream, c.g, V, xpad, y, c.partials, c.cg,
                         tl);
    else
      hipLaunchKernelGGL((k_spmv<true, false, 1>), dim3(nb), dim3(TPB), 0, c.stream, c.g, V, xpad, y, c.partials,
                         c.cg, tl);
    return;
  }
  if (dot && gated)
    hipLaunchKernelGGL((k_spmv<true, true>), dim3(nb), dim3(TPB), 0, c.stream, c.g, V, xpad, y, c.partials, c.cg, tl);
  else if (dot)
    hipLaunchKernelGGL((k_spmv<true, false>), dim3(nb), dim3(TPB), 0, c.stream, c.g, V, xpad, y, c.partials, c.cg, tl);
  else
    hipLaunchKernelGGL((k_spmv<false, false>), dim3(nb), dim3(TPB), 0, c.stream, c.g, V, xpad, y, c.partials, c.cg, tl);
}

void launch_update_u(Ctx& c) {
  hipLaunchKernelGGL(k_update_u, dim3(nblk(c.g.nown)), dim3(TPB), 0, c.stream, c.g, c.u_pad, c.du);
}

void launch_copy_owned_to_pad(Ctx& c, const double* owned, double* pad) {
  hipLaunchKernelGGL(k_owned_to_pad, dim3(nblk(c.g.nown)), dim3(TPB), 0, c.stream, c.g, owned, pad);
}

void launch_copy_pad_to_owned(Ctx& c, const double* pad, double* owned) {
  hipLaunchKernelGGL(k_pad_to_owned, dim3(nblk(c.g.nown)), dim3(TPB), 0, c.stream, c.g, pad, owned);
}

void launch_pack(Ctx& c, const double* xpad) {
  if (!c.halo.nsend) return;
  hipLaunchKernelGGL(k_pack, dim3(nblk(c.halo.nsend)), dim3(TPB), 0, c.stream, c.halo.d_send_idx, c.halo.nsend, xpad,
                     c.halo.d_sendbuf);
}

void launch_unpack(Ctx& c, double* xpad) {
  if (!c.halo.nrecv) return;
  hipLaunchKernelGGL(k_unpack, dim3(nblk(c.halo.nrecv)), dim3(TPB), 0, c.stream, c.halo.d_recv_idx, c.halo.nrecv,
                     c.halo.d_recvbuf, xpad);
}

// reduce partials into out (and, for RED_NORM, out[0] = sqrt); multi-rank: local sums are
// all-reduced over RCCL first.
void launch_group_sum(Ctx& c, const double* const* ptrs, int nranks, int count, double* out, int op) {
  hipLaunchKernelGGL(k_group_sum, dim3(1), dim3(64), 0, c.stream, ptrs, nranks, count, out, op);
}

void launch_vtu_cells(Ctx& c, const int* lo, const int* cnt, double* out) {
  const int64_t n = (int64_t)cnt[0] * cnt[1] * cnt[2];
  if (n <= 0) return;
  hipLaunchKernelGGL(k_vtu_cells, dim3((unsigned)((n + TPB - 1) / TPB)), dim3(TPB), 0, c.stream, c.g, c.u_pad, c.sig,
                     c.ftrial, lo[0], lo[1], lo[2], cnt[0], cnt[1], cnt[2], out);
}

void launch_force_layer(Ctx& c, int comp, int fa, int fixed, int a0, int na, int b0, int nb, double* out) {
  const int n = na * nb;
  if (n <= 0) return;
  hipLaunchKernelGGL(k_force_layer, dim3((n + TPB - 1) / TPB), dim3(TPB), 0, c.stream, c.g, c.sig, comp, fa, fixed,
                     a0, na, b0, nb, out);
}

// part: the partial sums (c.partials, or c.partials2 for the update's); single rank: the step
// runs on c.cg starting from *src (c.cg, or the fused path's other buffer c.cg + 1)
static int reduce_and_logic(Ctx& c, int nvals, int nparts, int mode, bool gated, const double* part,
                            const CgState* src) {
  if (c.nranks == 1 && !c.comm) {
    hipLaunchKernelGGL(k_reduce, dim3(1), dim3(1024), 0, c.stream, part, nparts, nvals, c.red, mode, c.cg, c.hist,
                       gated ? 1 : 0, src);
    return 0;
  }
  int rc0 = allreduce_prepare(c);
  if (rc0) return rc0;
  hipLaunchKernelGGL(k_reduce, dim3(1), dim3(1024), 0, c.stream, part, nparts, nvals, c.red_loc, (int)RED_STORE,
                     c.cg, c.hist, gated ? 1 : 0, c.cg);
  int rc = allreduce_sum(c, c.red_loc, c.red, nvals);
  if (rc) return rc;
  hipLaunchKernelGGL(k_cg_logic, dim3(1), dim3(64), 0, c.stream, c.red, mode, c.cg, c.hist, c.red);
  return 0;
}

void launch_reduce(Ctx& c, int nvals, int nparts, double* out) {
  (void)out;
  reduce_and_logic(c, nvals, nparts, RED_NORM, false, c.partials, c.cg);
}

void launch_cg_init(Ctx& c) {
  int nb = (int)nblk(c.g.nown);
  hipLaunchKernelGGL(k_cg_init, dim3(nb), dim3(TPB), 0, c.stream, c.g, c.b, c.dinv, c.du, c.r, c.z, c.partials, nb);
}

int cg_finish_init(Ctx& c) {
  int nb = (int)nblk(c.g.nown);
  return reduce_and_logic(c, 2, nb, RED_INIT, false, c.partials, c.cg);
}

static PQ pq_of(const Ctx& c) {
  return PQ{{c.p_pad, c.p_pad2, c.p_pad3, c.p_pad4, c.p_pad58[0], c.p_pad58[1], c.p_pad58[2], c.p_pad58[3]}};
}
static int pq_mask(const Ctx& c) { return c.xs_used ? 7 : 3; }

int launch_cg_xfinal(Ctx& c) {
  if (c.pqb_used) {
    if (c.xs_used) {  // the side stream's windows first
      MCX_HIP(hipStreamWaitEvent(c.stream, c.ev_xd[0], 0));
      MCX_HIP(hipStreamWaitEvent(c.stream, c.ev_xd[1], 0));
    }
    hipLaunchKernelGGL(k_cg_xfinal_qb, dim3(nblk(c.g.nown)), dim3(TPB), 0, c.stream, c.g, pq_of(c), c.du, c.cg,
                       c.xdone, pq_mask(c));
    return 0;
  }
  hipLaunchKernelGGL(k_cg_xfinal, dim3(nblk(c.g.nown)), dim3(TPB), 0, c.stream, c.g, c.p_pad,
                     c.fusep_used || c.pdb_used ? c.p_pad2 : nullptr, c.du, c.cg, c.pdb_used ? c.xdone : nullptr);
  return 0;
}

// CG vector kernels' Jacobi form: DIX (block-indexed value storage, option cg_dix) reads one
// diagonal-block index byte per node and recomputes z = D^-1 r from r where it is used, so the
// update writes no z and reads no dinv vector (two fewer vectors per iteration)
static bool cg_dix(const Ctx& c) { return c.cg_dix && c.fmt == FMT_VI && c.vi_block; }

// instantiate CALL with constexpr NT (non-temporal stores) and DX (DIX) from run-time flags
#define MCX_NT_DIX(ntv, dixv, CALL)                      \
  do {                                                   \
    if ((ntv) && (dixv)) {                               \
      constexpr bool NT = true, DX = true;               \
      CALL;                                              \
    } else if (ntv) {                                    \
      constexpr bool NT = true, DX = false;              \
      CALL;                                              \
    } else if (dixv) {                                   \
      constexpr bool NT = false, DX = true;              \
      CALL;                                              \
    } else {                                             \
      constexpr bool NT = false, DX = false;             \
      CALL;                                              \
    }                                                    \
  } while (0)

void launch_cg_pupdate(Ctx& c, int part) {
  const unsigned nbn = nblk(c.g.nown);
  const bool dix = cg_dix(c);
  const double* zs = dix ? c.r : c.z;
  const double* jd = dix ? c.jdd : c.dinv;
  if (c.pqb_used) {  // p in four buffers, x every fourth iteration
    // the host's hint of the iteration's kind (cg_par 2: deliberately wrong at it = 4m - 1 and 4m)
    const int hit = c.cg_it + (c.cg_par == 2);
    const int par = c.cg_par && c.cg_it >= 1 ? 1 + (hit >= 4 && (hit & 3) == 0) : 0;
    const PQ pq = pq_of(c);
    // P2D: the whole-subdomain update only (not the sent-node list), natural order
    const bool p2d = c.cg_p2d && part != 1 && !c.cg_rev;
    const dim3 g2d((unsigned)(c.g.ny * c.g.nz), (unsigned)((c.g.nx + TPB - 1) / TPB));
#define MCX_PQB_PAR(SKIPV, GRID, LIST, CNT)                                                                          \
  MCX_NT_DIX(c.cg_nt, dix, {                                                                                         \
    if (c.xs_used)                                                                                                   \
      hipLaunchKernelGGL((k_cg_pupdate_qb<NT, DX, SKIPV, 1, true>), dim3(GRID), dim3(TPB), 0, c.stream, c.g, zs, jd,  \
                         c.jix, pq, c.du, c.cg, c.xdone, LIST, CNT, c.cg_rev);                                       \
    else if (p2d && par == 1)                                                                                        \
      hipLaunchKernelGGL((k_cg_pupdate_qb<NT, DX, SKIPV, 1, false, true>), g2d, dim3(TPB), 0, c.stream, c.g, zs, jd,  \
                         c.jix, pq, c.du, c.cg, c.xdone, LIST, CNT, 0);                                              \
    else if (p2d && par == 2)                                                                                        \
      hipLaunchKernelGGL((k_cg_pupdate_qb<NT, DX, SKIPV, 2, false, true>), g2d, dim3(TPB), 0, c.stream, c.g, zs, jd,  \
                         c.jix, pq, c.du, c.cg, c.xdone, LIST, CNT, 0);                                              \
    else if (par == 1)                                                                                               \
      hipLaunchKernelGGL((k_cg_pupdate_qb<NT, DX, SKIPV, 1>), dim3(GRID), dim3(TPB), 0, c.stream, c.g, zs, jd, c.jix, \
                         pq, c.du, c.cg, c.xdone, LIST, CNT, c.cg_rev);                                              \
    else if (par == 2)                                                                                               \
      hipLaunchKernelGGL((k_cg_pupdate_qb<NT, DX, SKIPV, 2>), dim3(GRID), dim3(TPB), 0, c.stream, c.g, zs, jd, c.jix, \
                         pq, c.du, c.cg, c.xdone, LIST, CNT, c.cg_rev);                                              \
    else                                                                                                             \
      hipLaunchKernelGGL((k_cg_pupdate_qb<NT, DX, SKIPV, 0>), dim3(GRID), dim3(TPB), 0, c.stream, c.g, zs, jd, c.jix, \
                         pq, c.du, c.cg, c.xdone, LIST, CNT, c.cg_rev);                                              \
  })
    if (part == 1) {
      if (!c.halo.nbnd) return;
      MCX_PQB_PAR(false, nblk(c.halo.nbnd), c.halo.d_bnd, c.halo.nbnd);
    } else if (part == 2) {
      MCX_PQB_PAR(true, nbn, nullptr, (int64_t)c.g.nown);
    } else {
      MCX_PQB_PAR(false, nbn, nullptr, (int64_t)c.g.nown);
    }
#undef MCX_PQB_PAR
    return;
  }
  if (c.pdb_used) {  // p double-buffered, x every second iteration
    // cg_par: the kernel of the iteration's parity (the host's count; the kernel checks it)
    const int par = c.cg_par && c.cg_it >= 2 ? 1 + ((c.cg_it + (c.cg_par == 2)) & 1) : 0;
#define MCX_PDB_PAR(SKIPV, GRID, LIST, CNT)                                                                          \
  MCX_NT_DIX(c.cg_nt, dix, {                                                                                         \
    if (par == 1)                                                                                                    \
      hipLaunchKernelGGL((k_cg_pupdate_db<NT, DX, SKIPV, 1>), dim3(GRID), dim3(TPB), 0, c.stream, c.g, zs, jd, c.jix, \
                         c.p_pad, c.p_pad2, c.du, c.cg, c.xdone, LIST, CNT, c.cg_rev);                               \
    else if (par == 2)                                                                                               \
      hipLaunchKernelGGL((k_cg_pupdate_db<NT, DX, SKIPV, 2>), dim3(GRID), dim3(TPB), 0, c.stream, c.g, zs, jd, c.jix, \
                         c.p_pad, c.p_pad2, c.du, c.cg, c.xdone, LIST, CNT, c.cg_rev);                               \
    else                                                                                                             \
      hipLaunchKernelGGL((k_cg_pupdate_db<NT, DX, SKIPV, 0>), dim3(GRID), dim3(TPB), 0, c.stream, c.g, zs, jd, c.jix, \
                         c.p_pad, c.p_pad2, c.du, c.cg, c.xdone, LIST, CNT, c.cg_rev);                               \
  })
    if (part == 1) {
      if (!c.halo.nbnd) return;
      MCX_PDB_PAR(false, nblk(c.halo.nbnd), c.halo.d_bnd, c.halo.nbnd);
    } else if (part == 2) {
      MCX_PDB_PAR(true, nbn, nullptr, (int64_t)c.g.nown);
    } else {
      MCX_PDB_PAR(false, nbn, nullptr, (int64_t)c.g.nown);
    }
#undef MCX_PDB_PAR
    return;
  }
  if (part == 1) {
    if (!c.halo.nbnd) return;
    const unsigned nb = nblk(c.halo.nbnd);
    MCX_NT_DIX(c.cg_nt, dix,
               hipLaunchKernelGGL((k_cg_pupdate_list<NT, DX>), dim3(nb), dim3(TPB), 0, c.stream, c.g, zs, jd, c.jix,
                                  c.p_pad, c.du, c.cg, c.halo.d_bnd, c.halo.nbnd));
  } else if (part == 2) {
    MCX_NT_DIX(c.cg_nt, dix,
               hipLaunchKernelGGL((k_cg_pupdate<NT, DX, true>), dim3(nbn), dim3(TPB), 0, c.stream, c.g, zs, jd, c.jix,
                                  c.p_pad, c.du, c.cg));
  } else {
    MCX_NT_DIX(c.cg_nt, dix,
               hipLaunchKernelGGL((k_cg_pupdate<NT, DX>), dim3(nbn), dim3(TPB), 0, c.stream, c.g, zs, jd, c.jix,
                                  c.p_pad, c.du, c.cg));
  }
}

// Fused scalar steps (single rank, c.fuse, small grids: <= 1024 update blocks): the alpha step
// runs in the update kernel, the beta step in the next iteration's p update, and a chunk's last
// beta step in k_reduce so the host poll and the next chunk read c.cg.  first: the chunk's first
// iteration (its p update starts from c.cg).
static bool fused(const Ctx& c) { return c.fuse && c.nranks == 1 && !c.comm; }

// the solve's p update: double-buffered (PDB) unless the p update is fused into the SpMV
// (fusep) or into the scalar steps (single rank, <= 1,024 update blocks: k_cg_pupdate_fb)
bool cg_pdb(const Ctx& c) {
  const int nbu = (int)((c.g.nown + UTPB - 1) / UTPB);
  return c.cg_pdb && c.p_pad2 && c.xdone && !fusep(c) && !(fused(c) && nbu <= 1024);
}

// algorithmic bytes per owned node of one CG iteration's vector kernels (the last solve's forms):
// k_cg_update r, w in (+ D^-1 as a vector, + z out) or the Jacobi index byte (DIX), r out; the p
// update p(i-1), z or r (+ the index byte) in, p(i) out, and x's read + write plus the owed p
// terms amortised over the iterations that apply them (every 4th: PQB, every 2nd: PDB)
int64_t cg_vec_bytes_per_node(const Ctx& c) {
  const bool dix = cg_dix(c);
  const int64_t upd = dix ? 73 : 120;
  int64_t pup;
  if (c.fusep_used) pup = 48;  // p inside the SpMV (counted there); x every second iteration in the update
  else if (c.pqb_used) pup = (dix ? 73 : 72) + (48 + 3 * 24) / 4;
  else if (c.pdb_used) pup = (dix ? 73 : 72) + (48 + 24) / 2;
  else pup = dix ? 121 : 120;
  return upd + pup;
}

int cg_iteration(Ctx& c, hipEvent_t ev0, hipEvent_t ev1, bool first, bool last) {
  const int nbs = (int)spmv_nparts(c);
  const int nbu = (int)((c.g.nown + UTPB - 1) / UTPB);
  CgState* A = c.cg + 1;  // fused path: the state after the alpha step
  // both folds or none: at 256^3 (16,384 update blocks) the alpha prologue of every block costs
  // more than the k_reduce launch it saves (4.177 vs 4.159 ms per CG iteration); at 64^3 the two
  // folds save 1.6 % (profiles/old/r02_cg_ab_fuse{64,256}.log)
  const bool fa = fused(c) && nbu <= 1024, fb = fa;
  int rc;
  const bool dix = cg_dix(c);
  const double* zs = dix ? c.r : c.z;
  const double* jd = dix ? c.jdd : c.dinv;
  if (fusep(c) && !fa) {  // p update inside the SpMV (no k_cg_pupdate, no halo: single rank)
    c.fusep_used = true;
    if (ev0) MCX_HIP(hipEventRecord(ev0, c.stream));
    launch_spmv_fusep(c, c.w);
    if (ev1) MCX_HIP(hipEventRecord(ev1, c.stream));
    rc = reduce_and_logic(c, 1, nbs, RED_ALPHA, true, c.partials, c.cg);
    if (rc) return rc;
    if (c.cg_nt)
      hipLaunchKernelGGL(k_cg_update_x<true>, dim3(nbu), dim3(UTPB), 0, c.stream, c.g, c.w, c.jdd, c.jix, c.r, c.du,
                         c.p_pad, c.p_pad2, c.partials2, nbu, c.cg);
    else
      hipLaunchKernelGGL(k_cg_update_x<false>, dim3(nbu), dim3(UTPB), 0, c.stream, c.g, c.w, c.jdd, c.jix, c.r, c.du,
                         c.p_pad, c.p_pad2, c.partials2, nbu, c.cg);
    return reduce_and_logic(c, 2, nbu, RED_BETA, true, c.partials2, c.cg);
  }
  // p of this iteration (PDB: buffer it & 1, `it` = the host's count of launched iterations, which
  // is the device's cg->i for every iteration that runs; the fused small-grid path fb has one buffer)
  double* pcur = c.pqb_used ? pq_of(c).p[c.cg_it & pq_mask(c)] : (c.pdb_used && (c.cg_it & 1) ? c.p_pad2 : c.p_pad);
  // XS: p(it) overwrites p(it-8)'s buffer, read by the window kernel of iteration it-4
  const bool xwin = c.xs_used && c.cg_it >= 4 && (c.cg_it & 3) == 0;
  if (xwin && c.cg_it >= 8) MCX_HIP(hipStreamWaitEvent(c.stream, c.ev_xd[((c.cg_it >> 2) - 1) & 1], 0));
  if (fb && !first) {
    MCX_NT_DIX(c.cg_nt, dix,
               hipLaunchKernelGGL((k_cg_pupdate_fb<NT, DX>), dim3(nblk(c.g.nown)), dim3(TPB), 0, c.stream, c.g, zs, jd,
                                  c.jix, c.p_pad, c.du, c.partials2, nbu, A, c.cg, c.hist));
  } else if (c.nranks > 1 && c.overlap && c.halo.nbnd) {
    // the sent nodes' p first, then their exchange overlaps the interior p update
    launch_cg_pupdate(c, 1);
    if ((rc = halo_start(c, pcur))) return rc;
    launch_cg_pupdate(c, 2);
    if ((rc = halo_finish(c, pcur))) return rc;
  } else {
    launch_cg_pupdate(c, 0);
  }
  if (!(c.nranks > 1 && c.overlap && c.halo.nbnd) && (rc = halo_exchange(c, pcur))) return rc;
  if (xwin) {  // the window it-4 .. it-1 on the side stream, beside this iteration's SpMV and update
    MCX_HIP(hipEventRecord(c.ev_xp, c.stream));
    MCX_HIP(hipStreamWaitEvent(c.x_stream, c.ev_xp, 0));
    hipLaunchKernelGGL(k_cg_xwin, dim3(nblk(c.g.nown)), dim3(TPB), 0, c.x_stream, c.g, pq_of(c), c.du, c.cg, c.xdone,
                       c.cg_it);
    MCX_HIP(hipEventRecord(c.ev_xd[(c.cg_it >> 2) & 1], c.x_stream));
  }
  if (ev0) MCX_HIP(hipEventRecord(ev0, c.stream));
  launch_spmv(c, pcur, c.w, true, true);
  if (ev1) MCX_HIP(hipEventRecord(ev1, c.stream));
  if (fa) {
    MCX_NT_DIX(c.cg_nt, dix,
               hipLaunchKernelGGL((k_cg_update_fa<NT, DX>), dim3(nbu), dim3(UTPB), 0, c.stream, c.g, c.w, jd, c.jix,
                                  c.r, c.z, c.partials2, nbu, c.partials, nbs, c.cg, A));
    if (!fb || last) return reduce_and_logic(c, 2, nbu, RED_BETA, true, c.partials2, A);
    return 0;
  }
  rc = reduce_and_logic(c, 1, nbs, RED_ALPHA, true, c.partials, c.cg);
  if (rc) return rc;
  const int nbg = c.cg_ublocks > 0 ? std::min(nbu, c.cg_ublocks) : nbu;
  MCX_NT_DIX(c.cg_nt, dix,
             hipLaunchKernelGGL((k_cg_update<NT, DX>), dim3(nbg), dim3(UTPB), 0, c.stream, c.g, c.w, jd, c.jix, c.r,
                                c.z, c.partials2, nbg, c.cg));
  return reduce_and_logic(c, 2, nbg, RED_BETA, true, c.partials2, c.cg);
}

}  // namespace mcx
