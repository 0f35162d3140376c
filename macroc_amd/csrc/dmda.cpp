#include <algorithm>
// dmda.cpp — host-side DMDA decomposition of the MI355X MacroC path.
//
// Restates what PETSc's DMDACreate3d/DMSetUp (src/init.c:85-94 of the reference) produce for
// the MacroC grid: the PETSC_DECIDE rank grid (PETSc da3.c), the ownership split
// lx[i] = M/m + (M%m > i), rank-contiguous global numbering with x fastest, width-1 box
// ghosts.  Each rank additionally gets a padded ghost box (1 layer on every side, zeros
// outside the physical domain) so that device kernels never branch on the boundary.
#include <cmath>
#include <cstdio>

#include "mcx_internal.h"

namespace mcx {

int dmda_decide(int64_t M, int64_t N, int64_t P, int size, int* pm_, int* pn_, int* pp_) {
  int64_t m = *pm_ > 0 ? *pm_ : 0, n = *pn_ > 0 ? *pn_ : 0, p = *pp_ > 0 ? *pp_ : 0;
  if ((m && m > size) || (n && n > size) || (p && p > size)) return 1;
  if (m && n && p) {
    // fully specified
  } else if (!m && n && p) {
    m = size / (n * p);
  } else if (m && !n && p) {
    n = size / (m * p);
  } else if (m && n && !p) {
    p = size / (m * n);
  } else if (!m && !n && p) {  // squarish in x-y
    for (m = std::max<int64_t>(1, (int64_t)(0.5 + std::sqrt((double)M * size / ((double)N * p)))); m > 0; m--) {
      n = size / (m * p);
      if (m * n * p == size) break;
    }
    if (!m) return 3;
    if (M > N && m < n) std::swap(m, n);
  } else if (!m && n && !p) {  // squarish in x-z
    for (m = std::max<int64_t>(1, (int64_t)(0.5 + std::sqrt((double)M * size / ((double)P * n)))); m > 0; m--) {
      p = size / (m * n);
      if (m * n * p == size) break;
    }
    if (!m) return 3;
    if (M > P && m < p) std::swap(m, p);
  } else if (m && !n && !p) {  // squarish in y-z
    for (n = std::max<int64_t>(1, (int64_t)(0.5 + std::sqrt((double)N * size / ((double)P * m)))); n > 0; n--) {
      p = size / (m * n);
      if (m * n * p == size) break;
    }
    if (!n) return 3;
    if (N > P && n < p) std::swap(n, p);
  } else {  // all three decided: n from a cube root, then m
    n = (int64_t)(0.5 + std::pow((double)N * N * size / ((double)P * M), 1. / 3.));
    if (!n) n = 1;
    while (n > 0 && size % n) n--;
    if (!n) n = 1;
    for (m = std::max<int64_t>(1, (int64_t)(0.5 + std::sqrt((double)M * size / ((double)P * n)))); m > 0; m--) {
      p = size / (m * n);
      if (m * n * p == size) break;
    }
    if (M > P && m < p) std::swap(m, p);
  }
  if (m * n * p != size) return 2;
  if (M < m || N < n || P < p) return 4;
  *pm_ = (int)m;
  *pn_ = (int)n;
  *pp_ = (int)p;
  return 0;
}

static void split(int64_t M, int q, std::vector<int64_t>& w, std::vector<int64_t>& s) {
  w.resize(q);
  s.resize(q);
  int64_t acc = 0;
  for (int i = 0; i < q; i++) {
    w[i] = M / q + ((M % q) > i);
    s[i] = acc;
    acc += w[i];
  }
}

int setup_decomposition(Ctx& c) {
  const mcx_opts& o = c.o;
  if (o.NX < 2 || o.NY < 2 || o.NZ < 2) {
    set_error("grid needs at least 2 nodes per direction");
    return 2;
  }
  int m = o.px, n = o.py, p = o.pz;
  int rc = dmda_decide(o.NX, o.NY, o.NZ, c.nranks, &m, &n, &p);
  if (rc) {
    set_error("could not find a DMDA partition for the rank count (code " + std::to_string(rc) + ")");
    return 3;
  }
  c.m = m;
  c.n = n;
  c.p = p;
  c.pi = c.rank % m;
  c.pj = (c.rank % (m * n)) / m;
  c.pk = c.rank / (m * n);
  split(o.NX, m, c.wx, c.sx);
  split(o.NY, n, c.wy, c.sy);
  split(o.NZ, p, c.wz, c.sz);
  c.rank_node_off.assign(c.nranks + 1, 0);
  for (int r = 0; r < c.nranks; r++) {
    int a = r % m, b = (r % (m * n)) / m, d = r / (m * n);
    c.rank_node_off[r + 1] = c.rank_node_off[r] + c.wx[a] * c.wy[b] * c.wz[d];
  }
  Geo& g = c.g;
  g.NX = (int)o.NX;
  g.NY = (int)o.NY;
  g.NZ = (int)o.NZ;
  g.xs = (int)c.sx[c.pi];
  g.ys = (int)c.sy[c.pj];
  g.zs = (int)c.sz[c.pk];
  g.nx = (int)c.wx[c.pi];
  g.ny = (int)c.wy[c.pj];
  g.nz = (int)c.wz[c.pk];
  // padded row pitch: nx + 2 nodes, rounded to 16 (384 B = 3 lines) with pad_align, so the rows
  // of a padded vector keep one alignment
  g.PX = c.pad_align ? (g.nx + 2 + 15) / 16 * 16 : g.nx + 2;
  c.pad_off = c.pad_align == 1 ? 104 : 0;  // 104 + 24 = 128: node (0, j, k) starts a line
  g.PY = g.ny + 2;
  g.PZ = g.nz + 2;
  g.nown = g.nx * g.ny * g.nz;
  // elements evaluated here: every element touching an owned node
  int e0[3], e1[3];
  int xs[3] = {g.xs, g.ys, g.zs}, nn[3] = {g.nx, g.ny, g.nz}, NN[3] = {g.NX, g.NY, g.NZ};
  for (int d = 0; d < 3; d++) {
    e0[d] = std::max(xs[d] - 1, 0);
    e1[d] = std::min(xs[d] + nn[d] - 1, NN[d] - 2);
  }
  g.ex0 = e0[0];
  g.ey0 = e0[1];
  g.ez0 = e0[2];
  g.nex = e1[0] - e0[0] + 1;
  g.ney = e1[1] - e0[1] + 1;
  g.nez = e1[2] - e0[2] + 1;
  g.nelem = (int64_t)g.nex * g.ney * g.nez;
  g.bc_type = o.bc_type;
  g.lx = o.lx;
  g.lz = o.lz;
  // src/init.c:137-141
  g.dx = o.lx / (o.NX - 1);
  c.dy = o.ly / (o.NY - 1);
  g.dz = o.lz / (o.NZ - 1);
  g.wg = g.dx * c.dy * g.dz / NPE;
  g.rad = o.rad;
  c.ngroups = (g.nown + GROUP - 1) / GROUP;
  // sbaij storage: padded box with 64-aligned rows so every x-line of owned nodes starts a
  // 64-node group (a wave's loads never straddle two groups); node (i, j, k), i in -1..nx, at
  // 64 + i + (j+1)*UX + (k+1)*UXY (i = -1 lands in the unused last column of the row before)
  g.UX = (g.nx + 2 + GROUP - 1) / GROUP * GROUP;
  g.UXY = g.UX * g.PY;
  g.ncu = 256;
  c.npgroups = (GROUP + (int64_t)g.UXY * g.PZ + GROUP - 1) / GROUP;
  return 0;
}

// sbaij: values stored for the owned rows = 6 per node + 9 per in-domain upper neighbour
int64_t count_upper_values(const Ctx& c) {
  const Geo& g = c.g;
  auto cnt = [](int s, int w, int N, int d) {
    int64_t t = 0;
    for (int i = s; i < s + w; i++) t += (i + d >= 0 && i + d < N);
    return t;
  };
  int64_t tot = 6 * (int64_t)g.nown;
  for (int nb = 14; nb < 27; nb++)
    tot += 9 * cnt(g.xs, g.nx, g.NX, nb % 3 - 1) * cnt(g.ys, g.ny, g.NY, (nb / 3) % 3 - 1) *
           cnt(g.zs, g.nz, g.NZ, nb / 9 - 1);
  return tot;
}

int64_t petsc_node(const Ctx& c, int64_t i, int64_t j, int64_t k) {
  int a = 0, b = 0, d = 0;
  while (a + 1 < c.m && c.sx[a + 1] <= i) a++;
  while (b + 1 < c.n && c.sy[b + 1] <= j) b++;
  while (d + 1 < c.p && c.sz[d + 1] <= k) d++;
  int r = a + b * c.m + d * c.m * c.n;
  return c.rank_node_off[r] + (i - c.sx[a]) + (j - c.sy[b]) * c.wx[a] + (k - c.sz[d]) * c.wx[a] * c.wy[b];
}

int64_t count_nnz_rows(const Ctx& c, int64_t xs, int64_t ys, int64_t zs, int64_t nx, int64_t ny, int64_t nz) {
  // rows x 3 columns per in-domain neighbour node; separable per dimension
  auto sum1 = [](int64_t s, int64_t w, int64_t N) {
    int64_t t = 0;
    for (int64_t i = s; i < s + w; i++) t += (i > 0) + 1 + (i < N - 1);
    return t;
  };
  return 9 * sum1(xs, nx, c.o.NX) * sum1(ys, ny, c.o.NY) * sum1(zs, nz, c.o.NZ);
}

void plan_halo(Ctx& c, std::vector<int>& sidx, std::vector<int>& ridx) {
  HaloPlan& h = c.halo;
  const Geo& g = c.g;
  h.nbr_rank.clear();
  h.send_off.clear();
  h.send_cnt.clear();
  h.recv_off.clear();
  h.recv_cnt.clear();
  sidx.clear();
  ridx.clear();
  for (int dz = -1; dz <= 1; dz++)
    for (int dy = -1; dy <= 1; dy++)
      for (int dx = -1; dx <= 1; dx++) {
        if (!dx && !dy && !dz) continue;
        int qi = c.pi + dx, qj = c.pj + dy, qk = c.pk + dz;
        if (qi < 0 || qj < 0 || qk < 0 || qi >= c.m || qj >= c.n || qk >= c.p) continue;
        int nr = qi + qj * c.m + qk * c.m * c.n;
        int lo[3], hi[3], glo[3], ghi[3];
        int d3[3] = {dx, dy, dz}, n3[3] = {g.nx, g.ny, g.nz};
        for (int a = 0; a < 3; a++) {
          // padded coordinates: owned = 1..n, ghost = 0 and n+1
          if (d3[a] < 0) { lo[a] = 1; hi[a] = 2; glo[a] = 0; ghi[a] = 1; }
          else if (d3[a] > 0) { lo[a] = n3[a]; hi[a] = n3[a] + 1; glo[a] = n3[a] + 1; ghi[a] = n3[a] + 2; }
          else { lo[a] = 1; hi[a] = n3[a] + 1; glo[a] = 1; ghi[a] = n3[a] + 1; }
        }
        h.nbr_rank.push_back(nr);
        h.send_off.push_back((int64_t)sidx.size());
        h.recv_off.push_back((int64_t)ridx.size());
        for (int k = lo[2]; k < hi[2]; k++)
          for (int j = lo[1]; j < hi[1]; j++)
            for (int i = lo[0]; i < hi[0]; i++) sidx.push_back(i + j * g.PX + k * g.PX * g.PY);
        for (int k = glo[2]; k < ghi[2]; k++)
          for (int j = glo[1]; j < ghi[1]; j++)
            for (int i = glo[0]; i < ghi[0]; i++) ridx.push_back(i + j * g.PX + k * g.PX * g.PY);
        h.send_cnt.push_back((int64_t)sidx.size() - h.send_off.back());
        h.recv_cnt.push_back((int64_t)ridx.size() - h.recv_off.back());
      }
  h.nsend = (int64_t)sidx.size();
  h.nrecv = (int64_t)ridx.size();
}

int64_t pad_to_natural(const Ctx& c, int p) {
  const Geo& g = c.g;
  int i = p % g.PX, j = (p / g.PX) % g.PY, k = p / (g.PX * g.PY);
  int64_t gi = g.xs + i - 1, gj = g.ys + j - 1, gk = g.zs + k - 1;
  return gi + gj * (int64_t)g.NX + gk * (int64_t)g.NX * g.NY;
}

// Box-stencil forward halo: for every existing neighbour direction, the owned boundary slab
// is sent and the matching ghost slab of the padded box is received.  Both sides enumerate
// their region k, j, i ascending, so the message needs no index exchange.
int build_halo_plan(Ctx& c) {
  HaloPlan& h = c.halo;
  std::vector<int> sidx, ridx;
  plan_halo(c, sidx, ridx);
  if (h.nsend == 0) return 0;
  MCX_HIP(hipMalloc(&h.d_send_idx, sizeof(int) * h.nsend));
  MCX_HIP(hipMalloc(&h.d_recv_idx, sizeof(int) * h.nrecv));
  MCX_HIP(hipMalloc(&h.d_sendbuf, sizeof(double) * 3 * h.nsend));
  MCX_HIP(hipMalloc(&h.d_recvbuf, sizeof(double) * 3 * h.nrecv));
  MCX_HIP(hipMemcpy(h.d_send_idx, sidx.data(), sizeof(int) * h.nsend, hipMemcpyHostToDevice));
  MCX_HIP(hipMemcpy(h.d_recv_idx, ridx.data(), sizeof(int) * h.nrecv, hipMemcpyHostToDevice));
  c.device_bytes += (int64_t)(sizeof(int) + 3 * sizeof(double)) * (h.nsend + h.nrecv);
  // the sent nodes once each, as owned indices (their p update runs before the exchange)
  const Geo& g = c.g;
  std::vector<int> bnd(sidx);
  std::sort(bnd.begin(), bnd.end());
  bnd.erase(std::unique(bnd.begin(), bnd.end()), bnd.end());
  for (int& p : bnd) {
    const int pi = p % g.PX, pj = (p / g.PX) % g.PY, pk = p / (g.PX * g.PY);
    p = (pi - 1) + (pj - 1) * g.nx + (pk - 1) * g.nx * g.ny;
  }
  h.nbnd = (int64_t)bnd.size();
  MCX_HIP(hipMalloc(&h.d_bnd, sizeof(int) * h.nbnd));
  MCX_HIP(hipMemcpy(h.d_bnd, bnd.data(), sizeof(int) * h.nbnd, hipMemcpyHostToDevice));
  c.device_bytes += (int64_t)sizeof(int) * h.nbnd;
  return 0;
}

// Strain-displacement matrix of the unit reference hex at each Gauss point, the quantity
// calc_B (src/assembly.c:195-254) returns: dN_a/dxi_m = s_am * prod_{m'!=m} (1 + s_am' xg_m')
// / 8 * 2 with xg = +-0.577350269189626 (include/macroc.h:52,61-69), node order
// (---,+--,++-,-+-,--+,+-+,+++,-++), Voigt rows xx,yy,zz,xy,xz,yz (engineering shear).
// Each factor is formed as (1 + s*xg) (exact same IEEE value as the reference's 1 -/+ xg) and
// the product is rounded left to right like the reference expression.
void compute_B_table(double B[8][6][24]) {
  static const int S[8][3] = {{-1, -1, -1}, {1, -1, -1}, {1, 1, -1}, {-1, 1, -1},
                              {-1, -1, 1},  {1, -1, 1},  {1, 1, 1},  {-1, 1, 1}};
  const double X = 0.577350269189626;
  for (int gp = 0; gp < 8; gp++) {
    double xg[3] = {S[gp][0] * X, S[gp][1] * X, S[gp][2] * X};
    for (int a = 0; a < 8; a++) {
      double f[3];
      for (int m = 0; m < 3; m++) f[m] = 1 + S[a][m] * xg[m];
      double dN[3];
      dN[0] = (double)S[a][0] * f[1] * f[2] / 8. * 2. / 1.;
      dN[1] = (double)S[a][1] * f[0] * f[2] / 8. * 2. / 1.;
      dN[2] = (double)S[a][2] * f[0] * f[1] / 8. * 2. / 1.;
      for (int k = 0; k < 6; k++)
        for (int d = 0; d < 3; d++) B[gp][k][3 * a + d] = 0.;
      B[gp][0][3 * a + 0] = dN[0];
      B[gp][1][3 * a + 1] = dN[1];
      B[gp][2][3 * a + 2] = dN[2];
      B[gp][3][3 * a + 0] = dN[1];
      B[gp][3][3 * a + 1] = dN[0];
      B[gp][4][3 * a + 0] = dN[2];
      B[gp][4][3 * a + 2] = dN[0];
      B[gp][5][3 * a + 1] = dN[2];
      B[gp][5][3 * a + 2] = dN[1];
    }
  }
}

}  // namespace mcx
