"""Independent numpy/scipy restatement of MacroC's hot path + golden-fixture generator.

Why this exists: the reference (GG1991/macroc) needs PETSc and MicroPP, neither of which is
in this container or on the GPU box, so it cannot be run to produce vectors.
The C oracle (oracle/oracle.c) is therefore pinned two ways:
  1. the one known answer the reference holds — PETSc vs natural ordering of a 5x2 DMDA on 2
     ranks (tests/test_dm_1.c:5-19), checked in tests/test_oracle.py;
  2. this file: a second, independently written restatement (vectorised numpy + scipy.sparse,
     analytic formulas instead of the reference's loops) that must agree with the oracle —
     bit-exact on every integer artefact, to ~1e-12 on floating point — before fixtures are
     written.  A direct sparse solve (spsolve) checks the CG answer.
Fixtures (tests/golden/*.npz, allow_pickle=False) hold inputs' descriptors and outputs only.

Run:  python tests/golden/make_golden.py      (rewrites tests/golden/*.npz)
"""
import hashlib
import os
import sys

import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as spla

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

CONSTXG = 0.577350269189626  # include/macroc.h:52
NODE_SIGNS = np.array([[-1, -1, -1], [1, -1, -1], [1, 1, -1], [-1, 1, -1],
                       [-1, -1, 1], [1, -1, 1], [1, 1, 1], [-1, 1, 1]], dtype=np.float64)
GP_SIGNS = NODE_SIGNS  # xg[gp] = CONSTXG * sign (include/macroc.h:61-69)


# ----------------------------------------------------------------- DMDA (independent)
def widths(M, m):
    return np.array([M // m + ((M % m) > i) for i in range(m)], dtype=np.int64)


def decide(M, N, P, size, m=0, n=0, p=0):
    """PETSc da3.c PETSC_DECIDE (restated independently of oracle.c)."""
    D = 0
    if m and n and p:
        pass
    elif not m and n and p:
        m = size // (n * p)
    elif m and not n and p:
        n = size // (m * p)
    elif m and n and not p:
        p = size // (m * n)
    elif not m and not n and p:
        m = max(int(0.5 + np.sqrt(M * size / (N * p))), 1)
        while m > 0:
            n = size // (m * p)
            if m * n * p == size:
                break
            m -= 1
        if M > N and m < n:
            m, n = n, m
    elif not m and n and not p:
        m = max(int(0.5 + np.sqrt(M * size / (P * n))), 1)
        while m > 0:
            p = size // (m * n)
            if m * n * p == size:
                break
            m -= 1
        if M > P and m < p:
            m, p = p, m
    elif m and not n and not p:
        n = max(int(0.5 + np.sqrt(N * size / (P * m))), 1)
        while n > 0:
            p = size // (m * n)
            if m * n * p == size:
                break
            n -= 1
        if N > P and n < p:
            n, p = p, n
    else:
        n = max(int(0.5 + (N * N * size / (P * M)) ** (1.0 / 3.0)), 1)
        while n > 0:
            if size % n == 0:
                break
            n -= 1
        n = max(n, 1)
        m = max(int(0.5 + np.sqrt(M * size / (P * n))), 1)
        while m > 0:
            p = size // (m * n)
            if m * n * p == size:
                break
            m -= 1
        if M > P and m < p:
            m, p = p, m
    assert m * n * p == size, "no partition"
    return m, n, p


class Grid:
    def __init__(self, NX, NY, NZ, nranks=1, m=0, n=0, p=0):
        self.NX, self.NY, self.NZ = NX, NY, NZ
        self.m, self.n, self.p = decide(NX, NY, NZ, nranks, m, n, p)
        self.nranks = nranks
        self.w = [widths(NX, self.m), widths(NY, self.n), widths(NZ, self.p)]
        self.s = [np.concatenate([[0], np.cumsum(w)[:-1]]) for w in self.w]
        # processor coordinate of every node index, per dim
        self.pc = [np.repeat(np.arange(len(w)), w) for w in self.w]
        sizes = np.array([self.w[0][r % self.m] * self.w[1][(r % (self.m * self.n)) // self.m]
                          * self.w[2][r // (self.m * self.n)] for r in range(nranks)], dtype=np.int64)
        self.node_off = np.concatenate([[0], np.cumsum(sizes)])
        k, j, i = np.meshgrid(np.arange(NZ), np.arange(NY), np.arange(NX), indexing="ij")
        self.nat_to_petsc_node = self.petsc_node(i.ravel(), j.ravel(), k.ravel())

    def petsc_node(self, i, j, k):
        pi, pj, pk = self.pc[0][i], self.pc[1][j], self.pc[2][k]
        r = pi + pj * self.m + pk * self.m * self.n
        nx, ny = self.w[0][pi], self.w[1][pj]
        return self.node_off[r] + (i - self.s[0][pi]) + (j - self.s[1][pj]) * nx + (k - self.s[2][pk]) * nx * ny

    def rank_of_node(self, i, j, k):
        return self.pc[0][i] + self.pc[1][j] * self.m + self.pc[2][k] * self.m * self.n

    def dof_map(self):
        g = self.nat_to_petsc_node
        return (3 * g[:, None] + np.arange(3)[None, :]).ravel()

    def elements(self):
        """All elements (natural order) with owner rank = owner of the upper node (i+1,j+1,k+1)."""
        ez, ey, ex = np.meshgrid(np.arange(self.NZ - 1), np.arange(self.NY - 1), np.arange(self.NX - 1), indexing="ij")
        ex, ey, ez = ex.ravel(), ey.ravel(), ez.ravel()
        owner = self.rank_of_node(ex + 1, ey + 1, ez + 1)
        nodes = np.stack([self.petsc_node(ex + (s[0] > 0), ey + (s[1] > 0), ez + (s[2] > 0)) for s in NODE_SIGNS], 1)
        return nodes, owner, (ex, ey, ez)


# ----------------------------------------------------------------- element (independent)
def bmats():
    """B[gp] (6x24) from dN_a/dxi = s_a (1+eta s_a')(1+zeta s_a'')/8 * 2 (unit cube)."""
    out = np.zeros((8, 6, 24))
    for g in range(8):
        xi = CONSTXG * GP_SIGNS[g]
        for a in range(8):
            s = NODE_SIGNS[a]
            f = 1.0 + xi * s
            dN = np.array([s[0] * f[1] * f[2], s[1] * f[0] * f[2], s[2] * f[0] * f[1]]) / 8.0 * 2.0
            c = 3 * a
            out[g, 0, c] = dN[0]
            out[g, 1, c + 1] = dN[1]
            out[g, 2, c + 2] = dN[2]
            out[g, 3, c], out[g, 3, c + 1] = dN[1], dN[0]
            out[g, 4, c], out[g, 4, c + 2] = dN[2], dN[0]
            out[g, 5, c + 1], out[g, 5, c + 2] = dN[2], dN[1]
    return out


def elastic_C(E=1e7, nu=0.25):
    lam = E * nu / ((1 + nu) * (1 - 2 * nu))
    mu = E / (2 * (1 + nu))
    C = np.zeros((6, 6))
    C[:3, :3] = lam
    C[np.arange(3), np.arange(3)] += 2 * mu
    C[np.arange(3, 6), np.arange(3, 6)] = mu
    return C


class System:
    def __init__(self, grid, lx=50.0, ly=1.0, lz=50.0, dt=0.001, bc_type=1, rad=1.0):
        self.g = grid
        NX, NY, NZ = grid.NX, grid.NY, grid.NZ
        self.dx, self.dy, self.dz = lx / (NX - 1), ly / (NY - 1), lz / (NZ - 1)
        self.wg = self.dx * self.dy * self.dz / 8
        self.n = 3 * NX * NY * NZ
        B = bmats()
        C = elastic_C()
        self.Ke = self.wg * np.einsum("gki,kl,glj->ij", B, C, B)
        nodes, owner, _ = grid.elements()
        dofs = (3 * nodes[:, :, None] + np.arange(3)[None, None, :]).reshape(len(nodes), 24)
        self.edofs = dofs
        rows = np.repeat(dofs, 24, axis=1).ravel()
        cols = np.tile(dofs, (1, 24)).ravel()
        vals = np.tile(self.Ke.ravel(), len(nodes))
        self.K = sp.csr_matrix((vals, (rows, cols)), shape=(self.n, self.n))
        self.K.sort_indices()
        # Dirichlet set, analytic (bcs.c:254-338 union over ranks)
        k, j, i = np.meshgrid(np.arange(NZ), np.arange(NY), np.arange(NX), indexing="ij")
        i, j, k = i.ravel(), j.ravel(), k.ravel()
        gn = grid.petsc_node(i, j, k)
        if bc_type == 1:
            edge = (j == 0) & ((i == 0) | (i == NX - 1) | (k == 0) | (k == NZ - 1))
            x = lx / 2.0 - (i * self.dx + self.dx / 2.0)
            z = lz / 2.0 - (k * self.dz + self.dz / 2.0)
            circ = (j == NY - 1) & ((x * x + z * z) < rad * rad)
            dset = np.concatenate([(3 * gn[edge][:, None] + np.arange(3)).ravel(), 3 * gn[circ] + 1])
            self.dir = np.unique(dset)
            self.dir_vals = lambda U: (np.concatenate([np.zeros(3 * edge.sum()), np.full(circ.sum(), U)]),
                                       np.concatenate([(3 * gn[edge][:, None] + np.arange(3)).ravel(), 3 * gn[circ] + 1]))
        else:
            x0 = (i == 0)
            x1 = (i == NX - 1)
            idx0 = (3 * gn[x0][:, None] + np.arange(3)).ravel()
            idx1 = (3 * gn[x1][:, None] + np.arange(3)).ravel()
            self.dir = np.unique(np.concatenate([idx0, idx1]))
            self.dir_vals = lambda U: (np.concatenate([np.zeros(len(idx0)), np.tile([0.0, U, 0.0], x1.sum())]),
                                       np.concatenate([idx0, idx1]))
        mask = np.zeros(self.n, dtype=bool)
        mask[self.dir] = True
        self.mask = mask
        # MatZeroRowsColumns(diag=1), pattern kept
        A = self.K.tocoo()
        keep = ~(mask[A.row] | mask[A.col])
        v = np.where(keep, A.data, 0.0)
        v = np.where(mask[A.row] & (A.row == A.col), 1.0, v)
        self.A = sp.csr_matrix((v, (A.row, A.col)), shape=self.K.shape)
        self.A.sort_indices()

    def pattern(self):
        """27-box x 3x3 clipped pattern, built from node adjacency (not from elements)."""
        g = self.g
        NX, NY, NZ = g.NX, g.NY, g.NZ
        rows, cols = [], []
        k, j, i = np.meshgrid(np.arange(NZ), np.arange(NY), np.arange(NX), indexing="ij")
        i, j, k = i.ravel(), j.ravel(), k.ravel()
        for dk in (-1, 0, 1):
            for dj in (-1, 0, 1):
                for di in (-1, 0, 1):
                    ok = (i + di >= 0) & (i + di < NX) & (j + dj >= 0) & (j + dj < NY) & (k + dk >= 0) & (k + dk < NZ)
                    a = g.petsc_node(i[ok], j[ok], k[ok])
                    b = g.petsc_node(i[ok] + di, j[ok] + dj, k[ok] + dk)
                    for r in range(3):
                        for c in range(3):
                            rows.append(3 * a + r)
                            cols.append(3 * b + c)
        rows, cols = np.concatenate(rows), np.concatenate(cols)
        M = sp.csr_matrix((np.ones(len(rows)), (rows, cols)), shape=(self.n, self.n))
        M.sort_indices()
        return M.indptr.astype(np.int64), M.indices.astype(np.int32)

    def u_step1(self, dt=0.001):
        U = -1.0 * (1 * dt / 1.0)
        u = np.zeros(self.n)
        vals, idx = self.dir_vals(U)
        u[idx] = vals
        return u, U

    def residual(self, u):
        b = -(self.K @ u)
        b[self.mask] = 0.0
        return b

    def cg_petsc(self, b, rtol=1e-5, abstol=1e-50, dtol=1e4, maxits=10000):
        """KSPSolve_CG + PCJacobi, preconditioned norm (numpy restatement)."""
        d = self.A.diagonal().copy()
        dinv = np.where(d != 0, 1.0 / np.where(d != 0, d, 1.0), 1.0)
        x = np.zeros_like(b)
        r = b.copy()
        z = r * dinv
        dp = np.linalg.norm(z)
        hist = [dp]
        ttol, rn0 = max(rtol * dp, abstol), dp
        if dp <= ttol:
            return x, 0, hist
        beta = z @ r
        its = 0
        p = None
        dpi = 0.0
        betaold = 0.0
        for i in range(maxits):
            its = i + 1
            if beta == 0.0:
                break
            p = z.copy() if i == 0 else z + (beta / betaold) * p
            dpiold = dpi
            w = self.A @ p
            dpi = p @ w
            betaold = beta
            assert dpi > 0 and (i == 0 or dpi * dpiold > 0)
            a = beta / dpi
            x = x + a * p
            r = r - a * w
            z = r * dinv
            dp = np.linalg.norm(z)
            hist.append(dp)
            if dp <= ttol or dp >= dtol * rn0:
                break
            beta = z @ r
        return x, its, hist


# ----------------------------------------------------------------- MatMult row orders
def _row_sums(indptr, t, sel, s0, inode):
    """Per row: s0 + the selected terms (CSR order = ascending column) of t, either one at a time
    (MatMult_SeqAIJ) or in column pairs, sum + (t0 + t1) + (t2 + t3) + ... + t_last
    (MatMult_SeqAIJ_Inode's unrolled loop [ext]).  Vectorised over rows: pair sums first, then
    one pass per pair index, so every row's additions happen in its own order."""
    n = len(indptr) - 1
    rows = np.repeat(np.arange(n), np.diff(indptr))
    r, tt = rows[sel], t[sel]
    cnt = np.bincount(r, minlength=n)
    start = np.concatenate([[0], np.cumsum(cnt)[:-1]]).astype(np.int64)
    pos = np.arange(len(r)) - start[r]
    s = np.array(s0, dtype=np.float64, copy=True)
    if not inode:
        for k in range(int(cnt.max()) if n else 0):
            m = pos == k
            s[r[m]] = s[r[m]] + tt[m]
        return s
    first = np.nonzero((pos % 2 == 0) & (pos + 1 < cnt[r]))[0]
    ps, pr, pk = tt[first] + tt[first + 1], r[first], pos[first] // 2
    for k in range(int(pk.max()) + 1 if len(pk) else 0):
        m = pk == k
        s[pr[m]] = s[pr[m]] + ps[m]
    odd = cnt % 2 == 1
    s[odd] = s[odd] + tt[(start + cnt - 1)[odd]]
    return s


def spmv(indptr, indices, data, x, dof_off=None, inode=True):
    """MatMult of a CSR matrix in PETSc numbering, restated independently of oracle.c: one rank
    (dof_off None) = the SeqAIJ kernel over each row; several = MatMult_MPIAIJ, the owned-column
    block then MatMultAdd of the off-diagonal block from that sum — term by term whatever
    `inode` says: MatAssemblyEnd_MPIAIJ sets MAT_USE_INODES false on the off-diagonal block."""
    t = data * x[indices]
    n = len(indptr) - 1
    if dof_off is None:
        return _row_sums(indptr, t, np.ones(len(t), dtype=bool), np.zeros(n), inode)
    rows = np.repeat(np.arange(n), np.diff(indptr))
    rk = np.searchsorted(dof_off, rows, side="right") - 1
    own = (indices >= dof_off[rk]) & (indices < dof_off[rk + 1])
    s = _row_sums(indptr, t, own, np.zeros(n), inode)
    return _row_sums(indptr, t, ~own, s, False)


# ----------------------------------------------------------------- fixtures
CASES = [
    # name, grid, nranks, decomposition (0 = decide), ksp_rtol
    ("g442_r1", (4, 4, 2), 1, (0, 0, 0), 1e-5),     # BASELINE config 1 (+ -ts 2)
    ("g522_r1", (5, 2, 2), 1, (0, 0, 0), 1e-5),     # ctest grid
    ("g522_r2", (5, 2, 2), 2, (0, 0, 0), 1e-5),
    ("g522_r3", (5, 2, 2), 3, (0, 0, 0), 1e-5),
    ("g522_r4", (5, 2, 2), 4, (0, 0, 0), 1e-5),
    ("g444_r1", (4, 4, 4), 1, (0, 0, 0), 1e-5),     # ctest grid with one loaded node
    ("g534_r8", (5, 3, 4), 8, (0, 0, 0), 1e-5),     # ctest medium grid, 8 ranks
    ("g888_r1", (8, 8, 8), 1, (0, 0, 0), 1e-12),
    ("g888_r8", (8, 8, 8), 8, (2, 2, 2), 1e-12),
    ("g1088_r2", (10, 8, 8), 2, (2, 1, 1), 1e-12),
    ("g16_r1", (16, 16, 16), 1, (0, 0, 0), 1e-8),
]


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def generate(write=True, verbose=True):
    from oracle import oracle as O

    summary = []
    for name, (NX, NY, NZ), nr, (m, n, p), rtol in CASES:
        g = Grid(NX, NY, NZ, nr, m, n, p)
        S = System(g)
        P = O.Problem(NX, NY, NZ, nranks=nr, m=m, n=n, p=p, rtol=rtol)
        assert P.decomp() == (g.m, g.n, g.p), (name, P.decomp(), (g.m, g.n, g.p))
        # integers, bit-exact
        dm = P.dof_map()
        assert np.array_equal(dm, g.dof_map()), name
        rp, ci = P.csr()
        rp2, ci2 = S.pattern()
        assert np.array_equal(rp, rp2) and np.array_equal(ci, ci2), name
        dset = P.dirichlet_set()
        assert np.array_equal(dset, S.dir), name
        # elements: oracle per-rank connectivity (ghosted-local) -> global nodes
        nodes, owner, _ = g.elements()
        for r in range(nr):
            conn = P.elements(r)
            c = P.corners(r)
            Xs, Ys, Zs, Nx, Ny = c[6], c[7], c[8], c[9], c[10]
            li = conn % Nx + Xs
            lj = (conn // Nx) % Ny + Ys
            lk = conn // (Nx * Ny) + Zs
            glob = g.petsc_node(li, lj, lk)
            assert np.array_equal(glob, nodes[owner == r]), (name, r)
        # floating point
        out = P.newton_step1()
        u1, U = S.u_step1()
        b_ref = S.residual(u1)
        b_orc = P.b()
        assert np.allclose(b_orc, b_ref, rtol=1e-12, atol=1e-12 * np.abs(b_ref).max()), name
        Aref = S.A
        Aorc = P.A_values()
        assert np.allclose(Aorc, Aref.data, rtol=1e-12, atol=1e-13 * np.abs(Aref.data).max()), name
        # MatMult row orders: the oracle's inode (default) and plain kernels vs this restatement,
        # bit for bit on the oracle's matrix; the inode order differs from the plain one
        xr = np.random.default_rng(7).uniform(-1, 1, P.ndofs)
        off = None if nr == 1 else np.array([P.dof_offset(r) for r in range(nr)] + [P.ndofs])
        y_in = P.spmv(xr)
        assert np.array_equal(y_in, spmv(rp, ci, Aorc, xr, off, inode=True)), name
        assert np.array_equal(P.spmv(xr, "plain"), spmv(rp, ci, Aorc, xr, off, inode=False)), name
        assert np.allclose(y_in, Aref @ xr, rtol=1e-12, atol=1e-12 * np.abs(Aref.data).max()), name
        du_direct = spla.spsolve(Aref.tocsc(), b_ref)
        du_orc = P.du()
        rel_direct = np.linalg.norm(du_orc - du_direct) / np.linalg.norm(du_direct)
        x_np, its_np, hist_np = S.cg_petsc(b_ref, rtol=rtol)
        assert abs(its_np - out["its"]) <= 1, (name, its_np, out["its"])
        rel_np = np.linalg.norm(du_orc - x_np) / np.linalg.norm(x_np)
        if rtol <= 1e-12:
            assert rel_direct < 1e-9, (name, rel_direct)
        summary.append((name, P.ndofs, P.nnz, out["its"], its_np, rel_np, rel_direct))
        if verbose:
            print(f"{name:10s} ndofs={P.ndofs:6d} nnz={P.nnz:8d} its={out['its']:4d} (numpy {its_np:4d}) "
                  f"|du-np|/|du|={rel_np:.2e} |du-direct|/|du|={rel_direct:.2e} |RES|={out['res']:.6e}")
        if write:
            conns = [P.elements(r) for r in range(nr)]
            fx = dict(
                grid=np.array([NX, NY, NZ], dtype=np.int64), nranks=np.int64(nr),
                decomp=np.array(P.decomp(), dtype=np.int64), rtol=np.float64(rtol),
                corners=np.array([P.corners(r) for r in range(nr)], dtype=np.int64),
                dof_map=dm, dirichlet=dset,
                conn=np.concatenate(conns).astype(np.int32),
                conn_counts=np.array([len(c) for c in conns], dtype=np.int64),
                csr_rowptr_sha=np.array(sha(rp)), csr_colidx_sha=np.array(sha(ci)),
                nnz=np.int64(P.nnz), res=np.float64(out["res"]), U=np.float64(out["U"]),
                its=np.int64(out["its"]), reason=np.int64(out["reason"]),
                history=out["history"], b=b_orc, du=du_orc, u=P.u(), du_direct=du_direct,
                wg=np.float64(P.wg()),
            )
            if P.nnz <= 20000:
                fx["csr_rowptr"] = rp
                fx["csr_colidx"] = ci
                fx["A"] = Aorc
            np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **fx)
        P.close()
    # known answer tests/test_dm_1.c:5-19 (2-D 5x2 DMDA on 2 ranks -> NZ=1, dof 1)
    g = Grid(5, 2, 1, 2)
    order = (g.nat_to_petsc_node).reshape(2, 5)
    assert (order == np.array([[0, 1, 2, 6, 7], [3, 4, 5, 8, 9]])).all()
    # B table: independent formula vs calc_B restatement
    Bo = np.stack([O.calc_B(gp) for gp in range(8)])
    assert np.allclose(Bo, bmats(), rtol=0, atol=1e-15)
    if write:
        np.savez_compressed(os.path.join(HERE, "calc_B.npz"), B=Bo)
    return summary


if __name__ == "__main__":
    generate(write=True)
