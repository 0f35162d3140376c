"""ctypes view of the CPU oracle (oracle/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, as the checker / the timed CPU restatement of the reference path.  The
product (macroc_amd) never imports this module.  See oracle.h for citations and pinning.
"""
import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

BC_BENDING, BC_CIRCLE = 0, 1


class Opts(C.Structure):
    _fields_ = [
        ("NX", C.c_int64), ("NY", C.c_int64), ("NZ", C.c_int64),
        ("m", C.c_int), ("n", C.c_int), ("p", C.c_int), ("nranks", C.c_int),
        ("lx", C.c_double), ("ly", C.c_double), ("lz", C.c_double),
        ("dt", C.c_double), ("final_time", C.c_double),
        ("ts", C.c_int), ("bc_type", C.c_int), ("rad", C.c_double),
        ("newton_max_its", C.c_int), ("newton_min_tol", C.c_double), ("newton_rel_tol", C.c_double),
        ("rtol", C.c_double), ("abstol", C.c_double), ("dtol", C.c_double), ("maxits", C.c_int),
        ("E", C.c_double), ("nu", C.c_double), ("Sy", C.c_double), ("Ka", C.c_double), ("law", C.c_int),
    ]


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def use_library(path):
    """Load the oracle from another build of oracle.c (bench.py's -O3 -march=native timing
    build); must be called before the first lib()."""
    global _LIB
    if _LIB is not None:
        raise RuntimeError("oracle library already loaded")
    lib(path)


def lib(path=None):
    global _LIB
    if _LIB is None:
        path = path or os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        L = C.CDLL(path)
        P = C.c_void_p
        d = C.POINTER(C.c_double)
        L.orc_default_opts.argtypes = [C.POINTER(Opts)]
        L.orc_create.argtypes = [C.POINTER(Opts)]
        L.orc_create.restype = P
        L.orc_destroy.argtypes = [P]
        for fn in ("orc_ndofs", "orc_nnz", "orc_ngp"):
            getattr(L, fn).argtypes = [P]
            getattr(L, fn).restype = C.c_int64
        L.orc_get_decomp.argtypes = [P, C.POINTER(C.c_int)]
        L.orc_rank_corners.argtypes = [P, C.c_int, C.POINTER(C.c_int64)]
        L.orc_rank_nelem.argtypes = [P, C.c_int]
        L.orc_rank_nelem.restype = C.c_int64
        L.orc_rank_dof_offset.argtypes = [P, C.c_int]
        L.orc_rank_dof_offset.restype = C.c_int64
        L.orc_wg.argtypes = [P]
        L.orc_wg.restype = C.c_double
        L.orc_dof_map.argtypes = [P, C.POINTER(C.c_int64)]
        L.orc_rank_elements.argtypes = [P, C.c_int, C.POINTER(C.c_int32)]
        L.orc_rank_dirichlet.argtypes = [P, C.c_int, C.POINTER(C.c_int64), C.c_int64]
        L.orc_rank_dirichlet.restype = C.c_int64
        L.orc_dirichlet_set.argtypes = [P, C.POINTER(C.c_int64), C.c_int64]
        L.orc_dirichlet_set.restype = C.c_int64
        L.orc_csr_pattern.argtypes = [P, C.POINTER(C.c_int64), C.POINTER(C.c_int32)]
        L.orc_calc_B.argtypes = [C.c_int, d]
        for fn in ("orc_u", "orc_b", "orc_du", "orc_A_values", "orc_strain", "orc_stress"):
            getattr(L, fn).argtypes = [P]
            getattr(L, fn).restype = d
        L.orc_get_displacement.argtypes = [P, C.c_int]
        L.orc_get_displacement.restype = C.c_double
        L.orc_apply_bc_u.argtypes = [P, C.c_double]
        for fn in ("orc_set_strains", "orc_homogenize", "orc_assembly_res", "orc_assembly_jac", "orc_update_u",
                   "orc_sbaij_mirror", "orc_update_vars"):
            getattr(L, fn).argtypes = [P]
        L.orc_norm2.argtypes = [P, d]
        L.orc_norm2.restype = C.c_double
        L.orc_spmv.argtypes = [P, d, d]
        L.orc_spmv_order.argtypes = [P, d, d, C.c_int]
        L.orc_solve.argtypes = [P, C.POINTER(C.c_int), C.POINTER(C.c_double), C.POINTER(C.c_int), d]
        L.orc_dmda_decide.argtypes = [C.c_int64, C.c_int64, C.c_int64, C.c_int,
                                      C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int)]
        L.orc_run.argtypes = [P, C.c_char_p, d]
        L.orc_run_files.argtypes = [P, C.c_char_p, C.c_char_p, C.c_char_p, d]
        L.orc_write_vtu.argtypes = [P, C.c_char_p]
        L.orc_calc_force.argtypes = [P]
        L.orc_calc_force.restype = C.c_double
        L.orc_rank_nonlinear_gps.argtypes = [P, C.c_int]
        L.orc_rank_nonlinear_gps.restype = C.c_int64
        L.orc_nonlinear_gps.argtypes = [P, d]
        L.orc_nonlinear_gps.restype = C.c_int64
        L.orc_ctan.argtypes = [P]
        L.orc_ctan.restype = d
        L.orc_set_threads.argtypes = [C.c_int]
        L.orc_set_threads.restype = C.c_int
        L.orc_petsc_numbering.argtypes = [C.c_int64, C.c_int64, C.c_int64, C.c_int, C.c_int, C.c_int, C.c_int,
                                          C.POINTER(C.c_int64)]
        _LIB = L
    return _LIB


def _dp(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def calc_B(gp):
    B = np.zeros((6, 24), dtype=np.float64)
    lib().orc_calc_B(gp, _dp(B))
    return B


def dmda_decide(M, N, P, size, m=0, n=0, p=0):
    mm, nn, pp = C.c_int(m), C.c_int(n), C.c_int(p)
    rc = lib().orc_dmda_decide(M, N, P, size, C.byref(mm), C.byref(nn), C.byref(pp))
    if rc:
        raise ValueError(f"no DMDA partition (code {rc})")
    return mm.value, nn.value, pp.value


def set_threads(n):
    """OpenMP threads for the emulated ranks; returns the thread count in effect."""
    return lib().orc_set_threads(int(n))


def petsc_numbering(M, N, P, size, m=0, n=0, p=0):
    """natural node index -> PETSc global node index (DMDA, any dims)."""
    out = np.zeros(M * N * P, dtype=np.int64)
    rc = lib().orc_petsc_numbering(M, N, P, size, m, n, p, out.ctypes.data_as(C.POINTER(C.c_int64)))
    if rc:
        raise ValueError("no partition")
    return out


class Problem:
    """The global MacroC problem (PETSc global ordering), emulated over `nranks`."""

    def __init__(self, NX, NY, NZ, nranks=1, m=0, n=0, p=0, **kw):
        L = lib()
        o = Opts()
        L.orc_default_opts(C.byref(o))
        o.NX, o.NY, o.NZ, o.nranks, o.m, o.n, o.p = NX, NY, NZ, nranks, m, n, p
        for k, v in kw.items():
            setattr(o, k, v)
        self.opts = o
        self._p = L.orc_create(C.byref(o))
        if not self._p:
            raise ValueError("oracle: bad options / partition")
        self.ndofs = L.orc_ndofs(self._p)
        self.nnz = L.orc_nnz(self._p)
        self.ngp = L.orc_ngp(self._p)
        self.nranks = nranks

    def close(self):
        if self._p:
            lib().orc_destroy(self._p)
            self._p = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- integer artefacts
    def decomp(self):
        a = (C.c_int * 3)()
        lib().orc_get_decomp(self._p, a)
        return tuple(a)

    def corners(self, r):
        a = (C.c_int64 * 12)()
        lib().orc_rank_corners(self._p, r, a)
        return tuple(a)

    def wg(self):
        return lib().orc_wg(self._p)

    def dof_offset(self, r):
        return lib().orc_rank_dof_offset(self._p, r)

    def dof_map(self):
        m = np.zeros(self.ndofs, dtype=np.int64)
        lib().orc_dof_map(self._p, m.ctypes.data_as(C.POINTER(C.c_int64)))
        return m

    def elements(self, r):
        ne = lib().orc_rank_nelem(self._p, r)
        c = np.zeros(ne * 8, dtype=np.int32)
        lib().orc_rank_elements(self._p, r, c.ctypes.data_as(C.POINTER(C.c_int32)))
        return c.reshape(ne, 8)

    def rank_dirichlet(self, r):
        n = lib().orc_rank_dirichlet(self._p, r, None, 0)
        a = np.zeros(max(n, 1), dtype=np.int64)
        lib().orc_rank_dirichlet(self._p, r, a.ctypes.data_as(C.POINTER(C.c_int64)), n)
        return a[:n]

    def dirichlet_set(self):
        n = lib().orc_dirichlet_set(self._p, None, 0)
        a = np.zeros(max(n, 1), dtype=np.int64)
        lib().orc_dirichlet_set(self._p, a.ctypes.data_as(C.POINTER(C.c_int64)), n)
        return a[:n]

    def csr(self):
        rp = np.zeros(self.ndofs + 1, dtype=np.int64)
        ci = np.zeros(self.nnz, dtype=np.int32)
        lib().orc_csr_pattern(self._p, rp.ctypes.data_as(C.POINTER(C.c_int64)),
                              ci.ctypes.data_as(C.POINTER(C.c_int32)))
        return rp, ci

    # ---- state views (copies)
    def _vec(self, fn, n):
        ptr = getattr(lib(), fn)(self._p)
        return np.ctypeslib.as_array(ptr, shape=(n,)).copy()

    def u(self):
        return self._vec("orc_u", self.ndofs)

    def b(self):
        return self._vec("orc_b", self.ndofs)

    def du(self):
        return self._vec("orc_du", self.ndofs)

    def A_values(self):
        return self._vec("orc_A_values", self.nnz)

    def strain(self):
        return self._vec("orc_strain", self.ngp * 6).reshape(self.ngp, 6)

    def stress(self):
        return self._vec("orc_stress", self.ngp * 6).reshape(self.ngp, 6)

    def set_u(self, u):
        ptr = lib().orc_u(self._p)
        np.ctypeslib.as_array(ptr, shape=(self.ndofs,))[:] = u

    # ---- steps
    def get_displacement(self, time_s):
        return lib().orc_get_displacement(self._p, time_s)

    def apply_bc_u(self, U):
        lib().orc_apply_bc_u(self._p, U)

    def set_strains(self):
        lib().orc_set_strains(self._p)

    def homogenize(self):
        lib().orc_homogenize(self._p)

    def assembly_res(self):
        lib().orc_assembly_res(self._p)
        return self.b()

    def norm_b(self):
        return lib().orc_norm2(self._p, lib().orc_b(self._p))

    def assembly_jac(self):
        lib().orc_assembly_jac(self._p)

    def update_vars(self):
        lib().orc_update_vars(self._p)

    def nonlinear_gps(self):
        fm = np.zeros(1)
        n = lib().orc_nonlinear_gps(self._p, _dp(fm))
        return n, float(fm[0])

    def ctan(self):
        return self._vec("orc_ctan", self.ngp * 36).reshape(self.ngp, 36)

    def sbaij_mirror(self):
        """-dm_mat_type sbaij semantics: lower triangle := transpose of the upper triangle."""
        lib().orc_sbaij_mirror(self._p)

    def spmv(self, x, order=None):
        """MatMult.  order None: the problem's (the MATAIJ inode kernel's column pairs; after
        sbaij_mirror the plain loop), "inode", or "plain" (MatMult_SeqAIJ, one term at a time)."""
        x = np.ascontiguousarray(x, dtype=np.float64)
        y = np.zeros(self.ndofs)
        if order is None:
            lib().orc_spmv(self._p, _dp(x), _dp(y))
        else:
            lib().orc_spmv_order(self._p, _dp(x), _dp(y), {"inode": 0, "plain": 1}[order])
        return y

    def solve(self, history=False):
        its, rn, reason = C.c_int(), C.c_double(), C.c_int()
        h = np.zeros(self.opts.maxits + 2)
        lib().orc_solve(self._p, C.byref(its), C.byref(rn), C.byref(reason), _dp(h))
        out = dict(its=its.value, rnorm=rn.value, reason=reason.value)
        if history:
            out["history"] = h[: its.value + 1].copy()
        return out

    def update_u(self):
        lib().orc_update_u(self._p)

    def run(self, log_path=None, info_path=None, gauss_path=None):
        """src/main.c:49-109: time loop, Newton loop, post-processing rows (info.dat,
        gauss_evolution.dat)."""
        t = np.zeros(1)
        enc = lambda s: s.encode() if s else None  # noqa: E731
        lib().orc_run_files(self._p, enc(log_path), enc(info_path), enc(gauss_path), _dp(t))
        return float(t[0])

    def calc_force(self):
        """calc_force src/forces.c:25-166 (rank partials summed in rank order)."""
        return lib().orc_calc_force(self._p)

    def write_vtu(self, prefix):
        """write_pvtu src/output.c:25-267 for every emulated rank."""
        assert lib().orc_write_vtu(self._p, str(prefix).encode()) == 0

    def rank_nonlinear_gps(self, r):
        return lib().orc_rank_nonlinear_gps(self._p, r)

    def newton_step1(self):
        """Time step 1, Newton iteration 0 of src/main.c (the path that solves).
        Returns a dict with |RES|, its, rnorm, reason; leaves u updated."""
        self.apply_bc_u(self.get_displacement(0))
        U = self.get_displacement(1)
        self.apply_bc_u(U)
        self.set_strains()
        self.homogenize()
        self.assembly_res()
        res = self.norm_b()
        self.assembly_jac()
        out = self.solve(history=True)
        self.update_u()
        out["res"] = res
        out["U"] = U
        return out
