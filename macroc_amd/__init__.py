"""macroc_amd — MI355X-native MacroC Newton inner loop, Python host side.

The compute path is the HIP library libmacroc_amd.so (C-ABI, include/macroc_amd.h).  This
module is a thin ctypes mirror of the reference driver's functions (src/main.c, src/init.c,
src/assembly.c, src/bcs.c of GG1991/macroc) with the same names and argument meaning:

    m = Macroc(["-da_grid_x", "64", ...])       # init()            src/init.c:25
    m.apply_bc_on_u(m.get_displacement(1))      # apply_bc_on_u     src/bcs.c:29
    m.set_strains(); m.homogenize()             # set_strains + micropp_C_homogenize
    norm = m.assembly_res()                     # assembly_res + VecNorm
    m.assembly_jac()                            # assembly_jac (+ apply_bc_on_jac)
    its, rnorm, reason = m.solve_Ax()           # solve_Ax -> KSPSolve(CG, Jacobi)
    m.update_u()                                # VecAXPY(u, 1, du)
    m.finish()                                  # finish()

There is no CPU fallback: if the library is missing or no GPU is visible the calls raise.
"""
import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libmacroc_amd.so")
COMM_ID_BYTES = 128
ABI_VERSION = 3  # MCX_ABI_VERSION of include/macroc_amd.h this mirror's structs follow

BC_BENDING, BC_CIRCLE = 0, 1
KSP_REASONS = {2: "CONVERGED_RTOL", 3: "CONVERGED_ATOL", -3: "DIVERGED_ITS", -4: "DIVERGED_DTOL",
               -8: "DIVERGED_INDEFINITE_PC", -9: "DIVERGED_NANORINF", -10: "DIVERGED_INDEFINITE_MAT"}

# symbols declared in include/macroc_amd.h (checked by tests/test_abi.py)
EXPORTS = [
    "mcx_last_error", "mcx_version", "mcx_abi_version", "mcx_comm_info", "mcx_default_opts", "mcx_parse_args", "mcx_comm_unique_id", "mcx_plan", "mcx_plan_halo", "mcx_init",
    "mcx_local_group_create", "mcx_local_group_destroy", "mcx_local_group_barrier", "mcx_init_local",
    "mcx_finalize", "mcx_get_info", "mcx_material_set", "mcx_get_displacement", "mcx_zero_u", "mcx_apply_bc_u",
    "mcx_set_strains", "mcx_homogenize", "mcx_assembly_res", "mcx_assembly_jac", "mcx_solve", "mcx_update_u", "mcx_update_vars",
    "mcx_get_nonlinear_stats", "mcx_reduce_nonlinear", "mcx_calc_force", "mcx_write_vtu",
    "mcx_time_step", "mcx_get_u", "mcx_set_u", "mcx_get_b", "mcx_get_du", "mcx_get_strain", "mcx_get_stress",
    "mcx_owned_dofs", "mcx_dump_csr", "mcx_dump_dirichlet", "mcx_spmv", "mcx_get_ksp_history",
    "mcx_set_timing", "mcx_get_timing", "mcx_synchronize", "mcx_set_option", "mcx_time_spmv",
    "mcx_set_micropp", "mcx_set_device_law", "mcx_set_gp_stress", "mcx_set_gp_ctan", "mcx_get_gp_strain",
]

LAWS = {"elastic": 0, "plastic": 1, "external": 2}


class Opts(C.Structure):
    _fields_ = [
        ("NX", C.c_int64), ("NY", C.c_int64), ("NZ", C.c_int64),
        ("px", C.c_int), ("py", C.c_int), ("pz", C.c_int),
        ("lx", C.c_double), ("ly", C.c_double), ("lz", C.c_double),
        ("dt", C.c_double), ("final_time", C.c_double),
        ("ts", C.c_int), ("vtu_freq", C.c_int), ("bc_type", C.c_int), ("rad", C.c_double),
        ("newton_max_its", C.c_int), ("newton_min_tol", C.c_double), ("newton_rel_tol", C.c_double),
        ("ksp_rtol", C.c_double), ("ksp_abstol", C.c_double), ("ksp_dtol", C.c_double),
        ("ksp_max_it", C.c_int), ("micro_n", C.c_int), ("micro_type", C.c_int),
        ("micro_mat_1", C.c_double * 4), ("micro_mat_2", C.c_double * 4),
        ("device", C.c_int), ("ksp_monitor", C.c_int), ("mat_type", C.c_int), ("mat_law", C.c_int),
        ("mat_aij_split", C.c_int),
        ("mat_aij_vi", C.c_int),
        ("mat_vi_fma", C.c_int),
    ]


class Info(C.Structure):
    _fields_ = [
        ("NX", C.c_int64), ("NY", C.c_int64), ("NZ", C.c_int64),
        ("px", C.c_int), ("py", C.c_int), ("pz", C.c_int), ("rank", C.c_int), ("nranks", C.c_int),
        ("xs", C.c_int64), ("ys", C.c_int64), ("zs", C.c_int64), ("nx", C.c_int64), ("ny", C.c_int64), ("nz", C.c_int64),
        ("Xs", C.c_int64), ("Ys", C.c_int64), ("Zs", C.c_int64), ("Nx", C.c_int64), ("Ny", C.c_int64), ("Nz", C.c_int64),
        ("ndofs_global", C.c_int64), ("ndofs_local", C.c_int64), ("dof_offset", C.c_int64),
        ("nnz_local", C.c_int64), ("nnz_global", C.c_int64), ("nelem_local", C.c_int64), ("nelem_ext", C.c_int64),
        ("dx", C.c_double), ("dy", C.c_double), ("dz", C.c_double), ("wg", C.c_double),
        ("device_bytes", C.c_int64), ("device", C.c_int), ("storage", C.c_int), ("split_slots", C.c_int),
        ("split_bits", C.c_int),
        ("ex0", C.c_int64), ("ey0", C.c_int64), ("ez0", C.c_int64), ("nex", C.c_int64), ("ney", C.c_int64),
        ("nez", C.c_int64),
        ("vi_values", C.c_int), ("vi_bits", C.c_int), ("vi_blocks", C.c_int),
        ("spmv_tx", C.c_int), ("spmv_ty", C.c_int), ("spmv_kc", C.c_int),
        ("vi_exc_nodes", C.c_int64), ("split_escapes", C.c_int64), ("st_listed", C.c_int64),
    ]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


# MicroPP C-wrapper call shapes (micropp_c_wrapper.h, called at src/assembly.c:59,92,149,
# src/main.c:62,83, src/util.c:71,96)
SET_STRAIN3 = C.CFUNCTYPE(None, C.c_int, C.POINTER(C.c_double))
HOMOGENIZE = C.CFUNCTYPE(None)
GET_STRESS3 = C.CFUNCTYPE(None, C.c_int, C.POINTER(C.c_double))
GET_CTAN3 = C.CFUNCTYPE(None, C.c_int, C.POINTER(C.c_double))
UPDATE_VARS = C.CFUNCTYPE(None)
GET_NON_LINEAR_GPS = C.CFUNCTYPE(C.c_int)
GET_F_TRIAL_MAX = C.CFUNCTYPE(C.c_double)


class MicroppApi(C.Structure):
    _fields_ = [("set_strain3", SET_STRAIN3), ("homogenize", HOMOGENIZE), ("get_stress3", GET_STRESS3),
                ("get_ctan3", GET_CTAN3), ("update_vars", UPDATE_VARS), ("get_non_linear_gps", GET_NON_LINEAR_GPS),
                ("get_f_trial_max", GET_F_TRIAL_MAX)]


class DeviceLaw(C.Structure):
    """mcx_device_law: function pointers of a device constitutive law (built in C/HIP)."""
    _fields_ = [("homogenize", C.c_void_p), ("update_vars", C.c_void_p), ("nonlinear_stats", C.c_void_p),
                ("user", C.c_void_p)]


class Timing(C.Structure):
    _fields_ = [
        ("strains_ms", C.c_double), ("homogenize_ms", C.c_double), ("residual_ms", C.c_double),
        ("jacobian_ms", C.c_double), ("solve_ms", C.c_double), ("update_ms", C.c_double),
        ("spmv_launches", C.c_int64), ("spmv_ms_total", C.c_double), ("spmv_bytes_per_launch", C.c_int64),
        ("cg_vec_bytes_per_iter", C.c_int64),
    ]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


_LIB = None


class MacrocError(RuntimeError):
    pass


def lib():
    """Load libmacroc_amd.so (raises if it is missing — there is no fallback)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise MacrocError(f"{LIB_PATH} not built: run `make` (or __graft_entry__.build())")
    L = C.CDLL(LIB_PATH)
    if L.mcx_abi_version() != ABI_VERSION:  # the structs below would not match the library's
        raise MacrocError(f"{LIB_PATH}: ABI {L.mcx_abi_version()}, this mirror needs {ABI_VERSION}: rebuild (`make`)")
    vp, d, i64 = C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_int64)
    L.mcx_last_error.restype = C.c_char_p
    L.mcx_version.restype = C.c_char_p
    L.mcx_default_opts.argtypes = [C.POINTER(Opts)]
    L.mcx_parse_args.argtypes = [C.POINTER(Opts), C.c_int, C.POINTER(C.c_char_p)]
    L.mcx_comm_unique_id.argtypes = [C.c_void_p]
    L.mcx_init.argtypes = [C.POINTER(Opts), C.c_int, C.c_int, C.c_void_p, C.POINTER(C.c_void_p)]
    L.mcx_plan.argtypes = [C.POINTER(Opts), C.c_int, C.c_int, C.POINTER(Info)]
    L.mcx_plan_halo.argtypes = [C.POINTER(Opts), C.c_int, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int),
                                i64, i64, i64, i64, i64, i64]
    L.mcx_local_group_create.argtypes = [C.c_int, C.c_int, C.POINTER(C.c_void_p)]
    L.mcx_local_group_destroy.argtypes = [vp]
    L.mcx_local_group_barrier.argtypes = [vp, C.c_int]
    L.mcx_init_local.argtypes = [C.POINTER(Opts), C.c_int, vp, C.POINTER(C.c_void_p)]
    L.mcx_finalize.argtypes = [vp]
    L.mcx_get_info.argtypes = [vp, C.POINTER(Info)]
    L.mcx_comm_info.argtypes = [vp, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int)]
    L.mcx_material_set.argtypes = [vp, C.c_int, C.c_double, C.c_double, C.c_double, C.c_double, C.c_int]
    L.mcx_get_displacement.argtypes = [vp, C.c_int]
    L.mcx_get_displacement.restype = C.c_double
    L.mcx_apply_bc_u.argtypes = [vp, C.c_double]
    for fn in ("mcx_zero_u", "mcx_set_strains", "mcx_homogenize", "mcx_assembly_jac", "mcx_update_u",
               "mcx_synchronize", "mcx_update_vars"):
        getattr(L, fn).argtypes = [vp]
    L.mcx_assembly_res.argtypes = [vp, d]
    L.mcx_solve.argtypes = [vp, C.POINTER(C.c_int), d, C.POINTER(C.c_int)]
    L.mcx_time_step.argtypes = [vp, C.c_int, C.POINTER(C.c_int), d, C.POINTER(C.c_int), d]
    for fn in ("mcx_get_u", "mcx_set_u", "mcx_get_b", "mcx_get_du", "mcx_get_strain", "mcx_get_stress"):
        getattr(L, fn).argtypes = [vp, d]
    L.mcx_owned_dofs.argtypes = [vp, i64, i64]
    L.mcx_get_nonlinear_stats.argtypes = [vp, i64, d]
    L.mcx_reduce_nonlinear.argtypes = [vp, i64, i64, d]
    L.mcx_calc_force.argtypes = [vp, d]
    L.mcx_write_vtu.argtypes = [vp, C.c_char_p]
    L.mcx_dump_csr.argtypes = [vp, i64, i64, d]
    L.mcx_dump_dirichlet.argtypes = [vp, i64, i64]
    L.mcx_spmv.argtypes = [vp, d, d]
    L.mcx_get_ksp_history.argtypes = [vp, d, i64]
    L.mcx_set_timing.argtypes = [vp, C.c_int]
    L.mcx_get_timing.argtypes = [vp, C.POINTER(Timing)]
    L.mcx_set_option.argtypes = [vp, C.c_char_p, C.c_double]
    L.mcx_time_spmv.argtypes = [vp, C.c_int, d]
    L.mcx_set_micropp.argtypes = [vp, C.POINTER(MicroppApi)]
    L.mcx_set_device_law.argtypes = [vp, C.POINTER(DeviceLaw)]
    for fn in ("mcx_set_gp_stress", "mcx_set_gp_ctan", "mcx_get_gp_strain"):
        getattr(L, fn).argtypes = [vp, d]
    _LIB = L
    return L


def _dp(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def _ip(a):
    return a.ctypes.data_as(C.POINTER(C.c_int64))


def _check(rc, what):
    if rc:
        raise MacrocError(f"{what} failed ({rc}): {lib().mcx_last_error().decode()}")


def parse_args(argv):
    o = Opts()
    lib().mcx_default_opts(C.byref(o))
    argv = [str(a) for a in argv]
    arr = (C.c_char_p * max(len(argv), 1))(*[a.encode() for a in argv])
    _check(lib().mcx_parse_args(C.byref(o), len(argv), arr), "mcx_parse_args")
    return o


def comm_unique_id():
    buf = C.create_string_buffer(COMM_ID_BYTES)
    _check(lib().mcx_comm_unique_id(buf), "mcx_comm_unique_id")
    return buf.raw


def plan(argv, rank=0, nranks=1):
    """Host-only: the DMDA decomposition rank `rank` of `nranks` gets (no GPU needed)."""
    o = parse_args(argv)
    inf = Info()
    _check(lib().mcx_plan(C.byref(o), rank, nranks, C.byref(inf)), "mcx_plan")
    return inf.as_dict()


def plan_halo(argv, rank=0, nranks=1):
    """Host-only: forward-halo plan of a rank — list of (neighbour rank, sent natural node ids,
    received natural node ids) in message order."""
    o = parse_args(argv)
    L = lib()
    nn, ns, nr = C.c_int(), C.c_int64(), C.c_int64()
    _check(L.mcx_plan_halo(C.byref(o), rank, nranks, C.byref(nn), None, None, None, None, None,
                           C.byref(ns), C.byref(nr)), "mcx_plan_halo")
    ranks = (C.c_int * 26)()
    sc, rc = np.zeros(26, dtype=np.int64), np.zeros(26, dtype=np.int64)
    sn, rn = np.zeros(max(ns.value, 1), dtype=np.int64), np.zeros(max(nr.value, 1), dtype=np.int64)
    _check(L.mcx_plan_halo(C.byref(o), rank, nranks, C.byref(nn), ranks, _ip(sc), _ip(rc), _ip(sn), _ip(rn),
                           C.byref(ns), C.byref(nr)), "mcx_plan_halo")
    out, so, ro = [], 0, 0
    for q in range(nn.value):
        out.append((ranks[q], sn[so:so + sc[q]].copy(), rn[ro:ro + rc[q]].copy()))
        so += sc[q]
        ro += rc[q]
    return out


class LocalGroup:
    """In-process transport for `nranks` contexts on one device (one host thread per rank)."""

    def __init__(self, nranks, device=0):
        self.nranks = nranks
        self._g = C.c_void_p()
        _check(lib().mcx_local_group_create(nranks, device, C.byref(self._g)), "mcx_local_group_create")

    def barrier(self, rank):
        """MPI_Barrier of the group (host only): fails on a missing member or a mismatched collective."""
        _check(lib().mcx_local_group_barrier(self._g, int(rank)), "mcx_local_group_barrier")

    def destroy(self):
        if self._g:
            g, self._g = self._g, C.c_void_p()
            _check(lib().mcx_local_group_destroy(g), "mcx_local_group_destroy")


class Macroc:
    """One rank (= one GPU subdomain) of the MacroC hot path."""

    def __init__(self, argv=(), rank=0, nranks=1, comm_id=None, opts=None, group=None):
        L = lib()
        self.opts = opts if opts is not None else parse_args(argv)
        self._ctx = C.c_void_p()
        cid = None
        if nranks > 1 and group is None and (comm_id is None or len(comm_id) != COMM_ID_BYTES):
            raise MacrocError("nranks > 1 needs the 128-byte id from comm_unique_id() on every rank")
        if comm_id is not None and group is None:  # one rank + an id: a one-rank RCCL communicator
            cid = C.create_string_buffer(comm_id, COMM_ID_BYTES)
        if group is not None:
            _check(L.mcx_init_local(C.byref(self.opts), rank, group._g, C.byref(self._ctx)), "mcx_init_local")
        else:
            _check(L.mcx_init(C.byref(self.opts), rank, nranks, cid, C.byref(self._ctx)), "mcx_init")
        inf = Info()
        _check(L.mcx_get_info(self._ctx, C.byref(inf)), "mcx_get_info")
        self.info = inf.as_dict()
        self.n = self.info["ndofs_local"]

    # ---- lifecycle
    def finish(self):
        if self._ctx:
            ctx, self._ctx = self._ctx, C.c_void_p()  # freed even when finalize reports an error
            _check(lib().mcx_finalize(ctx), "mcx_finalize")

    close = finish

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.finish()

    def __del__(self):
        try:
            self.finish()
        except Exception:
            pass

    # ---- the reference's hot-path functions
    def get_displacement(self, time_s):
        return lib().mcx_get_displacement(self._ctx, int(time_s))

    def zero_u(self):
        _check(lib().mcx_zero_u(self._ctx), "VecZeroEntries(u)")

    def apply_bc_on_u(self, U):
        _check(lib().mcx_apply_bc_u(self._ctx, float(U)), "apply_bc_on_u")

    def set_strains(self):
        _check(lib().mcx_set_strains(self._ctx), "set_strains")

    def homogenize(self):
        _check(lib().mcx_homogenize(self._ctx), "micropp_C_homogenize")

    def material_set(self, mid, E, nu, Sy=1e4, Ka=1e7, typ=1):
        _check(lib().mcx_material_set(self._ctx, mid, E, nu, Sy, Ka, typ), "micropp_C_material_set")

    def assembly_res(self):
        nrm = C.c_double()
        _check(lib().mcx_assembly_res(self._ctx, C.byref(nrm)), "assembly_res")
        return nrm.value

    def assembly_jac(self):
        _check(lib().mcx_assembly_jac(self._ctx), "assembly_jac")

    def solve_Ax(self):
        its, rn, reason = C.c_int(), C.c_double(), C.c_int()
        _check(lib().mcx_solve(self._ctx, C.byref(its), C.byref(rn), C.byref(reason)), "solve_Ax")
        return its.value, rn.value, reason.value

    def update_u(self):
        _check(lib().mcx_update_u(self._ctx), "VecAXPY(u,1,du)")

    def update_vars(self):
        _check(lib().mcx_update_vars(self._ctx), "micropp_C_update_vars")

    def get_info(self):
        """mcx_get_info now (storage reflects the last assembly)."""
        inf = Info()
        _check(lib().mcx_get_info(self._ctx, C.byref(inf)), "mcx_get_info")
        return inf.as_dict()

    def comm_info(self):
        """(ranks in the communicator, this rank in it, HIP device): ncclCommCount /
        ncclCommUserRank / ncclCommCuDevice for RCCL, the group for the in-process transport."""
        n, r, d = C.c_int(), C.c_int(), C.c_int()
        _check(lib().mcx_comm_info(self._ctx, C.byref(n), C.byref(r), C.byref(d)), "mcx_comm_info")
        return n.value, r.value, d.value

    def nonlinear_stats(self):
        """micropp_C_get_non_linear_gps / get_f_trial_max of this rank."""
        n, f = C.c_int64(), C.c_double()
        _check(lib().mcx_get_nonlinear_stats(self._ctx, C.byref(n), C.byref(f)), "nonlinear_stats")
        return n.value, f.value

    def reduce_nonlinear(self):
        """get_non_linear_gps + get_f_trial_max (src/util.c:69-102), collective:
        (this rank's count, total over ranks, max f_trial over ranks)."""
        nl, nt, f = C.c_int64(), C.c_int64(), C.c_double()
        _check(lib().mcx_reduce_nonlinear(self._ctx, C.byref(nl), C.byref(nt), C.byref(f)), "reduce_nonlinear")
        return nl.value, nt.value, f.value

    def write_vtu(self, prefix):
        """write_pvtu (src/output.c:25-267), collective."""
        _check(lib().mcx_write_vtu(self._ctx, str(prefix).encode()), "write_vtu")

    def calc_force(self):
        """calc_force (src/forces.c:25-166), collective; every rank gets the total."""
        f = C.c_double()
        _check(lib().mcx_calc_force(self._ctx, C.byref(f)), "calc_force")
        return f.value

    def time_step(self, time_s):
        k = max(self.opts.newton_max_its, 1)
        nits = C.c_int()
        res, kr = np.zeros(k), np.zeros(k)
        ki = (C.c_int * k)()
        _check(lib().mcx_time_step(self._ctx, int(time_s), C.byref(nits), _dp(res), ki, _dp(kr)), "time_step")
        n = nits.value
        return dict(newton_its=n, res=res[: n + 1 if n < k else n].tolist(), ksp_its=list(ki)[:n],
                    ksp_rnorm=kr[:n].tolist())

    def synchronize(self):
        _check(lib().mcx_synchronize(self._ctx), "synchronize")

    # ---- the MicroPP Gauss-point callback boundary (-mat_law external)
    @property
    def ngp(self):
        """Gauss points of the callback box (mcx_info nelem_ext * 8), gpi = ie*8 + gp."""
        return 8 * self.info["nelem_ext"]

    def set_micropp(self, set_strain3=None, homogenize=None, get_stress3=None, get_ctan3=None, update_vars=None,
                    get_non_linear_gps=None, get_f_trial_max=None):
        """Register host callbacks with micropp_C_* call shapes (Python callables taking
        (gpi, ctypes double pointer) etc.); no arguments unregisters."""
        if set_strain3 is None:
            _check(lib().mcx_set_micropp(self._ctx, None), "mcx_set_micropp")
            self._mpp = None
            return
        api = MicroppApi(SET_STRAIN3(set_strain3), HOMOGENIZE(homogenize), GET_STRESS3(get_stress3),
                         GET_CTAN3(get_ctan3), UPDATE_VARS(update_vars) if update_vars else UPDATE_VARS(),
                         GET_NON_LINEAR_GPS(get_non_linear_gps) if get_non_linear_gps else GET_NON_LINEAR_GPS(),
                         GET_F_TRIAL_MAX(get_f_trial_max) if get_f_trial_max else GET_F_TRIAL_MAX())
        self._mpp = api  # the library keeps the function pointers: keep the thunks alive
        _check(lib().mcx_set_micropp(self._ctx, C.byref(api)), "mcx_set_micropp")

    def set_device_law(self, law):
        """Register an mcx_device_law (DeviceLaw structure filled by a C/HIP library); None unregisters."""
        self._dlaw = law
        _check(lib().mcx_set_device_law(self._ctx, C.byref(law) if law is not None else None), "mcx_set_device_law")

    def set_gp_stress(self, sig):
        sig = np.ascontiguousarray(sig, dtype=np.float64).reshape(self.ngp, 6)
        _check(lib().mcx_set_gp_stress(self._ctx, _dp(sig)), "mcx_set_gp_stress")

    def set_gp_ctan(self, ctan):
        ctan = np.ascontiguousarray(ctan, dtype=np.float64).reshape(self.ngp, 36)
        _check(lib().mcx_set_gp_ctan(self._ctx, _dp(ctan)), "mcx_set_gp_ctan")

    def gp_strain(self):
        """strains of the callback box, [ngp][6] in gpi order."""
        return self._get("mcx_get_gp_strain", self.ngp * 6).reshape(-1, 6)

    # ---- data access (owned rows, PETSc-local order)
    def _get(self, fn, n):
        a = np.zeros(n)
        _check(getattr(lib(), fn)(self._ctx, _dp(a)), fn)
        return a

    def u(self):
        return self._get("mcx_get_u", self.n)

    def set_u(self, u):
        u = np.ascontiguousarray(u, dtype=np.float64)
        assert u.shape == (self.n,)
        _check(lib().mcx_set_u(self._ctx, _dp(u)), "mcx_set_u")

    def b(self):
        return self._get("mcx_get_b", self.n)

    def du(self):
        return self._get("mcx_get_du", self.n)

    def strain(self):
        return self._get("mcx_get_strain", self.info["nelem_local"] * 48).reshape(-1, 6)

    def stress(self):
        return self._get("mcx_get_stress", self.info["nelem_local"] * 48).reshape(-1, 6)

    def owned_dofs(self):
        p = np.zeros(self.n, dtype=np.int64)
        nat = np.zeros(self.n, dtype=np.int64)
        _check(lib().mcx_owned_dofs(self._ctx, _ip(p), _ip(nat)), "mcx_owned_dofs")
        return p, nat

    def dump_csr(self, values=True):
        nnz = self.info["nnz_local"]
        rp = np.zeros(self.n + 1, dtype=np.int64)
        ci = np.zeros(nnz, dtype=np.int64)
        v = np.zeros(nnz) if values else None
        _check(lib().mcx_dump_csr(self._ctx, _ip(rp), _ip(ci), _dp(v) if values else None), "mcx_dump_csr")
        return rp, ci, v

    def dump_dirichlet(self):
        n = C.c_int64(0)
        _check(lib().mcx_dump_dirichlet(self._ctx, None, C.byref(n)), "mcx_dump_dirichlet")
        a = np.zeros(max(n.value, 1), dtype=np.int64)
        _check(lib().mcx_dump_dirichlet(self._ctx, _ip(a), C.byref(n)), "mcx_dump_dirichlet")
        return a[: n.value]

    def spmv(self, x):
        x = np.ascontiguousarray(x, dtype=np.float64)
        y = np.zeros(self.n)
        _check(lib().mcx_spmv(self._ctx, _dp(x), _dp(y)), "mcx_spmv")
        return y

    def ksp_history(self):
        n = C.c_int64(0)
        _check(lib().mcx_get_ksp_history(self._ctx, None, C.byref(n)), "history")
        h = np.zeros(max(n.value, 1))
        _check(lib().mcx_get_ksp_history(self._ctx, _dp(h), C.byref(n)), "history")
        return h[: n.value]

    def set_timing(self, on=True):
        _check(lib().mcx_set_timing(self._ctx, 1 if on else 0), "mcx_set_timing")

    def set_option(self, name, value):
        _check(lib().mcx_set_option(self._ctx, name.encode(), float(value)), "mcx_set_option")

    def time_spmv(self, iters=20):
        ms = C.c_double()
        _check(lib().mcx_time_spmv(self._ctx, int(iters), C.byref(ms)), "mcx_time_spmv")
        return ms.value

    def timing(self):
        t = Timing()
        _check(lib().mcx_get_timing(self._ctx, C.byref(t)), "mcx_get_timing")
        return t.as_dict()
