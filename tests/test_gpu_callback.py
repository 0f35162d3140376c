"""The MicroPP Gauss-point callback boundary (-mat_law external, include/macroc_amd.h).

The reference hands each Gauss point's strain to MicroPP's C wrapper and reads stress and tangent
back (src/assembly.c:59,92,149, src/main.c:62,83).  Here a constitutive law that lives OUTSIDE
libmacroc_amd replaces the device laws through that boundary, in the three ways the ABI offers:
  * host callbacks with the micropp_C_* call shapes (Python ctypes thunks here; a real MicroPP
    links straight in, see test_driver_links_a_micropp);
  * a device law (tests/csrc/testlaw.hip, its own HIP kernel on the context's stream);
  * batched injection of caller-computed stress / tangent (mcx_set_gp_stress / _ctan).
The external law computes the isotropic elastic answer with the same operation order as the
oracle's surrogate (sigma_k = sum_l C_kl eps_l, l ascending), so residual and assembled matrix must
be bit-identical to the oracle, and the solve must meet the north-star bar.
"""
import ctypes as C
import os
import subprocess
import threading

import numpy as np
import pytest

import macroc_amd as M
from oracle import oracle as O

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
TESTLAW = os.path.join(HERE, "libmcx_testlaw.so")
E_DEF, NU_DEF = 1.0e7, 0.25  # src/init.c:31-32


def iso_C(E, nu):
    lam = E * nu / ((1. + nu) * (1. - 2. * nu))
    mu = E / (2. * (1. + nu))
    Cm = np.zeros((6, 6))
    for a in range(3):
        for b in range(3):
            Cm[a, b] = lam + (2. * mu if a == b else 0.)
    for a in range(3, 6):
        Cm[a, a] = mu
    return Cm


def stress_of(eps, Cm):
    """sigma[:, k] = sum_l C[k, l] eps[:, l], l ascending (elementwise IEEE ops, no FMA)."""
    sig = np.zeros_like(eps)
    for k in range(6):
        s = np.zeros(len(eps))
        for l in range(6):
            s = s + Cm[k, l] * eps[:, l]
        sig[:, k] = s
    return sig


class HostMicropp:
    """A MicroPP-shaped host law driven through ctypes thunks; records the call sequence."""

    def __init__(self, ngp, Cm):
        self.eps = np.full((ngp, 6), np.nan)
        self.sig = None
        self.Cm = Cm
        self.order = []
        self.calls = {"homogenize": 0, "update_vars": 0}

    def set_strain3(self, gpi, p):
        self.order.append(gpi)
        self.eps[gpi] = np.ctypeslib.as_array(p, shape=(6,))

    def homogenize(self):
        self.calls["homogenize"] += 1
        self.sig = stress_of(self.eps, self.Cm)

    def get_stress3(self, gpi, p):
        np.ctypeslib.as_array(p, shape=(6,))[:] = self.sig[gpi]

    def get_ctan3(self, gpi, p):
        np.ctypeslib.as_array(p, shape=(36,))[:] = self.Cm.ravel()

    def update_vars(self):
        self.calls["update_vars"] += 1

    def register(self, m):
        m.set_micropp(self.set_strain3, self.homogenize, self.get_stress3, self.get_ctan3, self.update_vars,
                      lambda: 0, lambda: -1.0)


def _testlaw():
    L = C.CDLL(TESTLAW)
    L.testlaw_elastic_device.argtypes = [C.POINTER(M.DeviceLaw), C.c_double, C.c_double]
    L.testlaw_device_calls.argtypes = [C.POINTER(M.DeviceLaw), C.POINTER(C.c_int)]
    return L


def argv(NX, NY, NZ, rtol, extra=()):
    return ["-da_grid_x", NX, "-da_grid_y", NY, "-da_grid_z", NZ, "-ksp_rtol", repr(rtol), "-mat_law", "external",
            *extra]


def step_and_compare(m, P, inject=None):
    for ts in (0, 1):
        m.apply_bc_on_u(m.get_displacement(ts))
        P.apply_bc_u(P.get_displacement(ts))
    m.set_strains()
    P.set_strains()
    m.homogenize()
    P.homogenize()
    if inject:
        inject(m)
    assert np.array_equal(m.stress(), P.stress())
    res = m.assembly_res()
    P.assembly_res()
    assert np.array_equal(m.b(), P.b())
    assert abs(res - P.norm_b()) <= 1e-13 * P.norm_b()
    m.assembly_jac()
    P.assembly_jac()
    rp, ci, v = m.dump_csr()
    assert np.array_equal(v, P.A_values())
    its, rn, reason = m.solve_Ax()
    out = P.solve()
    assert abs(its - out["its"]) <= 1 and reason == out["reason"]
    ref = P.du()
    assert np.linalg.norm(m.du() - ref) <= 1e-10 * np.linalg.norm(ref)
    return its


@pytest.mark.parametrize("grid", [(8, 8, 8), (10, 6, 7)])
def test_host_micropp_callbacks(grid):
    rtol = 1e-12
    P = O.Problem(*grid, rtol=rtol)
    with M.Macroc(argv(*grid, rtol, ["-mat_aij_vi", 0, "-mat_aij_split", 0])) as m:
        law = HostMicropp(m.ngp, iso_C(E_DEF, NU_DEF))
        law.register(m)
        step_and_compare(m, P)
        # every Gauss point handed over once, in gpi = ie*8 + gp order, with the device strains
        assert law.order == list(range(m.ngp)) and law.calls["homogenize"] == 1
        assert np.array_equal(law.eps, m.gp_strain())
        m.update_vars()
        assert law.calls["update_vars"] == 1
        assert m.nonlinear_stats() == (0, -1.0)


def test_device_law_default_storage():
    """A device law from another library, default AIJ storage: its per-GP tangents are all the
    isotropic C, so the matrix is value-indexed (bit-exact matrix dump)."""
    grid, rtol = (8, 8, 8), 1e-12
    P = O.Problem(*grid, rtol=rtol)
    L = _testlaw()
    law = M.DeviceLaw()
    assert L.testlaw_elastic_device(C.byref(law), E_DEF, NU_DEF) == 0
    with M.Macroc(argv(*grid, rtol)) as m:
        m.set_option("split_maxq", 30)
        m.set_device_law(law)
        step_and_compare(m, P)
        assert m.get_info()["storage"] == 3
        m.update_vars()
        upd = C.c_int()
        assert L.testlaw_device_calls(C.byref(law), C.byref(upd)) == 1 and upd.value == 1


def test_injected_stress_and_tangent():
    """mcx_set_gp_stress / mcx_set_gp_ctan: values computed by the caller from mcx_get_gp_strain."""
    grid, rtol = (9, 7, 8), 1e-12
    P = O.Problem(*grid, rtol=rtol)
    Cm = iso_C(E_DEF, NU_DEF)

    def inject(m):
        eps = m.gp_strain()
        m.set_gp_stress(stress_of(eps, Cm))
        m.set_gp_ctan(np.tile(Cm.ravel(), (m.ngp, 1)))

    with M.Macroc(argv(*grid, rtol, ["-dm_mat_type", "sbaij"])) as m:
        # sbaij: the oracle's matrix is compared after mirroring its upper triangle
        for ts in (0, 1):
            m.apply_bc_on_u(m.get_displacement(ts))
            P.apply_bc_u(P.get_displacement(ts))
        m.set_strains(); P.set_strains()
        m.homogenize(); P.homogenize()
        inject(m)
        assert np.array_equal(m.stress(), P.stress())
        m.assembly_res(); P.assembly_res()
        assert np.array_equal(m.b(), P.b())
        m.assembly_jac(); P.assembly_jac(); P.sbaij_mirror()
        assert np.array_equal(m.dump_csr()[2], P.A_values())


def test_external_law_multirank_box():
    """2 ranks (in-process transport): each rank's callback box is its PETSc elements plus the
    upper ghost layer; injected per rank, the decomposed residual and matrix rows equal the
    one-rank oracle's in natural order."""
    grid, rtol = (10, 8, 8), 1e-12
    P = O.Problem(*grid, rtol=rtol)
    for ts in (0, 1):
        P.apply_bc_u(P.get_displacement(ts))
    P.set_strains(); P.homogenize(); P.assembly_res(); P.assembly_jac()
    Cm = iso_C(E_DEF, NU_DEF)
    args = argv(*grid, rtol, ["-da_processors_x", 2, "-mat_aij_vi", 0, "-mat_aij_split", 0])
    g = M.LocalGroup(2)
    out, errs = [None, None], []

    def worker(r):
        try:
            with M.Macroc(args, rank=r, nranks=2, group=g) as m:
                inf = m.info
                assert inf["nelem_ext"] == inf["nex"] * inf["ney"] * inf["nez"]
                for ts in (0, 1):
                    m.apply_bc_on_u(m.get_displacement(ts))
                m.set_strains()
                m.homogenize()
                eps = m.gp_strain()
                m.set_gp_stress(stress_of(eps, Cm))
                m.set_gp_ctan(np.tile(Cm.ravel(), (m.ngp, 1)))
                m.assembly_res()
                m.assembly_jac()
                petsc, nat = m.owned_dofs()
                out[r] = (nat, m.b(), m.dump_csr(), m.info["dof_offset"])
        except Exception as e:
            errs.append(e)

    ts = [threading.Thread(target=worker, args=(r,)) for r in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(300)
    g.destroy()
    assert not errs, errs
    b_ref, v_ref = P.b(), P.A_values()
    rp_ref, ci_ref = P.csr()
    to_petsc = O.petsc_numbering(*grid, 2, 2, 1, 1)  # natural node -> PETSc node of the 2-rank grid
    to_nat = np.empty_like(to_petsc)
    to_nat[to_petsc] = np.arange(len(to_petsc))
    for nat, b, (rp, ci, v), off in out:
        assert np.array_equal(b, b_ref[nat])
        for q in range(len(nat)):
            cols = 3 * to_nat[ci[rp[q]:rp[q + 1]] // 3] + ci[rp[q]:rp[q + 1]] % 3
            o = np.argsort(cols)
            lo, hi = rp_ref[nat[q]], rp_ref[nat[q] + 1]
            assert np.array_equal(cols[o], ci_ref[lo:hi]) and np.array_equal(v[rp[q]:rp[q + 1]][o], v_ref[lo:hi])


def test_driver_links_a_micropp(tmp_path):
    """The C driver built against a MicroPP-shaped library (make testlaw: -DMCX_WITH_MICROPP)
    runs -mat_law external and prints the same |RES| / KSP lines as the device elastic law."""
    exe = os.path.join(HERE, "macroc_amd_micropp")
    base = os.path.join(os.path.dirname(HERE), "macroc_amd", "driver", "macroc_amd")
    flags = ["-da_grid_x", "6", "-da_grid_y", "6", "-da_grid_z", "6", "-ts", "3", "-dt", "0.01", "-ksp_rtol", "1e-10"]

    def run(cmd, d):
        d.mkdir()
        r = subprocess.run(cmd, cwd=d, capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr
        return [ln for ln in r.stdout.splitlines() if ln.startswith(("|RES|", "KSP", "Time Step", "Non-Linear"))]

    ext = run([exe, *flags, "-mat_law", "external"], tmp_path / "ext")
    dev = run([base, *flags], tmp_path / "dev")
    assert ext == dev and any(ln.startswith("KSP") for ln in ext)
