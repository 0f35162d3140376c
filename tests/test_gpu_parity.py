"""GPU parity: the HIP path (through the C-ABI) against the CPU oracle and the golden fixtures.

Bars: integer artefacts bit-exact; on one rank the element kinematics,
strains, stresses, residual, assembled matrix and SpMV are bit-exact too (same operation
order, no FMA contraction); the CG solution differs only through the reduction order of the
dot products: iteration count within +-1 and |du - du_oracle| / |du| <= 1e-10 at
-ksp_rtol 1e-12 (the north-star tolerance), <= 50 * rtol at looser rtol.
Full-size grids are checked through size-independent properties (true residual, symmetry,
linearity, determinism).
"""
import os

import numpy as np
import pytest

import macroc_amd as M
from oracle import oracle as O

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
SINGLE = ["g442_r1", "g522_r1", "g444_r1", "g888_r1", "g16_r1"]


def load(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)


def argv_for(NX, NY, NZ, rtol, extra=()):
    return ["-da_grid_x", NX, "-da_grid_y", NY, "-da_grid_z", NZ, "-ksp_rtol", repr(rtol), "-ksp_monitor", *extra]


def du_tol(rtol):
    return 1e-10 if rtol <= 1e-12 else 50 * rtol


@pytest.mark.parametrize("name", SINGLE)
def test_newton_step_single_rank(name):
    """-mat_aij_split 0: AIJ stencil blocks, every row summed in the reference's MatMult order (inode column pairs)."""
    fx = load(name)
    NX, NY, NZ = (int(v) for v in fx["grid"])
    rtol = float(fx["rtol"])
    P = O.Problem(NX, NY, NZ, rtol=rtol)
    with M.Macroc(argv_for(NX, NY, NZ, rtol, ["-mat_aij_vi", 0, "-mat_aij_split", 0])) as m:
        petsc, nat = m.owned_dofs()
        assert np.array_equal(petsc, fx["dof_map"][nat])
        assert np.array_equal(m.dump_dirichlet(), fx["dirichlet"])
        # time step 0 then 1 (src/main.c:49-54)
        for ts in (0, 1):
            U = m.get_displacement(ts)
            assert U == P.get_displacement(ts)
            m.apply_bc_on_u(U)
            P.apply_bc_u(U)
        assert np.array_equal(m.u(), P.u())
        m.set_strains()
        P.set_strains()
        assert np.array_equal(m.strain(), P.strain())
        m.homogenize()
        P.homogenize()
        assert np.array_equal(m.stress(), P.stress())
        res = m.assembly_res()
        P.assembly_res()
        assert np.array_equal(m.b(), P.b())
        assert np.array_equal(m.b(), fx["b"])
        assert abs(res - float(fx["res"])) <= 1e-13 * max(float(fx["res"]), 1.0)
        m.assembly_jac()
        P.assembly_jac()
        rp, ci, v = m.dump_csr()
        orp, oci = P.csr()
        assert np.array_equal(rp, orp) and np.array_equal(ci, oci.astype(np.int64))
        assert np.array_equal(v, P.A_values())
        x = np.random.default_rng(42).uniform(-1, 1, m.n)
        assert np.array_equal(m.spmv(x), P.spmv(x))
        its, rn, reason = m.solve_Ax()
        P.solve()
        assert reason == int(fx["reason"]) or (its == 0 and int(fx["its"]) == 0)
        assert abs(its - int(fx["its"])) <= 1
        du = m.du()
        ref = fx["du"]
        if np.linalg.norm(ref) > 0:
            assert np.linalg.norm(du - ref) <= du_tol(rtol) * np.linalg.norm(ref)
            h = m.ksp_history()
            k = min(len(h), len(fx["history"]), 20)
            np.testing.assert_allclose(h[:k], fx["history"][:k], rtol=1e-9)
        else:
            assert np.linalg.norm(du) == 0
        m.update_u()
        assert np.linalg.norm(m.u() - fx["u"]) <= du_tol(rtol) * np.linalg.norm(fx["u"]) + 1e-300


@pytest.mark.parametrize("name", SINGLE)
def test_aij_vi_single_rank(name):
    """Default AIJ storage for the elastic law: value-indexed (one index byte per value into a
    dictionary of the matrix's distinct values).  Matrix dump and SpMV bit-exact with the
    oracle's CPU AIJ (same row order as the AIJ blocks), the dictionary sorted and small, the
    solve's residual history equal to the fixture's."""
    fx = load(name)
    NX, NY, NZ = (int(v) for v in fx["grid"])
    rtol = float(fx["rtol"])
    P = O.Problem(NX, NY, NZ, rtol=rtol)
    with M.Macroc(argv_for(NX, NY, NZ, rtol)) as m:
        for ts in (0, 1):
            m.apply_bc_on_u(m.get_displacement(ts))
            P.apply_bc_u(m.get_displacement(ts))
        m.set_strains(); m.homogenize(); m.assembly_res()
        P.set_strains(); P.homogenize(); P.assembly_res()
        m.assembly_jac()
        P.assembly_jac()
        info = m.get_info()
        rp, ci, v = m.dump_csr()
        assert np.array_equal(v, P.A_values())
        nval = len(np.unique(v.view(np.int64)))  # distinct bit patterns of the AIJ values
        assert info["storage"] == 3 and nval <= info["vi_values"] <= nval + 1  # + the clipped blocks' 0
        x = np.random.default_rng(42).uniform(-1, 1, m.n)
        y = m.spmv(x)
        assert np.array_equal(y, P.spmv(x))
        assert np.array_equal(m.spmv(x), y)
        # every slot takes <= 16 values and every block position few blocks: one byte per 3x3 block
        assert info["vi_bits"] == 4 and 0 < info["vi_blocks"] <= 256
        # the single-pass block build (default) and round 2's three-pass build: the same
        # dictionary order, so the same index bytes, matrix and products
        m.set_option("vib_onepass", 0)
        m.assembly_jac()
        i3 = m.get_info()
        assert (i3["vi_blocks"], i3["vi_values"], i3["vi_bits"]) == (info["vi_blocks"], info["vi_values"], 4)
        assert np.array_equal(m.dump_csr()[2], v) and np.array_equal(m.spmv(x), y)
        m.set_option("vib_onepass", 1)
        m.assembly_jac()
        m.set_option("vi_block", 0)  # per-slot nibble indices: the same matrix and products
        m.assembly_jac()
        assert m.get_info()["vi_blocks"] == 0 and np.array_equal(m.dump_csr()[2], v)
        assert np.array_equal(m.spmv(x), y)
        m.set_option("vi_stage", 0)  # x gathered instead of staged in LDS: the same products
        assert np.array_equal(m.spmv(x), y)
        m.set_option("vi_stage", 1)
        m.set_option("spmv_zblocks", 1)  # one z-chunk per tile: the staged ring marches every plane
        assert np.array_equal(m.spmv(x), y)
        m.set_option("spmv_zblocks", 0)
        assert np.array_equal(m.spmv(x), y)
        m.set_option("vi_stage", -1)
        m.set_option("vi_bits", 8)  # one byte per value into one dictionary: the same matrix and products
        m.assembly_jac()
        assert m.get_info()["vi_bits"] == 8 and np.array_equal(m.dump_csr()[2], v)
        assert np.array_equal(m.spmv(x), y)
        m.set_option("vi_bits", 4)
        m.set_option("vi_block", 1)
        m.assembly_jac()
        assert m.get_info()["vi_blocks"] > 0
        # block dictionary: gathered x, staged x, marching (-mat_vi_fma 0: products in the CPU AIJ
        # order): wave-uniform blocks from scalar loads on 16x4 patches or row quarters, or every
        # block from LDS with x read unpaired or paired — all bit-exact
        rp_, ci_, v_ = m.dump_csr()
        absrow = np.add.reduceat(np.abs(v_) * np.abs(x[ci_]), rp_[:-1])
        for stage, zblocks, uni, patch, xread in ((0, 0, 1, 1, 1), (1, 0, 1, 1, 1), (1, 1, 1, 1, 1), (1, 0, 1, 0, 1),
                                                  (1, 0, 0, 0, 1), (1, 1, 0, 0, 1), (1, 0, 0, 0, 0), (1, 1, 0, 0, 0)):
            for k_, v_o in (("vi_fma", 0), ("vi_stage", stage), ("spmv_zblocks", zblocks), ("vi_uni", uni),
                            ("vi_patch", patch), ("vi_xread", xread)):
                m.set_option(k_, v_o)
            assert np.array_equal(m.spmv(x), y), (stage, zblocks, uni, patch, xread)
        # the default staged kernel sums with fused multiply-adds: rows within rounding of the
        # CPU order, deterministic
        for k_, v_o in (("vi_fma", 1), ("vi_uni", 1), ("vi_patch", 1), ("vi_xread", 1), ("vi_stage", 1)):
            m.set_option(k_, v_o)
        for zblocks in (0, 1):
            m.set_option("spmv_zblocks", zblocks)
            yf = m.spmv(x)
            assert np.all(np.abs(yf - y) <= 1e-14 * absrow + 1e-300) and np.array_equal(m.spmv(x), yf)
        m.set_option("vi_stage", -1)
        m.set_option("spmv_zblocks", 0)
        its, rn, reason = m.solve_Ax()
        assert abs(its - int(fx["its"])) <= 1
        ref = fx["du"]
        if np.linalg.norm(ref) > 0:
            assert np.linalg.norm(m.du() - ref) <= du_tol(rtol) * np.linalg.norm(ref)
            h = m.ksp_history()
            k = min(len(h), len(fx["history"]), 20)
            np.testing.assert_allclose(h[:k], fx["history"][:k], rtol=1e-9)
        # the same matrix through -mat_aij_vi 0 -mat_aij_split 0 (AIJ blocks): identical products
        m.set_option("aij_vi", 0)
        m.set_option("aij_split", 0)
        m.assembly_jac()
        assert m.get_info()["storage"] == 0 and np.array_equal(m.spmv(x), y)


def test_aij_vi_fallback_and_toggle():
    """More than 256 distinct values (a plastic tangent) overflow the dictionary: the assembly
    falls back to the AIJ-split storage, bit-exact; an elastic matrix is value-indexed again
    once the option is re-enabled."""
    NX, NY, NZ, dt = 12, 10, 12, 0.05
    P = O.Problem(NX, NY, NZ, rtol=1e-10, law=1, dt=dt, bc_type=0)
    P.apply_bc_u(P.get_displacement(1))
    P.set_strains(); P.homogenize(); P.assembly_res(); P.assembly_jac(); P.solve(); P.update_u()
    u = P.u()
    P.set_strains(); P.homogenize(); P.assembly_jac()
    argv = ["-da_grid_x", NX, "-da_grid_y", NY, "-da_grid_z", NZ, "-dt", dt, "-mat_law", "plastic", "-bc_type", 0]
    with M.Macroc(argv) as m:
        m.apply_bc_on_u(m.get_displacement(1))
        m.set_strains(); m.homogenize(); m.assembly_res(); m.assembly_jac()
        assert m.get_info()["storage"] == 3  # still elastic everywhere: one tangent, few values
        m.solve_Ax(); m.update_u()
        m.set_u(u)
        m.set_strains(); m.homogenize(); m.assembly_jac()
        info = m.get_info()
        assert info["storage"] == 2 and info["vi_values"] == 0
        assert np.array_equal(m.dump_csr()[2], P.A_values())
    with pytest.raises(M.MacrocError):
        with M.Macroc(["-da_grid_x", 6, "-da_grid_y", 6, "-da_grid_z", 6, "-dm_mat_type", "sbaij"]) as m:
            m.set_option("aij_vi", 1)


def plastic_state(NX, NY, NZ, dt=0.01, rtol=1e-10):
    """Oracle J2 problem after one solved Newton iteration of time step 1 (default load): the
    Gauss points under the load are plastic, the rest on the elastic branch.  Returns the oracle
    (assembled at that state) and its u."""
    P = O.Problem(NX, NY, NZ, rtol=rtol, law=1, dt=dt)
    P.apply_bc_u(P.get_displacement(1))
    P.set_strains(); P.homogenize(); P.assembly_res(); P.assembly_jac(); P.solve(); P.update_u()
    u = P.u()
    P.set_strains(); P.homogenize(); P.assembly_res(); P.assembly_jac()
    assert P.nonlinear_gps()[0] > 0
    return P, u


@pytest.mark.parametrize("grid,stage,vi_tx,tile", [((12, 10, 14), 0, 0, (0, 0)), ((130, 9, 12), 1, 0, (64, 16)),
                                                   ((130, 9, 12), 1, 128, (128, 8)), ((260, 9, 10), 1, 256, (256, 4))])
def test_aij_vi_exception_nodes(grid, stage, vi_tx, tile):
    """A per-GP-tangent law (J2) with a few plastic Gauss points stays value-indexed: the nodes
    touching an element with a non-elastic tangent keep their 27 blocks as plain values
    (exception nodes), every other node indexes the elastic blocks' dictionary.  Matrix values
    bit-exact with the oracle's AIJ; the SpMV bit-exact with the CPU AIJ product (inode order) under
    -mat_vi_fma 0 (gathered kernel, and the 64x16 / 128x8 / 256x4 staged tiles), within
    1e-14 sum|a||x| with the fused multiply-adds; the solve within the north-star bar."""
    NX, NY, NZ = grid
    rtol = 1e-10
    P, u = plastic_state(NX, NY, NZ, rtol=rtol)
    rp1, ci1 = P.csr()
    v1 = P.A_values()
    x = np.random.default_rng(5).uniform(-1, 1, P.ndofs)
    y1 = P.spmv(x)
    absrow = np.add.reduceat(np.abs(v1) * np.abs(x[ci1]), rp1[:-1])
    b1 = P.b()
    ref_its = P.solve()["its"]
    argv = ["-da_grid_x", NX, "-da_grid_y", NY, "-da_grid_z", NZ, "-dt", 0.01, "-mat_law", "plastic",
            "-ksp_rtol", repr(rtol)]
    with M.Macroc(argv) as m:
        m.set_option("vi_stage", stage)
        m.set_option("vi_tx", vi_tx)
        m.set_u(u)
        m.set_strains(); m.homogenize(); m.assembly_res(); m.assembly_jac()
        info = m.get_info()
        assert info["storage"] == 3 and info["vi_blocks"] > 0, info
        assert 0 < info["vi_exc_nodes"] < NX * NY * NZ // 4, info
        assert (info["spmv_tx"], info["spmv_ty"]) == tile, info
        assert np.array_equal(m.b(), b1)
        assert np.array_equal(m.dump_csr()[2], v1)
        m.set_option("vi_fma", 0)
        assert np.array_equal(m.spmv(x), y1)
        # staged tiles: exception rows in their own kernel after the march (k_spmv_exc, default),
        # or round 4's forms: after the march by the whole tile block, in their plane (list size
        # 0), or both (a list of 3 that overflows): the same rows
        for xk, xl in ((0, 0), (0, 3), (0, 2048), (1, 2048)):
            m.set_option("vi_exc_kernel", xk)
            m.set_option("vi_exc_list", xl)
            assert np.array_equal(m.spmv(x), y1), (xk, xl)
        m.set_option("vi_fma", 1)
        y = m.spmv(x)
        assert np.all(np.abs(y - y1) <= 1e-14 * absrow + 1e-300)
        if tile == (64, 16):  # vi_st -1 with exception nodes (<= 10 %): the default-stencil path, exceptions listed
            assert m.get_info()["st_listed"] >= info["vi_exc_nodes"], m.get_info()
        m.set_option("vi_st", 0)  # the exception rows through k_spmv_exc / the in-tile pass below
        for xk, xl in ((0, 0), (0, 3), (0, 2048), (1, 2048)):
            m.set_option("vi_exc_kernel", xk)
            m.set_option("vi_exc_list", xl)
            assert np.array_equal(m.spmv(x), y), (xk, xl)
        m.set_option("vi_lg_exc", 0)  # per-block waits on the LDS path of the exception kernel: the same rows
        assert np.array_equal(m.spmv(x), y)
        m.set_option("vi_lg_exc", 1)
        m.set_option("vi_st", 1)  # default-stencil kernel: exception nodes among the listed rows
        assert np.array_equal(m.spmv(x), y)
        for l16 in (0, 1, -1):  # the listed rows one thread per node / 16 lanes per node (round 6) / by length
            m.set_option("vi_st_l16", l16)
            assert np.array_equal(m.spmv(x), y), l16
        its, rn, reason = m.solve_Ax()
        assert reason > 0 and abs(its - ref_its) <= 1
        assert np.linalg.norm(m.du() - P.du()) <= 50 * rtol * np.linalg.norm(P.du())
        # the CG's Jacobi from the diagonal index (exception nodes: jix 255 -> the Jacobi vector)
        # is bitwise the Jacobi vector's
        du = m.du()
        m.set_option("cg_dix", 0)
        its0, _, _ = m.solve_Ax()
        assert its0 == its and np.array_equal(m.du(), du)
        m.set_option("cg_dix", 1)
        # the same matrix with exceptions refused: AIJ-split, bit-exact too
        m.set_option("vi_exc_max", 0)
        m.assembly_jac()
        assert m.get_info()["storage"] == 2 and m.get_info()["vi_exc_nodes"] == 0
        assert np.array_equal(m.dump_csr()[2], v1)


@pytest.mark.parametrize("grid", [(130, 9, 12), (70, 20, 7)])
def test_aij_vi_exact_rows_end_to_end(grid):
    """-mat_vi_fma 0 (the exact rows: products and sums in the inode kernel's order, as the
    reference's MatMult) through the whole Newton step on the production 64x16 tiles: every
    SpMV of the solve equals the oracle's bit for bit, so only the CG's dot-product reduction
    order differs — the iteration count equals the oracle's and du is within 1e-10."""
    NX, NY, NZ = grid
    rtol = 1e-12
    P = O.Problem(NX, NY, NZ, rtol=rtol)
    out = P.newton_step1()
    with M.Macroc(argv_for(NX, NY, NZ, rtol, ["-mat_vi_fma", 0])) as m:
        m.set_option("vi_stage", 1)  # the grid is too flat for the default rule (>= 4 planes per chunk)
        for ts in (0, 1):
            m.apply_bc_on_u(m.get_displacement(ts))
        m.set_strains(); m.homogenize(); m.assembly_res(); m.assembly_jac()
        info = m.get_info()
        assert info["storage"] == 3 and (info["spmv_tx"], info["spmv_ty"]) == (64, 16), info
        x = np.random.default_rng(3).uniform(-1, 1, m.n)
        assert np.array_equal(m.spmv(x), P.spmv(x))
        its, rn, reason = m.solve_Ax()
        assert reason == out["reason"] and its == out["its"], (its, out["its"])
        assert np.linalg.norm(m.du() - P.du()) <= 1e-10 * np.linalg.norm(P.du())


def _exc_waves_per_plane(P, NX, NY, NZ, TX=64, TY=16):
    """Host restatement of which staged-SpMV waves hold exception nodes: the owned nodes of the
    elements with a Gauss-point tangent other than the elastic branch's (the mode of ctan), mapped
    to (tile, plane) -> set of 16x4-patch waves under the Latin-square layout (vi_wmap 1)."""
    ct = P.ctan().reshape(-1, 8, 36)
    vals, counts = np.unique(ct.reshape(-1, 36), axis=0, return_counts=True)
    cref = vals[np.argmax(counts)]
    nonplain = np.nonzero(np.any(np.any(ct != cref, axis=2), axis=1))[0]
    ex, ey, ez = nonplain % (NX - 1), (nonplain // (NX - 1)) % (NY - 1), nonplain // ((NX - 1) * (NY - 1))
    waves = {}
    for a in (0, 1):
        for b_ in (0, 1):
            for c in (0, 1):
                for i, j, k in zip(ex + a, ey + b_, ez + c):
                    lx, ly = i % TX, j % TY
                    px, py = lx // 16, ly // 4
                    wq = py * 4 + ((px + py) & 3) + 16 * (px // 4)
                    waves.setdefault((i // TX, j // TY, k), set()).add(wq)
    return waves


def test_aij_vi_exception_pass_deterministic():
    """The exception rows are deterministic by construction: slots come from an ordered
    compaction (owned-node order, not an atomic counter), the exception kernel's thread -> slot map
    and block partials are fixed (default), and round 4's block-wide pass (vi_exc_kernel 0) fills
    one list segment per wave in (plane, lane) order (ballot).  Precondition asserted: some tile
    plane holds exception nodes in two or more waves.  Repeated solves (default FMA rows, and
    -mat_vi_fma 0; both exception forms) are bitwise equal, with equal iteration counts; the slot
    order is the owned-node order (the matrix dump's exception blocks are read through it)."""
    NX, NY, NZ = 130, 9, 12
    rtol = 1e-10
    P, u = plastic_state(NX, NY, NZ, rtol=rtol)
    waves = _exc_waves_per_plane(P, NX, NY, NZ)
    assert max(len(w) for w in waves.values()) >= 2, waves
    argv = ["-da_grid_x", NX, "-da_grid_y", NY, "-da_grid_z", NZ, "-dt", 0.01, "-mat_law", "plastic",
            "-ksp_rtol", repr(rtol)]
    with M.Macroc(argv) as m:
        m.set_option("vi_stage", 1)  # the staged 64x16 tiles (the grid is too flat for the default rule)
        m.set_u(u)
        m.set_strains(); m.homogenize(); m.assembly_res(); m.assembly_jac()
        info = m.get_info()
        assert info["storage"] == 3 and info["vi_exc_nodes"] > 0 and (info["spmv_tx"], info["spmv_ty"]) == (64, 16)
        assert np.array_equal(m.dump_csr()[2], P.A_values())
        for xk in (1, 0):
            m.set_option("vi_exc_kernel", xk)
            for fma in (1, 0):
                m.set_option("vi_fma", fma)
                runs = []
                for _ in range(3):
                    its, rn, reason = m.solve_Ax()
                    runs.append((its, rn, m.du().copy()))
                assert reason > 0
                for its, rn, du in runs[1:]:
                    assert its == runs[0][0] and rn == runs[0][1] and np.array_equal(du, runs[0][2]), (xk, fma)
        # assembled again: the same slots, the same solve
        m.assembly_jac()
        its, rn, reason = m.solve_Ax()
        assert its == runs[0][0] and np.array_equal(m.du(), runs[0][2])


@pytest.mark.parametrize("name", SINGLE)
def test_aij_split_single_rank(name):
    """AIJ-split storage: upper blocks + bf16 lower corrections.  Every AIJ value is
    reconstructed bit for bit (matrix dump == oracle), the SpMV rows differ from the CPU order
    by rounding only (<= 1e-14 of sum |a_ij x_j|), the solve meets the north-star bar."""
    fx = load(name)
    NX, NY, NZ = (int(v) for v in fx["grid"])
    rtol = float(fx["rtol"])
    P = O.Problem(NX, NY, NZ, rtol=rtol)
    with M.Macroc(argv_for(NX, NY, NZ, rtol, ["-mat_aij_vi", 0])) as m:
        m.set_option("split_maxq", 30)  # tiny grids are boundary-dominated: dense corrections
        for ts in (0, 1):
            m.apply_bc_on_u(m.get_displacement(ts))
            P.apply_bc_u(m.get_displacement(ts))
        m.set_strains(); m.homogenize(); m.assembly_res()
        P.set_strains(); P.homogenize(); P.assembly_res()
        m.assembly_jac()
        P.assembly_jac()
        info = m.get_info()
        assert info["storage"] == 2 and 0 <= info["split_slots"] <= 117  # 0: exactly symmetric
        rp, ci, v = m.dump_csr()
        assert np.array_equal(v, P.A_values())
        x = np.random.default_rng(42).uniform(-1, 1, m.n)
        y, y_ref = m.spmv(x), P.spmv(x)
        absrow = np.add.reduceat(np.abs(v) * np.abs(x[ci]), rp[:-1])
        assert np.all(np.abs(y - y_ref) <= 1e-14 * absrow + 1e-300)
        assert np.array_equal(m.spmv(x), y)
        its, rn, reason = m.solve_Ax()
        assert abs(its - int(fx["its"])) <= 1
        ref = fx["du"]
        if np.linalg.norm(ref) > 0:
            assert np.linalg.norm(m.du() - ref) <= du_tol(rtol) * np.linalg.norm(ref)


@pytest.mark.parametrize("maxq,wide,dense,storage", [(4, 0, 0, 0), (4, 0, 1, 2), (4, 1, 1, 2), (30, 0, 1, 2),
                                                     (30, 1, 1, 2)])
def test_aij_split_dense_plastic(maxq, wide, dense, storage):
    """A plastic tangent fills all 117 correction slots.  Beyond split_maxq quads per node the
    split storage keeps all 120 slots in canonical order and adds them in a second pass
    (split_dense 1, the default) or the AIJ blocks are used (split_dense 0); within maxq the
    z-march walks them; bf16 or f32 (forced) — the matrix is bit-exact either way, the SpMV
    within rounding."""
    NX, NY, NZ, dt = 12, 10, 12, 0.05
    P = O.Problem(NX, NY, NZ, rtol=1e-10, law=1, dt=dt, bc_type=0)
    P.apply_bc_u(P.get_displacement(1))
    P.set_strains(); P.homogenize(); P.assembly_res(); P.assembly_jac(); P.solve(); P.update_u()
    u = P.u()
    P.set_strains(); P.homogenize(); P.assembly_jac()
    assert P.nonlinear_gps()[0] > 0
    argv = ["-da_grid_x", NX, "-da_grid_y", NY, "-da_grid_z", NZ, "-dt", dt, "-mat_law", "plastic", "-bc_type", 0]
    with M.Macroc(argv) as m:
        m.set_option("split_maxq", maxq)
        m.set_option("split_wide", wide)
        m.set_option("split_dense", dense)
        m.apply_bc_on_u(m.get_displacement(1))
        m.set_strains(); m.homogenize(); m.assembly_res(); m.assembly_jac(); m.solve_Ax(); m.update_u()
        m.set_u(u)
        m.set_strains(); m.homogenize(); m.assembly_jac()
        info = m.get_info()
        assert info["storage"] == storage
        if storage == 2:
            assert info["split_slots"] > 32 and info["split_bits"] == (32 if wide else 16)
        rp, ci, v = m.dump_csr()
        assert np.array_equal(v, P.A_values())
        x = np.random.default_rng(9).uniform(-1, 1, m.n)
        y, y_ref = m.spmv(x), P.spmv(x)
        absrow = np.add.reduceat(np.abs(v) * np.abs(x[ci]), rp[:-1])
        assert np.all(np.abs(y - y_ref) <= 1e-14 * absrow + 1e-300)


@pytest.mark.parametrize("esc", [1, 0])
def test_aij_split_dense_escapes(esc):
    """Dense plastic corrections (BC_BENDING, J2: every node plastic) where some correction is not
    exact in bf16 (12^3: one of 174,276 lower entries needs 9 significant bits): with split_esc 1
    (default) the corrections stay bf16 and that one keeps its truncated bf16 hi plus an exact
    double residual (an escape, added after the node's 120 slots in the dense pass); with
    split_esc 0 the whole matrix takes f32 corrections.  Either way the matrix is bit-exact with
    the oracle's AIJ, the SpMV within rounding, and the two products agree to rounding."""
    NX, NY, NZ, dt = 12, 12, 12, 0.05
    P = O.Problem(NX, NY, NZ, rtol=1e-10, law=1, dt=dt, bc_type=0)
    P.apply_bc_u(P.get_displacement(1))
    P.set_strains(); P.homogenize(); P.assembly_res(); P.assembly_jac(); P.solve(); P.update_u()
    u = P.u()
    P.set_strains(); P.homogenize(); P.assembly_res(); P.assembly_jac()
    argv = ["-da_grid_x", NX, "-da_grid_y", NY, "-da_grid_z", NZ, "-dt", dt, "-mat_law", "plastic", "-bc_type", 0,
            "-ksp_rtol", "1e-10"]
    with M.Macroc(argv) as m:
        m.set_option("split_esc", esc)
        m.set_u(u)
        m.set_strains(); m.homogenize(); m.assembly_jac()
        info = m.get_info()
        assert info["storage"] == 2, info
        if esc:
            assert info["split_bits"] == 16 and info["split_escapes"] > 0, info
        else:
            assert info["split_bits"] == 32 and info["split_escapes"] == 0, info
        rp, ci, v = m.dump_csr()
        assert np.array_equal(v, P.A_values())
        x = np.random.default_rng(13).uniform(-1, 1, m.n)
        y, y_ref = m.spmv(x), P.spmv(x)
        absrow = np.add.reduceat(np.abs(v) * np.abs(x[ci]), rp[:-1])
        assert np.all(np.abs(y - y_ref) <= 1e-14 * absrow + 1e-300)
        assert np.array_equal(m.spmv(x), y)
        m.assembly_res()
        its, rn, reason = m.solve_Ax()
        ref = P.solve()
        assert reason == 2 and abs(its - ref["its"]) <= 2
        assert np.linalg.norm(m.du() - P.du()) <= 50 * 1e-10 * np.linalg.norm(P.du())


def test_time_loop_matches_oracle_log():
    """mcx_time_step over -ts 2 on the BASELINE config-1 grid (4x4x2) against orc_run."""
    P = O.Problem(4, 4, 2, ts=2)
    with M.Macroc(["-da_grid_x", 4, "-da_grid_y", 4, "-da_grid_z", 2, "-ts", 2]) as m:
        out0 = m.time_step(0)
        assert out0["newton_its"] == 0 and out0["res"][0] == 0.0
        out1 = m.time_step(1)
    P.apply_bc_u(P.get_displacement(0))
    ref = P.newton_step1()
    assert out1["newton_its"] == 1
    assert abs(out1["res"][0] - ref["res"]) <= 1e-14 * ref["res"]  # VecNorm: reduction order only
    assert abs(out1["ksp_its"][0] - ref["its"]) <= 1
    # second Newton residual is below newton_rel_tol * |RES_0| (src/main.c:73)
    assert out1["res"][1] < 1e-4 * out1["res"][0]


def test_bending_bc_parity():
    NX, NY, NZ = 6, 4, 5
    P = O.Problem(NX, NY, NZ, bc_type=0, rtol=1e-12)
    with M.Macroc(argv_for(NX, NY, NZ, 1e-12, ["-bc_type", 0])) as m:
        assert np.array_equal(m.dump_dirichlet(), P.dirichlet_set())
        P.apply_bc_u(P.get_displacement(1))
        m.apply_bc_on_u(m.get_displacement(1))
        assert np.array_equal(m.u(), P.u())
        for f in ("set_strains", "homogenize"):
            getattr(m, f)()
        P.set_strains()
        P.homogenize()
        m.assembly_res()
        P.assembly_res()
        assert np.array_equal(m.b(), P.b())
        m.assembly_jac()
        P.assembly_jac()
        assert np.array_equal(m.dump_csr()[2], P.A_values())
        m.solve_Ax()
        P.solve()
        assert np.linalg.norm(m.du() - P.du()) <= 1e-10 * np.linalg.norm(P.du())


def test_ksp_edge_cases():
    """maxits hit -> DIVERGED_ITS with its == maxits; zero rhs -> converged at its 0."""
    with M.Macroc(argv_for(8, 8, 8, 1e-12, ["-ksp_max_it", 5])) as m:
        m.apply_bc_on_u(m.get_displacement(1))
        m.set_strains()
        m.homogenize()
        m.assembly_res()
        m.assembly_jac()
        its, rn, reason = m.solve_Ax()
        assert (its, reason) == (5, -3)
    with M.Macroc(argv_for(5, 2, 2, 1e-5)) as m:
        m.apply_bc_on_u(m.get_displacement(1))
        m.set_strains()
        m.homogenize()
        assert m.assembly_res() == 0.0
        m.assembly_jac()
        its, rn, reason = m.solve_Ax()
        assert its == 0 and reason in (2, 3)


@pytest.mark.parametrize("maxits", [1, 2, 5])
def test_ksp_maxits_iterate(maxits):
    """DIVERGED_ITS after 1, 2, 5 iterations returns the iterate of the last one: KSPSolve_CG
    applies x += alpha p before its stopping test, and the device loop defers that update into
    the next p update (k_cg_xfinal applies the last one)."""
    N, rtol = 8, 1e-12
    P = O.Problem(N, N, N, rtol=rtol, maxits=maxits)
    P.apply_bc_u(P.get_displacement(1))
    P.set_strains(); P.homogenize(); P.assembly_res(); P.assembly_jac()
    out = P.solve()
    with M.Macroc(argv_for(N, N, N, rtol, ["-ksp_max_it", maxits])) as m:
        m.apply_bc_on_u(m.get_displacement(1))
        m.set_strains(); m.homogenize(); m.assembly_res(); m.assembly_jac()
        its, rn, reason = m.solve_Ax()
        assert (its, reason) == (out["its"], out["reason"]) == (maxits, -3)
        du = m.du()
    assert np.linalg.norm(du) > 0
    assert np.linalg.norm(du - P.du()) <= 1e-12 * np.linalg.norm(P.du())


def _solve_big(N, rtol):
    m = M.Macroc(argv_for(N, N, N, rtol))
    m.apply_bc_on_u(m.get_displacement(1))
    m.set_strains()
    m.homogenize()
    res = m.assembly_res()
    m.assembly_jac()
    its, rn, reason = m.solve_Ax()
    return m, res, its, reason


def test_64cubed_properties():
    """BASELINE config 2 (64^3, rtol 1e-8): convergence, true residual, symmetry, linearity,
    determinism of assembly + SpMV."""
    m, res, its, reason = _solve_big(64, 1e-8)
    try:
        assert reason == 2 and 650 <= its <= 800  # scipy restatement: 720
        b, du = m.b(), m.du()
        r = m.spmv(du) - b
        assert np.linalg.norm(r) <= 1e-4 * np.linalg.norm(b)
        rng = np.random.default_rng(7)
        x, y = rng.uniform(-1, 1, m.n), rng.uniform(-1, 1, m.n)
        Ax, Ay = m.spmv(x), m.spmv(y)
        assert abs(y @ Ax - x @ Ay) <= 1e-12 * np.linalg.norm(Ax) * np.linalg.norm(y)
        np.testing.assert_allclose(m.spmv(2.0 * x + y), 2.0 * Ax + Ay, rtol=1e-12, atol=1e-6)
        v1 = m.dump_csr()[2]
        m.assembly_jac()
        assert np.array_equal(m.dump_csr()[2], v1)
        assert np.array_equal(m.spmv(x), Ax)
    finally:
        m.finish()


@pytest.mark.parametrize("NX,NY,NZ", [(8, 8, 8), (16, 16, 16), (12, 7, 9), (130, 6, 5)])
def test_sbaij_single_rank(NX, NY, NZ):
    """-dm_mat_type sbaij: matrix bit-exact vs the oracle's MATSBAIJ emulation; the pull SpMV
    (spmv_kernel 0) bit-exact too.  The z-marching kernels (1..11, one the default) add the mirrored
    lower blocks as whole 3-vectors, so their rows differ from the oracle's order by rounding
    only: checked to 1e-14 of sum|a||x| per row, and run-to-run identical (no atomics).  The
    solution agrees with the reference's AIJ path within the north-star tolerance."""
    rtol = 1e-12
    P = O.Problem(NX, NY, NZ, rtol=rtol)
    ref_aij = O.Problem(NX, NY, NZ, rtol=rtol)
    ref_aij.newton_step1()
    with M.Macroc(argv_for(NX, NY, NZ, rtol, ["-dm_mat_type", "sbaij", "-mat_ignore_lower_triangular"])) as m:
        for ts in (0, 1):
            m.apply_bc_on_u(m.get_displacement(ts))
            P.apply_bc_u(P.get_displacement(ts))
        m.set_strains(); m.homogenize(); m.assembly_res()
        P.set_strains(); P.homogenize(); P.assembly_res()
        m.assembly_jac()
        P.assembly_jac()
        P.sbaij_mirror()
        rp, ci, v = m.dump_csr()
        assert np.array_equal(v, P.A_values())
        x = np.random.default_rng(5).uniform(-1, 1, m.n)
        y_ref = P.spmv(x)
        absrow = np.add.reduceat(np.abs(v) * np.abs(x[ci]), rp[:-1])  # sum |a_ij x_j| per row
        phased = []
        for kern in range(12):
            m.set_option("spmv_kernel", kern)
            y = m.spmv(x)
            if kern == 0:
                assert np.array_equal(y, y_ref)
            else:
                assert np.all(np.abs(y - y_ref) <= 1e-14 * absrow + 1e-300), kern
                assert np.array_equal(m.spmv(x), y), kern
            if kern >= 7:
                phased.append(y)
        # phased kernels: one canonical row order whatever the tile shape (LDS or pulled terms)
        for y in phased[1:]:
            assert np.array_equal(y, phased[0])
        m.set_option("spmv_kernel", 7 if NX >= 128 else 8)  # the init-time default
        its, rn, reason = m.solve_Ax()
        o_its = P.solve()["its"]
        assert abs(its - o_its) <= 1
        du = m.du()
        assert np.linalg.norm(du - P.du()) <= 1e-10 * np.linalg.norm(P.du())
        assert np.linalg.norm(du - ref_aij.du()) <= 1e-10 * np.linalg.norm(ref_aij.du())


@pytest.mark.parametrize("NX,NY,NZ", [(70, 40, 9), (64, 64, 12)])
def test_aij_split_tile_shapes(NX, NY, NZ):
    """AIJ-split SpMV over every tile shape (256x4 default, 256x2, 128x4, 128x8, 64x4, 64x16;
    partial tiles at 70 x 40): y-edge terms come from helper threads, x-edge and partial-tile
    terms are pulled by the target, in-tile ones arrive through LDS, yet every row adds its terms
    in one canonical order — results bitwise equal across shapes, rows within 1e-14 sum|a||x|
    of the oracle's CPU order."""
    P = O.Problem(NX, NY, NZ, rtol=1e-8)
    with M.Macroc(argv_for(NX, NY, NZ, 1e-8, ["-mat_aij_vi", 0])) as m:
        m.set_option("split_maxq", 30)
        for ts in (0, 1):
            m.apply_bc_on_u(m.get_displacement(ts))
            P.apply_bc_u(P.get_displacement(ts))
        m.set_strains(); m.homogenize(); m.assembly_res(); m.assembly_jac()
        P.set_strains(); P.homogenize(); P.assembly_res(); P.assembly_jac()
        assert m.get_info()["storage"] == 2
        rp, ci, v = m.dump_csr()
        assert np.array_equal(v, P.A_values())
        x = np.random.default_rng(11).uniform(-1, 1, m.n)
        y_ref = P.spmv(x)
        absrow = np.add.reduceat(np.abs(v) * np.abs(x[ci]), rp[:-1])
        ys = []
        for tx, ty in ((0, 0), (256, 2), (128, 4), (128, 8), (64, 4), (64, 16), (256, 4)):
            m.set_option("split_tx", tx)
            m.set_option("split_ty", ty)
            y = m.spmv(x)
            assert np.all(np.abs(y - y_ref) <= 1e-14 * absrow + 1e-300), (tx, ty)
            ys.append(y)
        for y in ys[1:]:
            assert np.array_equal(y, ys[0])


@pytest.mark.parametrize("vi_tx,tile", [(0, (64, 16)), (128, (128, 8)), (256, (256, 4))])
@pytest.mark.parametrize("NX,NY,NZ", [(260, 6, 5), (130, 9, 6), (70, 20, 7)])
def test_aij_vi_production_tiles(NX, NY, NZ, vi_tx, tile):
    """The headline kernel at the tile shapes it runs (k_spmv_vibm 64x16, the default, and the
    selectable 128x8 / 256x4), with partial tiles in x (260 = 4 x 64 + 4 = 256 + 4, 130,
    70) and y (6, 9, 20 rows against 16 / 8 / 4), with per-lane block indices (default) and the
    wave descriptors (vi_wdesc 1: a uniform wave's indices from its patch record; 2: two-set waves
    in one pass per set; bitwise the same rows): matrix dump bit-exact, and the SpMV bit-exact with the
    oracle's CPU AIJ (MatMult_SeqAIJ_Inode order, the MATAIJ matrix of src/init.c:92 applied by
    KSPSolve, src/assembly.c:179-192) under -mat_vi_fma 0 for several z-chunkings and wave
    layouts; the default fused multiply-add rows within 1e-14 sum|a||x|; the solve within the
    north-star bar."""
    rtol = 1e-12
    P = O.Problem(NX, NY, NZ, rtol=rtol)
    with M.Macroc(argv_for(NX, NY, NZ, rtol)) as m:
        m.set_option("vi_stage", 1)  # the grid is too flat for the default rule (>= 4 planes per chunk)
        m.set_option("vi_tx", vi_tx)
        for ts in (0, 1):
            m.apply_bc_on_u(m.get_displacement(ts))
            P.apply_bc_u(P.get_displacement(ts))
        m.set_strains(); m.homogenize(); m.assembly_res(); m.assembly_jac()
        P.set_strains(); P.homogenize(); P.assembly_res(); P.assembly_jac()
        info = m.get_info()
        assert info["storage"] == 3 and info["vi_blocks"] > 0, info
        assert (info["spmv_tx"], info["spmv_ty"]) == tile, info
        rp, ci, v = m.dump_csr()
        assert np.array_equal(v, P.A_values())
        x = np.random.default_rng(17).uniform(-1, 1, m.n)
        y_ref = P.spmv(x)
        absrow = np.add.reduceat(np.abs(v) * np.abs(x[ci]), rp[:-1])
        for zblocks in (0, 1, 2, 3 * NZ):  # chunks of 1, NZ, NZ/2, ... planes per tile
            m.set_option("spmv_zblocks", zblocks)
            # -mat_vi_fma 0: the reference's MatMult order (inode column pairs), bit-exact (scalar-dictionary 16x4 patches, row
            # quarters, every block from LDS); the default fused multiply-adds: within rounding
            m.set_option("vi_wdesc", 0)  # per-lane index words (the descriptors are the default, below)
            for uni, patch in ((1, 1), (1, 0), (0, 0)):
                m.set_option("vi_fma", 0)
                m.set_option("vi_uni", uni)
                m.set_option("vi_patch", patch)
                assert np.array_equal(m.spmv(x), y_ref), (zblocks, uni, patch)
            m.set_option("vi_uni", 1)
            m.set_option("vi_patch", 1)
            m.set_option("vi_wdesc", 1)  # uniform waves' block indices from the wave descriptors
            assert np.array_equal(m.spmv(x), y_ref), (zblocks, "wdesc")
            m.set_option("vi_wdesc", 0)
            m.set_option("vi_ypair", 1)  # the scalar path's y as 16-B lane-pair stores: the same rows
            assert np.array_equal(m.spmv(x), y_ref), (zblocks, "ypair")
            m.set_option("vi_ypair", 0)
            m.set_option("vi_fma", 1)
            yf = m.spmv(x)
            assert np.all(np.abs(yf - y_ref) <= 1e-14 * absrow + 1e-300), zblocks
            assert np.array_equal(m.spmv(x), yf)
            # the default-stencil kernel (64 x 16 tiles, the default there) and the per-node index
            # path compute the same FMA rows: bitwise
            m.set_option("vi_st", 0)
            assert np.array_equal(m.spmv(x), yf), (zblocks, "vi_st 0")
            m.set_option("vi_st", 1)
            assert np.array_equal(m.spmv(x), yf), (zblocks, "vi_st 1")
            m.set_option("vi_st_tail", 1)  # the faces and listed rows by the march blocks instead of k_spmv_face
            assert np.array_equal(m.spmv(x), yf), (zblocks, "vi_st_tail 1")
            m.set_option("vi_st_tail", 0)
            m.set_option("vi_ypair", 1)
            assert np.array_equal(m.spmv(x), yf), (zblocks, "ypair")
            m.set_option("vi_ypair", 0)
            for lg in (2, 3):  # LDS-dictionary waves: the reads of 2 / 3 blocks issued together
                m.set_option("vi_lg", lg)
                assert np.array_equal(m.spmv(x), yf), (zblocks, "vi_lg", lg)
            m.set_option("vi_lg", 1)
            m.set_option("vi_wdesc", 1)
            assert np.array_equal(m.spmv(x), yf), (zblocks, "wdesc")
            m.set_option("vi_wdesc", 2)  # two-set waves: one scalar pass per set, each lane keeping its own
            assert np.array_equal(m.spmv(x), yf), (zblocks, "two-set")
            m.set_option("vi_fma", 0)
            assert np.array_equal(m.spmv(x), y_ref), (zblocks, "two-set exact")
            m.set_option("vi_fma", 1)
            m.set_option("vi_wdesc", 0)
        m.set_option("spmv_zblocks", 1)  # every tile marches all planes: the prefetch ring end to end
        assert m.get_info()["spmv_kc"] == NZ
        its, rn, reason = m.solve_Ax()
        out = P.solve()
        assert reason == out["reason"] and abs(its - out["its"]) <= 1
        assert np.linalg.norm(m.du() - P.du()) <= 1e-10 * np.linalg.norm(P.du())



def test_round4_options_refused():
    """The round-4 A/B options take their documented values only; a refused value raises and
    leaves the setting as it was (the solve after it matches the one before)."""
    with M.Macroc(argv_for(24, 20, 12, 1e-10)) as m:
        m.apply_bc_on_u(m.get_displacement(1))
        m.set_strains(); m.homogenize(); m.assembly_res(); m.assembly_jac()
        its0, _, _ = m.solve_Ax()
        du0 = m.du()
        for name, bad in (("vi_lg", 4), ("vi_lg", 0), ("vi_wdesc", 3), ("cg_ublocks", -1), ("cg_ublocks", 2.5)):
            with pytest.raises(M.MacrocError):
                m.set_option(name, bad)
        its1, _, _ = m.solve_Ax()
        assert its1 == its0 and np.array_equal(m.du(), du0)


@pytest.mark.parametrize("N", [37, 48])
def test_st_face_classes(N):
    """The default-stencil SpMV's stencil classes (k_st_setup): the interior is marched, the 6 domain
    faces computed in patches with their class's stencil (st_faces); only edge / corner nodes, nodes
    next to Dirichlet nodes and exception nodes are listed.  On a cube (37: partial tiles, patches
    and face patches, an odd plane count against the two-plane steps; 48: whole tiles) the rows are
    bitwise the per-node index path's (vi_st 0), with the faces in k_spmv_face (default) and in the
    march blocks' tail, and the listed count is a small fraction of the face nodes."""
    rtol = 1e-12
    P = O.Problem(N, N, N, rtol=rtol)
    with M.Macroc(argv_for(N, N, N, rtol)) as m:
        m.set_option("vi_stage", 1)  # the staged tiles (at this size the default rule chunks z finer)
        m.set_option("vi_st", 1)  # (by default from 2^23 nodes)
        for ts in (0, 1):
            m.apply_bc_on_u(m.get_displacement(ts))
            P.apply_bc_u(P.get_displacement(ts))
        m.set_strains(); m.homogenize(); m.assembly_res(); m.assembly_jac()
        P.set_strains(); P.homogenize(); P.assembly_res(); P.assembly_jac()
        x = np.random.default_rng(5).uniform(-1, 1, m.n)
        y_ref = P.spmv(x)
        rp, ci, v = m.dump_csr()
        absrow = np.add.reduceat(np.abs(v) * np.abs(x[ci]), rp[:-1])
        info = m.get_info()
        faces = 6 * (N - 2) ** 2
        assert 0 < info["st_listed"] < faces // 4, (info["st_listed"], faces)
        y = m.spmv(x)
        assert np.all(np.abs(y - y_ref) <= 1e-14 * absrow + 1e-300)
        for zblocks in (0, 1, 5):
            m.set_option("spmv_zblocks", zblocks)
            y = m.spmv(x)
            m.set_option("vi_st", 0)
            assert np.array_equal(m.spmv(x), y), zblocks
            m.set_option("vi_st", 1)
            m.set_option("vi_st_tail", 1)
            assert np.array_equal(m.spmv(x), y), zblocks
            m.set_option("vi_st_tail", 0)
            for l16 in (0, 1):  # listed rows one thread per node (st_tail) / 16 lanes per node (st_tail16)
                m.set_option("vi_st_l16", l16)
                assert np.array_equal(m.spmv(x), y), (zblocks, "l16", l16)
            m.set_option("vi_st_l16", -1)
            m.set_option("vi_st_fstream", 1)  # the face kernel on its own stream beside the march
            assert np.array_equal(m.spmv(x), y), (zblocks, "fstream")
            m.set_option("vi_st_fstream", 0)
            # the x-pair march k_spmv_sp (round 6), 64 x 16 and 64 x 8 tiles: the same rows
            m.set_option("vi_st_pair", 1)
            for ty in (16, 8):
                m.set_option("vi_st_ty", ty)
                assert np.array_equal(m.spmv(x), y), (zblocks, "sp", ty)
            m.set_option("vi_st_pair", 0)


@pytest.mark.parametrize("maxits", [None, 37, 38, 39, 40, 1, 2, 3, 4, 5])
@pytest.mark.parametrize("storage", ["vi", "vi_staged", "split"])
def test_cg_pdb_bitwise(maxits, storage):
    """Option cg_pdb 1: p double-buffered and VecAXPY(x) applied on odd iterations only, both
    owed terms in PETSc's order, the rest by k_cg_xfinal; cg_pdb 4 (the default): four buffers,
    the four owed terms every fourth iteration (cg_xs 1: eight buffers, the four terms by k_cg_xwin
    on a side stream beside the next iterations) — bitwise the solve of the single-buffer p
    update: converged, and stopped by maxits at every residue mod 4 (1 to 5 included); with and
    without the parity-specialised kernels (cg_par 1), with a deliberately wrong parity hint
    (cg_par 2: the kernels follow the device's count) and the reversed node order
    (cg_rev)."""
    NX, NY, NZ = 70, 20, 12
    extra = ["-mat_aij_vi", 0] if storage == "split" else []
    argv = argv_for(NX, NY, NZ, 1e-12, extra) + (["-ksp_max_it", maxits] if maxits else [])
    out = []
    with M.Macroc(argv) as m:
        m.set_option("cg_fuse", 0)  # the unfused scalar steps (grids > 1,024 update blocks)
        if storage == "vi_staged":  # the z-marching SpMV (idle blocks included)
            m.set_option("vi_stage", 1)
        m.apply_bc_on_u(m.get_displacement(1))
        m.set_strains(); m.homogenize(); m.assembly_res(); m.assembly_jac()
        for pdb, par, rev, xs, p2d in ((0, 0, 0, 0, 0), (1, 0, 0, 0, 0), (0, 1, 0, 0, 0), (1, 1, 0, 0, 0), (1, 1, 1, 0, 0),
                                       (1, 0, 1, 0, 0), (4, 0, 0, 0, 0), (4, 1, 0, 0, 0), (4, 1, 1, 0, 0), (4, 1, 0, 1, 0),
                                       (4, 0, 1, 1, 0), (4, 1, 0, 0, 1), (4, 2, 0, 0, 0), (4, 2, 1, 0, 0),
                                       (1, 2, 0, 0, 0)):
            m.set_option("cg_pdb", pdb)
            m.set_option("cg_par", par)
            m.set_option("cg_rev", rev)
            m.set_option("cg_xs", xs)
            m.set_option("cg_p2d", p2d)
            its, rn, reason = m.solve_Ax()
            out.append((its, reason, m.du()))
    for its, reason, du in out[1:]:
        assert (its, reason) == out[0][:2] and np.array_equal(du, out[0][2])
    if maxits:
        assert out[0][:2] == (maxits, -3)

@pytest.mark.parametrize("st", [0, 1])
@pytest.mark.parametrize("maxits", [0, 5, 6])
def test_cg_fused_p_update_bitwise(maxits, st):
    """Option cg_fusep: the CG's p update inside the value-indexed SpMV (two p buffers) and
    VecAXPY(x) every second iteration in the update kernel give bitwise the solve of the separate
    kernels — converged, and stopped by maxits after an odd and an even number of iterations
    (the pending x update of the last iteration, k_cg_xfinal).  vi_st 0: k_spmv_vibm's FP march;
    vi_st 1 (+ vi_st_pair 1): the default-stencil march k_spmv_sp's FP instantiation (round 6), then k_spmv_face
    from p's buffer of the iteration.  Both sides of a comparison run the same SpMV kernels (the
    default-stencil path sums p.Ap over other partials than k_spmv_vibm)."""
    NX, NY, NZ = 70, 20, 12
    argv = argv_for(NX, NY, NZ, 1e-12) + (["-ksp_max_it", maxits] if maxits else [])
    out = []
    with M.Macroc(argv) as m:
        m.set_option("vi_stage", 1)
        m.set_option("vi_st", st)
        m.set_option("vi_st_pair", st)  # the fused default-stencil march is k_spmv_sp's
        m.apply_bc_on_u(m.get_displacement(1))
        m.set_strains(); m.homogenize(); m.assembly_res(); m.assembly_jac()
        for fusep in (0, 1, 0):
            m.set_option("cg_fusep", fusep)
            its, rn, reason = m.solve_Ax()
            out.append((its, reason, m.du()))
    for its, reason, du in out[1:]:
        assert (its, reason) == out[0][:2] and np.array_equal(du, out[0][2])
    if maxits:
        assert out[0][:2] == (maxits, -3)


def test_partials_guard_near_the_limit():
    """the SpMV's partial sums (the march's blocks, then k_spmv_face's: its patches and
    listed-row blocks) must fit half of the partials buffer, because the fused update kernels read
    the SpMV's half while writing the other.  Every grid-changing option is checked against
    spmv_nparts (not just the march's grid): spmv_zblocks raised step by step with vi_st 1 (the
    march's grid grows to its cap of one plane per block) is either refused (the setting left as
    it was) or the solve stays the unperturbed one."""
    NX, NY, NZ = 70, 20, 12
    rtol = 1e-12
    with M.Macroc(argv_for(NX, NY, NZ, rtol)) as m:
        m.set_option("vi_stage", 1)
        m.set_option("vi_st", 1)
        m.apply_bc_on_u(m.get_displacement(1))
        m.set_strains(); m.homogenize(); m.assembly_res(); m.assembly_jac()
        assert m.get_info()["st_listed"] >= 0
        its0, _, reason0 = m.solve_Ax()
        du0 = m.du()
        refused = accepted = 0
        for zb in (1, 4, 16, 64, 256, 1024, 4096, 16384, 65536):
            try:
                m.set_option("spmv_zblocks", zb)
            except M.MacrocError as e:
                assert "partials buffer too small" in str(e)
                refused += 1
                continue
            accepted += 1
            its, _, reason = m.solve_Ax()
            assert reason == reason0 and abs(its - its0) <= 1, (zb, its, its0)
            assert np.linalg.norm(m.du() - du0) <= 1e-10 * np.linalg.norm(du0), zb
        assert accepted, (accepted, refused)
        # a refused value left the last accepted one in place: the solve is still the same
        its, _, reason = m.solve_Ax()
        assert reason == reason0 and abs(its - its0) <= 1
