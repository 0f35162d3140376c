"""The CPU oracle (test infrastructure) pinned against the reference's known answer and the
committed golden fixtures (tests/golden/, generated + cross-checked by make_golden.py)."""
import glob
import hashlib
import os

import numpy as np
import pytest

from oracle import oracle as O

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
CASES = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "g*.npz")))


def load(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def test_known_answer_test_dm_1():
    # tests/test_dm_1.c:5-19: 5x2 DMDA on 2 ranks, PETSc global ordering
    order = O.petsc_numbering(5, 2, 1, 2).reshape(2, 5)
    assert order.tolist() == [[0, 1, 2, 6, 7], [3, 4, 5, 8, 9]]
    assert O.dmda_decide(5, 2, 1, 2) == (2, 1, 1)


def test_decide_cube_8():
    assert O.dmda_decide(512, 512, 512, 8) == (2, 2, 2)
    assert O.dmda_decide(256, 256, 256, 1) == (1, 1, 1)
    assert O.dmda_decide(5, 3, 4, 8, 0, 0, 0)[0] * O.dmda_decide(5, 3, 4, 8)[1] * O.dmda_decide(5, 3, 4, 8)[2] == 8


def test_calc_B_fixture():
    Bo = np.stack([O.calc_B(gp) for gp in range(8)])
    assert np.array_equal(Bo, load("calc_B")["B"])


def _golden_module():
    import importlib.util
    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(GOLDEN, "make_golden.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_inode_pairing_by_hand():
    """MatMult_SeqAIJ_Inode's unrolled loop [ext]: sum += v0*x0 + v1*x1 per column pair, then the odd
    last term.  Terms chosen so the pairing shows in the rounding: (t0 + t1) + (t2 + t3) keeps the two
    sub-half-ulp terms' sum, ((t0 + t1) + t2) + t3 loses both; an odd row ends with its last term."""
    G = _golden_module()
    t = np.array([1.0, 0.0, 0.75e-16, 0.75e-16, 0.5, 0.25, 3.0])
    indptr = np.array([0, 4, 7])
    y_in = G.spmv(indptr, np.array([0, 1, 2, 3, 0, 1, 2]), t, np.ones(4), inode=True)
    y_pl = G.spmv(indptr, np.array([0, 1, 2, 3, 0, 1, 2]), t, np.ones(4), inode=False)
    assert y_in[0] == 1.0 + 2.0 ** -52 and y_pl[0] == 1.0
    assert y_in[1] == (0.0 + (0.5 + 0.25)) + 3.0


@pytest.mark.parametrize("grid,nranks", [((6, 5, 4), 1), ((6, 5, 4), 2), ((7, 4, 5), 3), ((6, 6, 6), 8)])
def test_spmv_orders_vs_numpy(grid, nranks):
    """The oracle's MatMult in both row orders (the MATAIJ inode kernel, the default; the plain
    SeqAIJ loop) against make_golden.py's independent numpy restatement, bit for bit, on an
    assembled matrix with Dirichlet rows and clipped boundary stencils; MPIAIJ = owned block
    then off-diagonal block.  The two orders differ, and both agree with scipy to rounding."""
    G = _golden_module()
    P = O.Problem(*grid, nranks=nranks)
    P.apply_bc_u(P.get_displacement(1))
    P.set_strains(); P.homogenize(); P.assembly_jac()
    rp, ci = P.csr()
    v = P.A_values()
    x = np.random.default_rng(11).uniform(-1, 1, P.ndofs)
    off = None if nranks == 1 else np.array([P.dof_offset(r) for r in range(nranks)] + [P.ndofs])
    y_in, y_pl = P.spmv(x), P.spmv(x, "plain")
    assert np.array_equal(y_in, P.spmv(x, "inode"))
    assert np.array_equal(y_in, G.spmv(rp, ci, v, x, off, inode=True))
    assert np.array_equal(y_pl, G.spmv(rp, ci, v, x, off, inode=False))
    assert not np.array_equal(y_in, y_pl)
    import scipy.sparse as sp
    ys = sp.csr_matrix((v, ci, rp), shape=(P.ndofs, P.ndofs)) @ x
    assert np.allclose(y_in, ys, rtol=1e-12, atol=1e-12 * np.abs(v).max())
    P.close()


@pytest.mark.parametrize("name", CASES)
def test_oracle_vs_golden(name):
    fx = load(name)
    NX, NY, NZ = (int(v) for v in fx["grid"])
    m, n, p = (int(v) for v in fx["decomp"])
    nr = int(fx["nranks"])
    P = O.Problem(NX, NY, NZ, nranks=nr, m=m, n=n, p=p, rtol=float(fx["rtol"]))
    # integer artefacts: bit-exact
    assert P.decomp() == (m, n, p)
    assert np.array_equal(P.dof_map(), fx["dof_map"])
    assert np.array_equal(P.dirichlet_set(), fx["dirichlet"])
    conn = np.concatenate([P.elements(r) for r in range(nr)])
    assert np.array_equal(conn, fx["conn"])
    assert np.array_equal(np.array([P.corners(r) for r in range(nr)]), fx["corners"])
    rp, ci = P.csr()
    assert sha(rp) == str(fx["csr_rowptr_sha"]) and sha(ci) == str(fx["csr_colidx_sha"])
    # floating point: the oracle is deterministic, so bit-exact against its own fixture
    out = P.newton_step1()
    assert out["its"] == int(fx["its"]) and out["reason"] == int(fx["reason"])
    assert np.array_equal(P.b(), fx["b"])
    assert np.array_equal(P.du(), fx["du"])
    assert np.array_equal(out["history"], fx["history"])
    if "A" in fx:
        assert np.array_equal(P.A_values(), fx["A"])
    # and the direct solve agrees where the solve is tight
    if float(fx["rtol"]) <= 1e-12:
        d = fx["du_direct"]
        assert np.linalg.norm(P.du() - d) <= 1e-9 * np.linalg.norm(d)
    P.close()


def test_ctest_grids_never_solve():
    # on 5x2x2 no node is inside the load circle -> zero residual, no KSPSolve
    fx = load("g522_r1")
    assert float(fx["res"]) == 0.0 and int(fx["its"]) == 0


def test_oracle_log_matches_reference_format(tmp_path):
    P = O.Problem(4, 4, 2, ts=2)
    log = tmp_path / "log.txt"
    P.run(str(log))
    txt = log.read_text()
    assert "Time Step = 1" in txt and "|RES| = 1.029218e+06" in txt
    assert "KSP : |Ax - b|/|Ax| = " in txt and "Its = 39" in txt


def test_oracle_force_and_info_rows(tmp_path):
    """Post-processing restatement (src/main.c:86-97, src/forces.c:115-166): the reaction force
    is a property of the field, so emulated rank grids with one rank in y agree to the solver
    tolerance (their CG dot products differ in summation order);
    the info.dat row has the reference's six tab-separated columns."""
    forces = []
    for nr in (1, 2, 4):
        P = O.Problem(41, 5, 41, ts=2, rtol=1e-10, nranks=nr)
        P.run(None, str(tmp_path / f"info{nr}.dat"), str(tmp_path / f"gauss{nr}.dat"))
        forces.append(P.calc_force())
        rows = (tmp_path / f"info{nr}.dat").read_text().splitlines()
        assert len(rows) == 2 and all(len(r.split("\t")) == 6 for r in rows)
        assert rows[1].split("\t")[:3] == ["1", "1.000000e-03", "-1.000000e-03"]
        assert len((tmp_path / f"gauss{nr}.dat").read_text().splitlines()[0].split("\t")) == nr + 2
        P.close()
    assert forces[0] < 0.0
    for f in forces[1:]:
        assert abs(f - forces[0]) <= 1e-9 * abs(forces[0])
