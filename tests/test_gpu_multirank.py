"""Multi-rank parity on one GPU: N contexts (one host thread each) over the in-process
transport run the decomposed path — halo exchanges, owner-computes assembly on subdomains,
all-reduced CG scalars — and must reproduce the single-rank answer.

Owner-computes makes every row independent of the rank grid: strains, residual, assembled
matrix and SpMV are bit-identical to the one-rank oracle in natural ordering; only the CG dot
products change summation order (its +-1, du within the north-star tolerance).  The RCCL
transport differs from this one only in the two calls that move the bytes.
"""
import os
import threading

import numpy as np
import pytest

import macroc_amd as M
from oracle import oracle as O

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def run_group(argv, nranks, fn, timeout=300):
    g = M.LocalGroup(nranks)
    results, errors = [None] * nranks, []

    def worker(r):
        try:
            m = M.Macroc(argv, rank=r, nranks=nranks, group=g)
            try:
                results[r] = fn(m)
            finally:
                m.finish()
        except Exception as e:  # surfaced below
            errors.append((r, e))

    ts = [threading.Thread(target=worker, args=(r,), daemon=True) for r in range(nranks)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout)
    assert not any(t.is_alive() for t in ts), f"group hung; errors={errors}"
    assert not errors, errors
    g.destroy()
    return results


def newton_step(x_global_nat, options=()):
    def fn(m):
        for k, v in options:
            m.set_option(k, v)
        petsc, nat = m.owned_dofs()
        m.apply_bc_on_u(m.get_displacement(0))
        m.apply_bc_on_u(m.get_displacement(1))
        m.set_strains()
        m.homogenize()
        res = m.assembly_res()
        m.assembly_jac()
        rp, ci, v = m.dump_csr()
        y = m.spmv(x_global_nat[nat])
        its, rn, reason = m.solve_Ax()
        m.update_u()
        return dict(petsc=petsc, nat=nat, b=m.b(), du=m.du(), u=m.u(), res=res, its=its, reason=reason,
                    rp=rp, ci=ci, v=v, y=y, dir=m.dump_dirichlet(), info=m.get_info())
    return fn


@pytest.mark.parametrize("name", ["g1088_r2", "g888_r8", "g522_r3", "g534_r8"])
def test_multirank_newton_step(name):
    """AIJ blocks in the reference's MatMult order (inode column pairs) (-mat_aij_split 0): SpMV bit-exact on any rank grid."""
    _multirank(name, sbaij=False, extra=["-mat_aij_vi", 0, "-mat_aij_split", 0])


@pytest.mark.parametrize("name", ["g1088_r2", "g888_r8", "g522_r3", "g534_r8"])
def test_multirank_aij_vi(name):
    """Default AIJ storage for the elastic law: value-indexed (one byte per value + a per-rank
    dictionary), rows in the reference's MatMult order (inode column pairs): matrix and SpMV bit-exact on any rank grid."""
    _multirank(name, sbaij=False, vi=True)


@pytest.mark.parametrize("name", ["g1088_r2", "g888_r8", "g534_r8"])
def test_multirank_aij_split(name):
    """AIJ-split storage (upper blocks + bf16 corrections): matrix bit-exact, SpMV rounding."""
    _multirank(name, sbaij=False, extra=["-mat_aij_vi", 0], split=True)


@pytest.mark.parametrize("name", ["g1088_r2", "g888_r8"])
def test_multirank_sbaij(name):
    _multirank(name, sbaij=True)


def _multirank(name, sbaij, extra=(), split=False, vi=False):
    fx = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    NX, NY, NZ = (int(v) for v in fx["grid"])
    nr = int(fx["nranks"])
    px, py, pz = (int(v) for v in fx["decomp"])
    rtol = float(fx["rtol"])
    argv = ["-da_grid_x", NX, "-da_grid_y", NY, "-da_grid_z", NZ, "-da_processors_x", px, "-da_processors_y", py,
            "-da_processors_z", pz, "-ksp_rtol", repr(rtol)] + (["-dm_mat_type", "sbaij"] if sbaij else []) + list(extra)
    ref = O.Problem(NX, NY, NZ, rtol=rtol)  # one rank: natural order == PETSc order
    x = np.random.default_rng(3).uniform(-1, 1, ref.ndofs)
    out = run_group(argv, nr, newton_step(x, [("split_maxq", 30)] if split else []))
    aij_du = None
    if sbaij:  # the sbaij classification is by natural index: decomposition independent
        ref.apply_bc_u(ref.get_displacement(0))
        ref.apply_bc_u(ref.get_displacement(1))
        ref.set_strains(); ref.homogenize(); ref.assembly_res(); ref.assembly_jac(); ref.sbaij_mirror()
        ref.solve(); ref.update_u()
    else:
        ref.newton_step1()
    A1 = {}
    rp1, ci1 = ref.csr()
    v1 = ref.A_values()
    y1 = ref.spmv(x)
    dm = fx["dof_map"]  # natural -> PETSc of the nr-rank decomposition
    inv = np.empty_like(dm)
    inv[dm] = np.arange(len(dm))
    b = np.zeros(ref.ndofs)
    du = np.zeros(ref.ndofs)
    dset = []
    for r, o in enumerate(out):
        assert np.array_equal(o["petsc"], dm[o["nat"]])  # integer artefact: bit-exact
        b[o["nat"]] = o["b"]
        du[o["nat"]] = o["du"]
        dset.append(o["dir"])
        if split:
            assert o["info"]["storage"] == 2
        if vi:
            assert o["info"]["storage"] == 3 and 0 < o["info"]["vi_values"] <= 256
        if sbaij or split:  # z-marching kernels: whole-3-vector mirrored terms, rounding-level
            absrow = np.add.reduceat(np.abs(v1) * np.abs(x[ci1]), rp1[:-1])
            assert np.all(np.abs(o["y"] - y1[o["nat"]]) <= 1e-14 * absrow[o["nat"]] + 1e-300)
        else:
            assert np.array_equal(o["y"], y1[o["nat"]])  # SpMV bit-exact
        assert abs(o["its"] - int(fx["its"])) <= 1 + (1 if sbaij or split else 0)
        assert o["res"] == out[0]["res"]
        # matrix rows: global PETSc columns, values bit-exact vs the one-rank matrix
        for q in range(len(o["nat"])):
            row_nat = o["nat"][q]
            cols_p = o["ci"][o["rp"][q]:o["rp"][q + 1]]
            vals = o["v"][o["rp"][q]:o["rp"][q + 1]]
            lo, hi = rp1[row_nat], rp1[row_nat + 1]
            ref_cols = ci1[lo:hi]
            ref_vals = v1[lo:hi]
            order = np.argsort(inv[cols_p])
            assert np.array_equal(inv[cols_p][order], ref_cols)
            assert np.array_equal(vals[order], ref_vals)
    assert np.array_equal(np.sort(np.concatenate(dset)), fx["dirichlet"])
    assert np.array_equal(b, ref.b())  # residual bit-exact in natural order
    assert abs(out[0]["res"] - ref.norm_b()) <= 1e-14 * max(ref.norm_b(), 1.0)
    duref = ref.du()
    if np.linalg.norm(duref) > 0:
        tol = 1e-10 if rtol <= 1e-12 else 50 * rtol
        assert np.linalg.norm(du - duref) <= tol * np.linalg.norm(duref)
    else:
        assert not du.any()


@pytest.mark.parametrize("mat", ["aij", "aij-tall", "aij-dense", "sbaij", "sbaij-phased"])
@pytest.mark.parametrize("grid,procs", [((140, 10, 8), (2, 1, 1)), ((132, 12, 12), (2, 2, 2))])
def test_multirank_full_tiles(grid, procs, mat):
    """Subdomains wide enough for full z-marching tiles (64 x 4) next to partial ones: internal
    subdomain faces at a tile's lane 0 and row 0 (helper-computed edge terms pulling real
    ghosts), at partial tiles' last lanes and rows (pulled by the target), and the global
    boundary (skipped ghosts).  Rows within rounding of the one-rank oracle's product, the
    solve within the north-star tolerance."""
    NX, NY, NZ = grid
    px, py, pz = procs
    nr, rtol = px * py * pz, 1e-10
    argv = ["-da_grid_x", NX, "-da_grid_y", NY, "-da_grid_z", NZ, "-da_processors_x", px, "-da_processors_y", py,
            "-da_processors_z", pz, "-ksp_rtol", repr(rtol), "-dm_mat_type", mat.split("-")[0]]
    if mat.startswith("aij"):
        argv += ["-mat_aij_vi", 0]  # the z-marching AIJ-split kernels
    # 8: phased 64x4; aij-tall: 64x16 AIJ-split tiles (internal x faces at every tile's lanes 0 / 63)
    # aij-dense: split_maxq 0 sends every correction to the dense second pass (k_split_dense)
    opts = {"aij": [("split_maxq", 30)], "aij-tall": [("split_maxq", 30), ("split_tx", 64), ("split_ty", 16)],
            "aij-dense": [("split_maxq", 0)], "sbaij": [],
            "sbaij-phased": [("spmv_kernel", 8)]}[mat]
    ref = O.Problem(NX, NY, NZ, rtol=rtol)
    ref.apply_bc_u(ref.get_displacement(0))
    ref.apply_bc_u(ref.get_displacement(1))
    ref.set_strains(); ref.homogenize(); ref.assembly_res(); ref.assembly_jac()
    if mat.startswith("sbaij"):
        ref.sbaij_mirror()
    rp1, ci1 = ref.csr()
    v1 = ref.A_values()
    x = np.random.default_rng(11).uniform(-1, 1, ref.ndofs)
    y1 = ref.spmv(x)
    absrow = np.add.reduceat(np.abs(v1) * np.abs(x[ci1]), rp1[:-1])
    ref.solve()
    duref = ref.du()
    out = run_group(argv, nr, newton_step(x, opts))
    du = np.zeros(ref.ndofs)
    for o in out:
        assert np.all(np.abs(o["y"] - y1[o["nat"]]) <= 1e-14 * absrow[o["nat"]] + 1e-300)
        du[o["nat"]] = o["du"]
    assert np.linalg.norm(du - duref) <= 1e-8 * np.linalg.norm(duref)


@pytest.mark.parametrize("grid,procs", [((20, 12, 10), (2, 2, 1)), ((12, 10, 14), (2, 2, 2))])
def test_halo_overlap_bitwise(grid, procs):
    """The CG's halo exchange overlapped with the interior p update (sent nodes updated first,
    exchange on the comm stream, rest of p meanwhile) computes exactly what the serialised
    exchange computes: du bitwise equal, same iteration count."""
    NX, NY, NZ = grid
    px, py, pz = procs
    argv = ["-da_grid_x", NX, "-da_grid_y", NY, "-da_grid_z", NZ, "-da_processors_x", px, "-da_processors_y", py,
            "-da_processors_z", pz, "-ksp_rtol", "1e-10"]
    x = np.zeros(3 * NX * NY * NZ)
    on = run_group(argv, px * py * pz, newton_step(x, [("halo_overlap", 1)]))
    off = run_group(argv, px * py * pz, newton_step(x, [("halo_overlap", 0)]))
    for a, b in zip(on, off):
        assert a["its"] == b["its"] and np.array_equal(a["du"], b["du"])


@pytest.mark.parametrize("grid,procs", [((16, 12, 10), (1, 1, 1)), ((20, 12, 10), (2, 2, 1)),
                                        ((12, 10, 14), (2, 2, 2))])
def test_cg_dix_bitwise(grid, procs):
    """Block-indexed storage: the CG's Jacobi scaling from each node's diagonal-block index
    byte with z recomputed from r (option cg_dix, default) computes exactly what the dinv / z
    vectors compute, through the single-rank kernels and the decomposed ones (sent nodes
    first, interior after): du bitwise equal, same iteration count."""
    NX, NY, NZ = grid
    px, py, pz = procs
    argv = ["-da_grid_x", NX, "-da_grid_y", NY, "-da_grid_z", NZ, "-da_processors_x", px, "-da_processors_y", py,
            "-da_processors_z", pz, "-ksp_rtol", "1e-10"]
    x = np.zeros(3 * NX * NY * NZ)
    on = run_group(argv, px * py * pz, newton_step(x, [("cg_dix", 1)]))
    off = run_group(argv, px * py * pz, newton_step(x, [("cg_dix", 0)]))
    for a, b in zip(on, off):
        assert a["info"]["storage"] == 3 and a["info"]["vi_blocks"] > 0
        assert a["its"] == b["its"] and a["reason"] == b["reason"] and np.array_equal(a["du"], b["du"])


@pytest.mark.parametrize("grid,procs", [((20, 12, 10), (2, 2, 1)), ((12, 10, 14), (2, 2, 2))])
def test_cg_pdb_multirank_bitwise(grid, procs):
    """The double-buffered p update (cg_pdb) on decomposed subdomains: sent nodes first, halo of
    the iteration's p buffer overlapping the interior update; du bitwise the single-buffer
    solve's, same iteration count."""
    NX, NY, NZ = grid
    px, py, pz = procs
    argv = ["-da_grid_x", NX, "-da_grid_y", NY, "-da_grid_z", NZ, "-da_processors_x", px, "-da_processors_y", py,
            "-da_processors_z", pz, "-ksp_rtol", "1e-10"]
    x = np.zeros(3 * NX * NY * NZ)
    on = run_group(argv, px * py * pz, newton_step(x, [("cg_pdb", 1), ("cg_par", 0)]))
    par = run_group(argv, px * py * pz, newton_step(x, [("cg_pdb", 1), ("cg_par", 1)]))
    off = run_group(argv, px * py * pz, newton_step(x, [("cg_pdb", 0)]))
    quad = run_group(argv, px * py * pz, newton_step(x, [("cg_pdb", 4), ("cg_par", 1)]))
    for a, b, c, q in zip(on, off, par, quad):
        assert a["its"] == b["its"] and a["reason"] == b["reason"] and np.array_equal(a["du"], b["du"])
        assert c["its"] == b["its"] and c["reason"] == b["reason"] and np.array_equal(c["du"], b["du"])
        assert q["its"] == b["its"] and q["reason"] == b["reason"] and np.array_equal(q["du"], b["du"])


def test_rccl_transport_one_rank():
    """The RCCL transport on one GPU: a one-rank communicator routes every reduction through
    the multi-rank path (k_reduce partial sums, ncclAllReduce on the compute stream,
    k_cg_logic) and the host all-reduces (force, non-linear counts) through ncclAllReduce;
    the result must be bitwise what the single-rank path computes."""
    argv = ["-da_grid_x", 16, "-da_grid_y", 12, "-da_grid_z", 10, "-ksp_rtol", "1e-10"]
    outs = []
    for cid in (None, M.comm_unique_id()):
        with M.Macroc(argv, rank=0, nranks=1, comm_id=cid) as m:
            m.apply_bc_on_u(m.get_displacement(1))
            m.set_strains(); m.homogenize()
            res = m.assembly_res()
            m.assembly_jac()
            its, rn, reason = m.solve_Ax()
            m.update_u()
            m.set_strains(); m.homogenize()
            outs.append((res, its, reason, m.du(), m.calc_force(), m.reduce_nonlinear()))
    (r0, i0, c0, d0, f0, n0), (r1, i1, c1, d1, f1, n1) = outs
    assert (i0, c0, f0, n0) == (i1, c1, f1, n1) and np.array_equal(d0, d1)
    assert abs(r0 - r1) <= 1e-15 * r0


@pytest.mark.parametrize("fma,vi_tx,tile", [(0, 0, (64, 16)), (1, 0, (64, 16)), (1, 256, (256, 4))])
@pytest.mark.parametrize("grid,procs", [((516, 5, 4), (2, 1, 1)), ((260, 9, 10), (1, 1, 2))])
def test_multirank_vi_production_tiles(grid, procs, fma, vi_tx, tile):
    """The value-indexed SpMV's 64x16 (default) and 256x4 tiles on decomposed subdomains (258
    wide: an internal x face at a partial tile's last lane; or a z split with internal z faces at the
    chunk ends): every rank's matrix rows bit-exact with the one-rank oracle, the SpMV too under
    -mat_vi_fma 0 (MATAIJ MatMult, src/init.c:85-93) and within 1e-14 sum|a||x| with the default
    fused multiply-adds; du within the north-star bar at rtol 1e-12."""
    NX, NY, NZ = grid
    px, py, pz = procs
    rtol = 1e-12
    argv = ["-da_grid_x", NX, "-da_grid_y", NY, "-da_grid_z", NZ, "-da_processors_x", px, "-da_processors_y", py,
            "-da_processors_z", pz, "-ksp_rtol", repr(rtol)]
    ref = O.Problem(NX, NY, NZ, rtol=rtol)
    ref.newton_step1()
    v1 = ref.A_values()
    rp1, ci1 = ref.csr()
    x = np.random.default_rng(23).uniform(-1, 1, ref.ndofs)
    y1 = ref.spmv(x)
    absrow = np.add.reduceat(np.abs(v1) * np.abs(x[ci1]), rp1[:-1])
    out = run_group(argv, px * py * pz, newton_step(x, [("vi_stage", 1), ("vi_fma", fma), ("vi_tx", vi_tx)]))
    du = np.zeros(ref.ndofs)
    for o in out:
        info = o["info"]
        assert info["storage"] == 3 and info["vi_blocks"] > 0 and (info["spmv_tx"], info["spmv_ty"]) == tile, info
        if fma:
            assert np.all(np.abs(o["y"] - y1[o["nat"]]) <= 1e-14 * absrow[o["nat"]] + 1e-300)
        else:
            assert np.array_equal(o["y"], y1[o["nat"]])
        for q in range(0, len(o["nat"]), 7):  # rows bit-exact (every 7th: the dump is large)
            row = o["nat"][q]
            assert np.array_equal(np.sort(o["v"][o["rp"][q]:o["rp"][q + 1]].view(np.int64)),
                                  np.sort(v1[rp1[row]:rp1[row + 1]].view(np.int64)))
        du[o["nat"]] = o["du"]
    assert np.linalg.norm(du - ref.du()) <= 1e-10 * np.linalg.norm(ref.du())


@pytest.mark.parametrize("grid,procs", [((516, 5, 4), (2, 1, 1)), ((260, 9, 10), (1, 1, 2)), ((72, 40, 36), (2, 2, 1))])
def test_multirank_st_bitwise(grid, procs):
    """The default-stencil SpMV (vi_st 1: the interior marched with one stencil, the GLOBAL domain's
    faces by their class stencils, the rest listed) on decomposed subdomains: a rank's internal
    faces are interior nodes of the march (their neighbours from the halo exchange), only the
    global faces are classes.  Every rank's y bitwise the per-node index path's (vi_st 0, the
    z-march with index bytes), and the solve within the north-star bar of the one-rank oracle."""
    NX, NY, NZ = grid
    px, py, pz = procs
    rtol = 1e-12
    argv = ["-da_grid_x", NX, "-da_grid_y", NY, "-da_grid_z", NZ, "-da_processors_x", px, "-da_processors_y", py,
            "-da_processors_z", pz, "-ksp_rtol", repr(rtol)]
    ref = O.Problem(NX, NY, NZ, rtol=rtol)
    ref.newton_step1()
    x = np.random.default_rng(29).uniform(-1, 1, ref.ndofs)
    outs = [run_group(argv, px * py * pz, newton_step(x, [("vi_stage", 1), ("vi_st", st), ("vi_st_pair", sp)]))
            for st, sp in ((0, 0), (1, 0), (1, 1))]
    du = np.zeros(ref.ndofs)
    for a, b, c in zip(*outs):
        assert a["info"]["st_listed"] == -1 and b["info"]["st_listed"] >= 0, (a["info"], b["info"])
        assert np.array_equal(a["y"], b["y"])
        assert np.array_equal(a["y"], c["y"])  # k_spmv_sp (x-pair lanes, round 6)
        du[b["nat"]] = b["du"]
    assert np.linalg.norm(du - ref.du()) <= 1e-10 * np.linalg.norm(ref.du())


@pytest.mark.parametrize("grid,procs,stage", [((20, 12, 10), (2, 2, 1), 0), ((130, 9, 12), (2, 1, 1), 1),
                                              ((24, 16, 14), (2, 2, 2), 0)])
def test_multirank_vi_exception_nodes(grid, procs, stage):
    """J2 law with a few plastic Gauss points on decomposed subdomains: each rank's nodes that
    touch a non-elastic element are exception nodes (their own 27 blocks), the rest index the
    rank's dictionary.  Every rank's rows bit-exact with the one-rank oracle, the SpMV too
    (-mat_vi_fma 0), du within the north-star bar."""
    from test_gpu_parity import plastic_state

    NX, NY, NZ = grid
    px, py, pz = procs
    rtol = 1e-10
    P, u = plastic_state(NX, NY, NZ, rtol=rtol)
    v1 = P.A_values()
    rp1, ci1 = P.csr()
    x = np.random.default_rng(29).uniform(-1, 1, P.ndofs)
    y1 = P.spmv(x)
    P.solve()
    argv = ["-da_grid_x", NX, "-da_grid_y", NY, "-da_grid_z", NZ, "-da_processors_x", px, "-da_processors_y", py,
            "-da_processors_z", pz, "-ksp_rtol", repr(rtol), "-dt", 0.01, "-mat_law", "plastic"]

    def fn(m):
        m.set_option("vi_stage", stage)
        m.set_option("vi_fma", 0)
        petsc, nat = m.owned_dofs()
        m.set_u(u[nat])
        m.set_strains(); m.homogenize(); m.assembly_res(); m.assembly_jac()
        rp, ci, v = m.dump_csr()
        y = m.spmv(x[nat])
        its, rn, reason = m.solve_Ax()
        return dict(nat=nat, rp=rp, v=v, y=y, du=m.du(), its=its, info=m.get_info())

    out = run_group(argv, px * py * pz, fn)
    du = np.zeros(P.ndofs)
    assert sum(o["info"]["vi_exc_nodes"] for o in out) > 0
    for o in out:
        assert o["info"]["storage"] == 3, o["info"]
        assert np.array_equal(o["y"], y1[o["nat"]])
        for q in range(len(o["nat"])):
            row = o["nat"][q]
            assert np.array_equal(np.sort(o["v"][o["rp"][q]:o["rp"][q + 1]].view(np.int64)),
                                  np.sort(v1[rp1[row]:rp1[row + 1]].view(np.int64)))
        du[o["nat"]] = o["du"]
    assert np.linalg.norm(du - P.du()) <= 50 * rtol * np.linalg.norm(P.du())


def test_back_to_back_halos():
    """Halo exchanges with no all-reduce between them (set_strains twice, then SpMVs back to
    back): each exchange's device copies into a rank's receive buffer are ordered after that
    rank's previous unpack, so every product is the one-rank oracle's, bit for bit."""
    NX, NY, NZ = 20, 12, 10
    argv = ["-da_grid_x", NX, "-da_grid_y", NY, "-da_grid_z", NZ, "-da_processors_x", 2, "-da_processors_y", 2,
            "-da_processors_z", 2]
    ref = O.Problem(NX, NY, NZ)
    ref.apply_bc_u(ref.get_displacement(1))
    ref.set_strains(); ref.homogenize(); ref.assembly_res(); ref.assembly_jac()
    rng = np.random.default_rng(31)
    xs = [rng.uniform(-1, 1, ref.ndofs) for _ in range(4)]
    ys = [ref.spmv(x) for x in xs]

    def fn(m):
        m.apply_bc_on_u(m.get_displacement(1))
        m.set_strains()
        e1 = m.strain()
        m.set_strains()
        e2 = m.strain()
        m.homogenize()
        m.assembly_res()
        m.assembly_jac()
        _, nat = m.owned_dofs()
        out = [m.spmv(x[nat]) for x in xs]
        return dict(nat=nat, same=np.array_equal(e1, e2), b=m.b(), y=out)

    out = run_group(argv, 8, fn)
    b = np.zeros(ref.ndofs)
    for o in out:
        assert o["same"]
        b[o["nat"]] = o["b"]
        for y, yr in zip(o["y"], ys):
            assert np.array_equal(y, yr[o["nat"]])
    assert np.array_equal(b, ref.b())


def test_group_member_withheld_or_mismatched_fails(monkeypatch):
    """VERDICT r04 items 1 and 5 on the device path: (a) a group whose second member never
    initialises fails rank 0's mcx_init_local after MCX_COMM_TIMEOUT instead of hanging; (b) a
    member that finalizes while the other exchanges a halo makes both calls fail with the two
    collectives named, and neither reads the other's freed buffers (the process survives and a
    fresh group works afterwards)."""
    import time
    monkeypatch.setenv("MCX_COMM_TIMEOUT", "2")
    argv = ["-da_grid_x", 12, "-da_grid_y", 10, "-da_grid_z", 8, "-da_processors_x", 2]
    g = M.LocalGroup(2)
    t0 = time.time()
    with pytest.raises(M.MacrocError, match="waited 2 s in mcx_init_local"):
        M.Macroc(argv, rank=0, nranks=2, group=g)
    assert time.time() - t0 < 30
    g.destroy()

    g = M.LocalGroup(2)
    errs = [None, None]

    def worker(r):
        try:
            m = M.Macroc(argv, rank=r, nranks=2, group=g)
            try:
                if r == 0:
                    m.apply_bc_on_u(m.get_displacement(1))
                    m.set_strains()  # halo exchange of u: rank 1 is finalizing instead
            finally:
                m.finish()
        except M.MacrocError as e:
            errs[r] = str(e)

    ts = [threading.Thread(target=worker, args=(r,), daemon=True) for r in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(60)
    assert not any(t.is_alive() for t in ts)
    g.destroy()
    assert errs[0] and errs[1], errs
    assert all("mismatched collectives" in e or "in-process group" in e for e in errs), errs
    assert any("mcx_finalize" in e and "halo exchange" in e for e in errs), errs
    monkeypatch.delenv("MCX_COMM_TIMEOUT")
    out = run_group(argv, 2, lambda m: (m.apply_bc_on_u(m.get_displacement(1)), m.set_strains(), m.homogenize(),
                                        m.assembly_res())[-1])  # the library still works
    assert out[0] == out[1] > 0
