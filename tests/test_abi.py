"""C-ABI checks that need no GPU: the library loads, exports every symbol include/*.h declares,
parses the reference's flag surface and fails loudly (no CPU fallback) without a device."""
import glob
import os
import re
import subprocess
import sys

import numpy as np
import pytest

import macroc_amd as M

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    syms = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        txt = open(h).read()
        syms |= set(re.findall(r"\b(mcx_[a-z_0-9]+)\s*\(", txt))
    return syms


def test_library_exports_header():
    out = subprocess.run(["nm", "-D", "--defined-only", M.LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r" T (mcx_[a-z_0-9]+)", out))
    declared = header_symbols()
    assert declared, "no symbols parsed from include/"
    assert declared <= exported, declared - exported
    assert set(M.EXPORTS) == declared
    for s in declared:
        getattr(M.lib(), s)


def test_parse_args_reference_flags():
    o = M.parse_args(["-da_grid_x", "64", "-da_grid_y", "32", "-da_grid_z", "16", "-da_processors_x", "2",
                      "-ts", "2", "-ksp_rtol", "1e-8", "-micro_mat_1", "2e7,0.3,1e4,1e7", "-newton_max_its", "3",
                      "-bc_type", "0", "-ksp_type", "cg", "-pc_type", "jacobi"])
    assert (o.NX, o.NY, o.NZ, o.px, o.ts, o.newton_max_its, o.bc_type) == (64, 32, 16, 2, 2, 3, 0)
    assert o.ksp_rtol == 1e-8 and list(o.micro_mat_1) == [2e7, 0.3, 1e4, 1e7]
    d = M.parse_args([])
    assert (d.NX, d.NY, d.NZ, d.ts, d.lx, d.ly, d.lz) == (40, 3, 40, 1, 50.0, 1.0, 50.0)
    assert (d.ksp_rtol, d.ksp_abstol, d.ksp_dtol, d.ksp_max_it) == (1e-5, 1e-50, 1e4, 10000)
    with pytest.raises(M.MacrocError):
        M.parse_args(["-ksp_type", "gmres"])


def test_plan_matches_oracle_decomposition():
    from oracle import oracle as O
    for grid, nr in (((5, 2, 2), 3), ((5, 3, 4), 8), ((10, 8, 8), 2), ((17, 9, 5), 6)):
        argv = ["-da_grid_x", grid[0], "-da_grid_y", grid[1], "-da_grid_z", grid[2]]
        P = O.Problem(*grid, nranks=nr)
        dm = P.dof_map()
        petsc = np.zeros(3 * np.prod(grid), dtype=np.int64)
        for r in range(nr):
            pl = M.plan(argv, r, nr)
            c = P.corners(r)
            assert (pl["xs"], pl["ys"], pl["zs"], pl["nx"], pl["ny"], pl["nz"]) == c[:6]
            assert (pl["Xs"], pl["Ys"], pl["Zs"], pl["Nx"], pl["Ny"], pl["Nz"]) == c[6:]
            assert (pl["px"], pl["py"], pl["pz"]) == P.decomp()
            assert pl["dof_offset"] == P.dof_offset(r)
            assert pl["nelem_local"] == len(P.elements(r))
            rp, _ = P.csr()
            off = pl["dof_offset"]
            assert pl["nnz_local"] == rp[off + pl["ndofs_local"]] - rp[off]
            # rebuild the global PETSc numbering from the plan alone
            i, j, k = np.meshgrid(np.arange(pl["nx"]), np.arange(pl["ny"]), np.arange(pl["nz"]), indexing="ij")
            loc = (i + j * pl["nx"] + k * pl["nx"] * pl["ny"]).ravel()
            nat = ((pl["xs"] + i) + (pl["ys"] + j) * grid[0] + (pl["zs"] + k) * grid[0] * grid[1]).ravel()
            for d in range(3):
                petsc[3 * nat + d] = off + 3 * loc + d
        assert np.array_equal(petsc, dm)
        P.close()


def test_halo_plan_is_symmetric():
    argv = ["-da_grid_x", "9", "-da_grid_y", "7", "-da_grid_z", "6"]
    nr = 8
    plans = [dict((q, (s, rv)) for q, s, rv in M.plan_halo(argv, r, nr)) for r in range(nr)]
    for r in range(nr):
        for q, (s, rv) in plans[r].items():
            # what r sends to q is exactly what q receives from r, in the same order
            assert np.array_equal(plans[q][r][1], s)


def test_init_without_gpu_fails_loudly():
    if os.path.exists("/dev/kfd"):
        pytest.skip("a GPU is visible")
    with pytest.raises(M.MacrocError, match="device"):
        M.Macroc(["-da_grid_x", "4", "-da_grid_y", "4", "-da_grid_z", "2"])


def test_no_exception_crosses_the_abi():
    """every extern "C" entry is a function-try-block.  MCX_TEST_THROW=<entries>
    (read once when the library loads: ADVICE r05) makes those entries throw std::bad_alloc at their
    start (the failure of an absurd host allocation); the caller gets code 90 and the message
    instead of std::terminate killing the process.  Run in a child process that loads the library
    with the variable set; this process (loaded without it) is unaffected."""
    fns = ["mcx_plan", "mcx_parse_args", "mcx_init", "mcx_local_group_create"]
    code = f"""
import ctypes as C, sys
sys.path.insert(0, {ROOT!r})
import macroc_amd as M
L = M.lib()
o = M.Opts(); L.mcx_default_opts(C.byref(o))
inf = M.Info()
calls = {{"mcx_plan": lambda: L.mcx_plan(C.byref(o), 0, 1, C.byref(inf)),
          "mcx_parse_args": lambda: L.mcx_parse_args(C.byref(o), 0, None),
          "mcx_init": lambda: L.mcx_init(C.byref(o), 0, 1, None, C.byref(C.c_void_p())),
          "mcx_local_group_create": lambda: L.mcx_local_group_create(2, 0, C.byref(C.c_void_p()))}}
for fn, call in calls.items():
    rc = call()
    msg = L.mcx_last_error().decode()
    assert rc == 90 and fn in msg and "bad_alloc" in msg, (fn, rc, msg)
assert L.mcx_get_info(None, C.byref(inf)) != 90  # an entry not listed does not throw
print("ok")
"""
    env = dict(os.environ, MCX_TEST_THROW=",".join(fns))
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0 and out.stdout.strip().endswith("ok"), out.stdout + out.stderr
    L = M.lib()
    o = M.parse_args(["-da_grid_x", 8, "-da_grid_y", 8, "-da_grid_z", 8])
    inf = M.Info()
    assert L.mcx_plan(M.C.byref(o), 0, 1, M.C.byref(inf)) == 0 and inf.nx == 8


def test_abi_version_and_comm_info_without_context():
    """the struct-carrying entries changed size in round 5; the library reports its ABI
    revision (the mirror refuses another), and mcx_comm_info rejects a NULL context."""
    L = M.lib()
    assert L.mcx_abi_version() == M.ABI_VERSION == 3
    assert "abi 3" in L.mcx_version().decode()
    assert L.mcx_comm_info(None, None, None, None) != 0


def test_local_group_withheld_member_fails_within_deadline(monkeypatch):
    """VERDICT r04 item 5 (in-process transport): a member that never reaches the collective makes
    the others' crossing fail after MCX_COMM_TIMEOUT seconds instead of hanging; the broken group
    fails every later crossing at once.  The same barrier guards every collective entry point
    (halo exchange, all-reduce, init, finalize)."""
    import threading
    import time
    monkeypatch.setenv("MCX_COMM_TIMEOUT", "1")
    g = M.LocalGroup(2)
    try:
        ok = []
        ts = [threading.Thread(target=lambda r=r: (g.barrier(r), ok.append(r))) for r in range(2)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(10)
        assert sorted(ok) == [0, 1]  # both members: the crossing completes
        t0 = time.time()
        with pytest.raises(M.MacrocError, match=r"rank 0 waited 1 s in mcx_local_group_barrier: 1 of 2"):
            g.barrier(0)  # rank 1 withheld
        assert time.time() - t0 < 5
        t0 = time.time()
        with pytest.raises(M.MacrocError, match="in-process group"):
            g.barrier(1)
        assert time.time() - t0 < 0.5
    finally:
        g.destroy()
