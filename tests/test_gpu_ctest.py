"""The reference's own test suite on the GPU path: the ten ctest runs of tests/CMakeLists.txt:21-32
(`mpirun -np {1,2,3,4} macroc -da_grid_x 5 -da_grid_y 2 -da_grid_z 2 -ts 5`, `-np 8` on 5x3x{3,4,5},
serial 3^3, 4^3, 5x2x2, all `-ts 5`).  The reference passes on exit status 0 alone; here every
rank grid runs through the in-process transport (one thread per rank) and each time step's Newton
log — |RES| per iteration, KSP iterations, non-linear GP count, reaction force, info.dat row — is
compared with the oracle running the same rank grid (emulated ranks).  Only 4^3 has a node in the
load circle, so it is the one grid whose time steps solve; the others pin the zero-load
plumbing (|RES| = 0, no Jacobian, no KSP)."""
import threading

import numpy as np
import pytest

import macroc_amd as M
from oracle import oracle as O

pytestmark = pytest.mark.gpu

CTEST = [(1, (5, 2, 2)), (2, (5, 2, 2)), (3, (5, 2, 2)), (4, (5, 2, 2)), (8, (5, 3, 3)), (8, (5, 3, 4)),
         (8, (5, 3, 5)), (1, (3, 3, 3)), (1, (4, 4, 4)), (1, (5, 2, 2))]


def parse_log(text):
    """per time step: list of |RES| values, list of KSP its, non-linear count, f_trial_max line"""
    steps, cur = [], None
    for ln in text.splitlines():
        if ln.startswith("Time Step = "):
            cur = {"res": [], "its": [], "nl": None}
            steps.append(cur)
        elif ln.startswith("|RES| = "):
            cur["res"].append(float(ln.split("=")[1]))
        elif ln.startswith("KSP : "):
            cur["its"].append(int(ln.split("Its =")[1]))
        elif ln.startswith("Non-Linear Gauss points : "):
            cur["nl"] = int(ln.split(":")[1])
    return steps


@pytest.mark.parametrize("nranks,grid", CTEST, ids=[f"np{n}-{g[0]}x{g[1]}x{g[2]}" for n, g in CTEST])
def test_reference_ctest_run(nranks, grid, tmp_path):
    ts = 5
    P = O.Problem(*grid, nranks=nranks, ts=ts)
    log, info = tmp_path / "oracle.log", tmp_path / "info.dat"
    P.run(str(log), str(info))
    ref = parse_log(log.read_text())
    ref_info = [ln.split("\t") for ln in info.read_text().splitlines()]
    P.close()
    argv = ["-da_grid_x", grid[0], "-da_grid_y", grid[1], "-da_grid_z", grid[2], "-ts", ts]
    g = M.LocalGroup(nranks) if nranks > 1 else None
    out, errs = [None] * nranks, []

    def worker(r):
        try:
            kw = dict(rank=r, nranks=nranks, group=g) if g else {}
            with M.Macroc(argv, **kw) as m:
                steps = []
                for t in range(ts):
                    st = m.time_step(t)
                    nl_loc, nl, ftm = m.reduce_nonlinear()
                    force = m.calc_force()
                    steps.append(dict(st, nl=nl, force=force, ftm=ftm, U=m.get_displacement(t)))
                out[r] = steps
        except Exception as e:  # surfaced below
            errs.append((r, e))

    ths = [threading.Thread(target=worker, args=(r,)) for r in range(nranks)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(300)
    if g:
        g.destroy()
    assert not errs, errs
    for r in range(1, nranks):  # every rank sees the same collective results
        for a, b in zip(out[0], out[r]):
            assert a["res"] == b["res"] and a["ksp_its"] == b["ksp_its"] and a["force"] == b["force"]
    assert len(ref) == ts
    for t, (st, o) in enumerate(zip(out[0], ref)):
        assert len(st["res"]) == len(o["res"]), (t, st, o)
        np.testing.assert_allclose(st["res"], o["res"], rtol=1e-6, atol=0)  # the log prints %e
        assert len(st["ksp_its"]) == len(o["its"]) and all(abs(a - b) <= 1 for a, b in zip(st["ksp_its"], o["its"]))
        assert st["nl"] == o["nl"]
        row = ref_info[t]
        assert int(row[0]) == t and float(row[2]) == float(f"{st['U']:e}")
        assert abs(st["force"] - float(row[3])) <= 1e-6 * max(abs(float(row[3])), 1e-300) + 1e-300
    if grid == (4, 4, 4):
        assert any(st["ksp_its"] for st in out[0]), "4^3 has a loaded node: its steps must solve"
    else:
        assert all(st["res"] == [0.0] and not st["ksp_its"] for st in out[0])
