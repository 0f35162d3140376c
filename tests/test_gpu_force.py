"""Per-time-step post-processing of src/main.c:86-97 on the GPU against the oracle:
reaction force (calc_force, src/forces.c:25-166), non-linear Gauss-point counts and
f_trial_max (src/util.c:69-102), and the C driver's info.dat / gauss_evolution.dat rows
against the oracle's time loop.

Bars: with the same displacement field, the elastic stresses are bit-exact, so the force is
bit-exact too (same element set, loop order and rank order).  The plastic law agrees to
sqrt/division rounding (1e-12).  Driver rows: the integer and input columns match exactly;
the force matches to the solver tolerance.
"""
import os
import subprocess
import threading

import numpy as np
import pytest

import macroc_amd as M
from oracle import oracle as O

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DRIVER = os.path.join(ROOT, "macroc_amd", "driver", "macroc_amd")

# (NX, NY, NZ, bc_type, law, dt): 41x5x41 puts four top-layer elements inside the load circle
CASES = [(41, 5, 41, 1, 0, 0.001), (41, 5, 41, 1, 1, 0.3), (9, 6, 7, 0, 0, 0.001), (9, 6, 7, 0, 1, 0.05)]


def argv_for(NX, NY, NZ, bc, law, dt, extra=()):
    return ["-da_grid_x", NX, "-da_grid_y", NY, "-da_grid_z", NZ, "-bc_type", bc, "-dt", dt,
            "-mat_law", "plastic" if law else "elastic", "-ksp_rtol", "1e-10", *extra]


def solved_u(NX, NY, NZ, bc, law, dt):
    """u after time step 1's first Newton update, from the oracle (one rank: natural order)."""
    P = O.Problem(NX, NY, NZ, rtol=1e-10, bc_type=bc, law=law, dt=dt)
    P.apply_bc_u(P.get_displacement(0))
    P.apply_bc_u(P.get_displacement(1))
    P.set_strains(); P.homogenize(); P.assembly_res(); P.assembly_jac(); P.solve(); P.update_u()
    u = P.u()
    P.close()
    return u


@pytest.mark.parametrize("NX,NY,NZ,bc,law,dt", CASES)
def test_force_single_rank(NX, NY, NZ, bc, law, dt):
    u = solved_u(NX, NY, NZ, bc, law, dt)
    P = O.Problem(NX, NY, NZ, rtol=1e-10, bc_type=bc, law=law, dt=dt)
    P.set_u(u)
    P.set_strains()
    P.homogenize()
    with M.Macroc(argv_for(NX, NY, NZ, bc, law, dt)) as m:
        m.set_u(u)
        m.set_strains()
        m.homogenize()
        f = m.calc_force()
        ref = P.calc_force()
        assert ref != 0.0
        nl, nt, fm = m.reduce_nonlinear()
        on, ofm = P.nonlinear_gps()
        if law == 0:
            assert np.array_equal(m.stress(), P.stress())
            assert f == ref
            assert (nl, nt, fm) == (0, 0, 0.0) and (on, ofm) == (0, 0.0)
        else:
            assert abs(f - ref) <= 1e-12 * abs(ref)
            assert nl == nt == on and on > 0
            assert abs(fm - ofm) <= 1e-12 * abs(ofm)


def run_group(argv, nranks, fn):
    g = M.LocalGroup(nranks)
    out, errors = [None] * nranks, []

    def worker(r):
        try:
            m = M.Macroc(argv, rank=r, nranks=nranks, group=g)
            try:
                out[r] = fn(m)
            finally:
                m.finish()
        except Exception as e:  # surfaced below
            errors.append((r, e))

    ts = [threading.Thread(target=worker, args=(r,), daemon=True) for r in range(nranks)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(300)
    assert not any(t.is_alive() for t in ts), errors
    assert not errors, errors
    g.destroy()
    return out


@pytest.mark.parametrize("NX,NY,NZ,bc,nranks", [(41, 5, 41, 1, 2), (41, 5, 41, 1, 4), (9, 6, 7, 0, 2),
                                                (9, 6, 7, 0, 4)])
def test_force_multirank(NX, NY, NZ, bc, nranks):
    """Per-rank partials over each rank's own PETSc element set, summed in rank order: the
    in-process group reproduces the oracle's emulated ranks bit for bit."""
    u_nat = solved_u(NX, NY, NZ, bc, 0, 0.001)
    P = O.Problem(NX, NY, NZ, rtol=1e-10, bc_type=bc, nranks=nranks)
    dm = P.dof_map()
    u_petsc = np.empty_like(u_nat)
    u_petsc[dm] = u_nat
    P.set_u(u_petsc)
    P.set_strains()
    P.homogenize()
    ref = P.calc_force()
    assert ref != 0.0

    def fn(m):
        petsc, nat = m.owned_dofs()
        m.set_u(u_nat[nat])
        m.set_strains()
        m.homogenize()
        return m.calc_force(), m.reduce_nonlinear()

    out = run_group(argv_for(NX, NY, NZ, bc, 0, 0.001), nranks, fn)
    for f, (nl, nt, fm) in out:
        assert f == ref
        assert (nt, fm) == (0, 0.0)


def test_force_circle_quirk_two_ranks_in_y():
    """src/forces.c:130-133 tests the ghost y-corner plus the owned ny: with two ranks in y no
    rank qualifies and the reference reports 0 — kept."""
    NX, NY, NZ = 41, 6, 41
    u_nat = solved_u(NX, NY, NZ, 1, 0, 0.001)
    P = O.Problem(NX, NY, NZ, rtol=1e-10, nranks=2, m=1, n=2, p=1)
    dm = P.dof_map()
    u_petsc = np.empty_like(u_nat)
    u_petsc[dm] = u_nat
    P.set_u(u_petsc)
    P.set_strains()
    P.homogenize()
    assert P.calc_force() == 0.0

    def fn(m):
        petsc, nat = m.owned_dofs()
        m.set_u(u_nat[nat])
        m.set_strains()
        m.homogenize()
        return m.calc_force()

    argv = argv_for(NX, NY, NZ, 1, 0, 0.001, ["-da_processors_x", 1, "-da_processors_y", 2, "-da_processors_z", 1])
    assert run_group(argv, 2, fn) == [0.0, 0.0]


@pytest.mark.parametrize("law,dt,ts", [(0, 0.001, 3), (1, 0.3, 2)])
def test_driver_info_dat(tmp_path, law, dt, ts):
    """The C driver's info.dat / gauss_evolution.dat rows against the oracle's time loop."""
    NX, NY, NZ = 41, 5, 41
    args = [str(v) for v in argv_for(NX, NY, NZ, 1, law, dt, ["-ts", ts])]
    r = subprocess.run([DRIVER, *args], cwd=tmp_path, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "Non-Linear Gauss points" in r.stdout and "F_trial_max" in r.stdout
    P = O.Problem(NX, NY, NZ, rtol=1e-10, law=law, dt=dt, ts=ts)
    P.run(None, str(tmp_path / "o_info.dat"), str(tmp_path / "o_gauss.dat"))
    g_rows = [l.split("\t") for l in (tmp_path / "info.dat").read_text().splitlines()]
    o_rows = [l.split("\t") for l in (tmp_path / "o_info.dat").read_text().splitlines()]
    assert len(g_rows) == len(o_rows) == ts
    for g, o in zip(g_rows, o_rows):
        assert g[:3] == o[:3]  # time_s, time, U: the same formatted inputs
        assert g[5] == o[5]  # non-linear GP count
        fg, fo = float(g[3]), float(o[3])
        assert abs(fg - fo) <= 1e-6 * max(abs(fo), 1e-300)  # through the solve: solver tolerance
        assert abs(float(g[4]) - float(o[4])) <= 1e-6 * max(abs(float(o[4])), 1e-300)
    assert float(g_rows[-1][3]) != 0.0
    assert (tmp_path / "gauss_evolution.dat").read_text() == (tmp_path / "o_gauss.dat").read_text()
