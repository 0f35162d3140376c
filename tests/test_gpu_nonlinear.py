"""Non-linear Newton (BASELINE config 5's path): J2-plastic Gauss-point law behind the callback,
history committed by update_vars (src/main.c:83), several Newton iterations per time step and
several time steps — GPU against the oracle, which runs the same law.  Parity vs MicroPP itself
is unpinned (MicroPP is not available); GPU vs oracle: strains/stresses/tangents to 1e-12
(sqrt/division rounding), Newton iteration counts equal, u to 1e-9."""
import numpy as np
import pytest

import macroc_amd as M
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def newton(step, res_fn, rel=1e-4, abs_tol=0.1, max_its=5):
    norms = []
    for it in range(max_its):
        n = res_fn()
        norms.append(n)
        if n < abs_tol or n < norms[0] * rel:
            break
        step()
    return norms


@pytest.mark.parametrize("mat", ["aij", "sbaij"])
def test_plastic_time_steps(mat):
    """Time step 1 (zero history): every Newton iterate matches the oracle.  Later steps start
    with Gauss points exactly on the yield surface (f_trial = 0 up to rounding), where the
    elastic / elastoplastic tangent choice is decided by the last bit on either side, so only
    tightly converged states are compared there."""
    NX, NY, NZ, dt, rtol = 12, 10, 12, 0.01, 1e-12
    P = O.Problem(NX, NY, NZ, law=1, dt=dt, rtol=rtol)
    argv = ["-da_grid_x", NX, "-da_grid_y", NY, "-da_grid_z", NZ, "-dt", dt, "-ksp_rtol", repr(rtol),
            "-mat_law", "plastic", "-dm_mat_type", mat]

    def o_newton_step():
        P.assembly_jac()
        if mat == "sbaij":
            P.sbaij_mirror()
        P.solve()
        P.update_u()

    with M.Macroc(argv) as m:
        for ts in range(3):
            m.apply_bc_on_u(m.get_displacement(ts))
            P.apply_bc_u(P.get_displacement(ts))
            strict = ts <= 1
            g_norms, o_norms = [], []
            for it in range(12):
                m.set_strains(); m.homogenize(); n = m.assembly_res()
                P.set_strains(); P.homogenize(); P.assembly_res(); on = P.norm_b()
                g_norms.append(n)
                o_norms.append(on)
                if strict:
                    np.testing.assert_allclose(m.strain(), P.strain(), rtol=1e-9, atol=1e-15)
                    s_ref = P.stress()
                    np.testing.assert_allclose(m.stress(), s_ref, rtol=0, atol=1e-9 * np.abs(s_ref).max() + 1e-300)
                    assert abs(n - on) <= 1e-7 * max(on, 1.0)
                tol = 1e-4 if strict else 1e-10
                g_done = n < 0.1 or n < g_norms[0] * tol
                o_done = on < 0.1 or on < o_norms[0] * tol
                if strict:
                    assert g_done == o_done
                if not g_done:
                    m.assembly_jac(); m.solve_Ax(); m.update_u()
                if not o_done:
                    o_newton_step()
                if g_done and o_done:
                    break
            gn, gf = m.nonlinear_stats()
            on_, of = P.nonlinear_gps()
            if strict:
                assert gn == on_
            else:
                assert abs(gn - on_) <= max(2, on_ // 20)
            m.update_vars()
            P.update_vars()
            u, uref = m.u(), P.u()
            assert np.linalg.norm(u - uref) <= (1e-9 if strict else 1e-7) * np.linalg.norm(uref)
            if ts == 1:
                assert gn > 0, "the load must drive Gauss points plastic"
                assert len(g_norms) >= 3, "plasticity must need more than one Newton iteration"
