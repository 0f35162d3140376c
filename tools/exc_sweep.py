"""Crossover of the AIJ storages for a per-Gauss-point-tangent law (J2) as the plastic share grows
(VERDICT r03 item 4): value-indexed with exception nodes vs AIJ-split vs SBAIJ at a seeded share of
exception nodes.  The displacement u_y = -gamma * max(0, x_f - x) shears the slab x < x_f beyond
yield (every Gauss point there on the plastic branch, a tangent of its own), the rest stays
elastic; exception nodes = the nodes touching a plastic element, about x_f / lx of the body.
Per storage: the Jacobian assembly and a fixed-length CG (-ksp_max_it, no convergence test that
can stop it) timed by the library's HIP events; ms per CG iteration, per SpMV and per Jacobian.
Diagnosis tool (not a test); run on the GPU box:

    python tools/exc_sweep.py --grid 128 --fracs 0.05,0.1,0.25,0.5,0.75,1.0
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import macroc_amd as M  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--grid", type=int, default=128)
ap.add_argument("--fracs", default="0.05,0.1,0.25,0.5,0.75,1.0")
ap.add_argument("--storages", default="aij-vi,aij-split,sbaij")
ap.add_argument("--its", type=int, default=200, help="CG iterations timed per storage")
ap.add_argument("--gamma", type=float, default=1e-2, help="shear strain of the plastic slab (yield ~1e-3)")
a = ap.parse_args()
G = a.grid
ARGS = {"aij-vi": ["-dm_mat_type", "aij"], "aij-vi-exck": ["-dm_mat_type", "aij"], "aij-vi-pass": ["-dm_mat_type", "aij"],
        "aij-vi-l1": ["-dm_mat_type", "aij"], "aij-vi-l16": ["-dm_mat_type", "aij"],
        "aij-split": ["-dm_mat_type", "aij"], "sbaij": ["-dm_mat_type", "sbaij"]}
# aij-vi: the default (default-stencil kernel, exception rows among its listed rows); aij-vi-exck: vi_st 0 with
# the exception kernel; aij-vi-pass: vi_st 0 with round 4's in-tile exception pass (vi_exc_kernel 0);
# aij-vi-l1 / aij-vi-l16: as aij-vi with the listed rows one thread per node (vi_st_l16 0, round 5's form) /
# 16 lanes per node (vi_st_l16 1); aij-vi: the rule (vi_st_l16 -1)
lx = 50.0
dx = lx / (G - 1)
i = np.arange(G)


def field(frac):
    xf = frac * lx
    uy = -a.gamma * np.maximum(0.0, xf - i * dx)  # per x index
    u = np.zeros((G, G, G, 3))  # [k][j][i][d], natural order on one rank
    u[:, :, :, 1] = uy[None, None, :]
    return u.ravel()


out = []
for frac in [float(f) for f in a.fracs.split(",")]:
    u = field(frac)
    for st in a.storages.split(","):
        m = M.Macroc(["-da_grid_x", G, "-da_grid_y", G, "-da_grid_z", G, "-mat_law", "plastic", "-ksp_rtol", "1e-300",
                      "-ksp_max_it", a.its] + ARGS[st])
        try:
            if st.startswith("aij-vi"):
                m.set_option("vi_exc_max", 1000)
                m.set_option("vi_exc_kernel", 0 if st == "aij-vi-pass" else 1)
                m.set_option("vi_st", 1 if st in ("aij-vi", "aij-vi-l1", "aij-vi-st") else 0)
                m.set_option("vi_st_l16", 0 if st == "aij-vi-l1" else (1 if st == "aij-vi-l16" else -1))
            elif st == "aij-split":
                m.set_option("vi_exc_max", 0)
            m.set_u(u)
            m.set_strains(); m.homogenize(); m.assembly_res()
            m.assembly_jac()
            m.solve_Ax()  # warm
            m.set_timing(True)
            t0 = time.perf_counter()
            m.assembly_jac()
            its, rn, reason = m.solve_Ax()
            m.synchronize()
            wall = time.perf_counter() - t0
            tm = m.timing()
            info = m.get_info()
            rec = {"frac": frac, "storage": st, "storage_id": info["storage"], "vi_exc_nodes": info["vi_exc_nodes"],
                   "exc_share": info["vi_exc_nodes"] / G ** 3, "nonlinear_gps": m.nonlinear_stats()[0],
                   "its": its, "reason": reason, "ms_per_cg_iter": tm["solve_ms"] / max(its, 1),
                   "spmv_avg_ms": tm["spmv_ms_total"] / max(tm["spmv_launches"], 1),
                   "jacobian_ms": tm["jacobian_ms"], "wall_s": wall, "device_gb": info["device_bytes"] / 1e9}
        finally:
            m.finish()
        out.append(rec)
        print(json.dumps(rec), flush=True)
print("summary (ms per CG iteration):")
for frac in sorted({r["frac"] for r in out}):
    row = {r["storage"]: r for r in out if r["frac"] == frac}
    print(f"  frac {frac:5.2f}: " + "  ".join(
        f"{k} {v['ms_per_cg_iter']:.4f} (storage {v['storage_id']}, exc {v['exc_share']:.3f})" for k, v in row.items()))
