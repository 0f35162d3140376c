"""Interleaved A/B of whole CG solves for one option (same matrix, same process): assembles the
time-step-1 Newton system once, then alternates solves with option values.
    python tools/cg_ab.py --grid 256 --option cg_nt --values 0,1 --rounds 3"""
import argparse
import os
import statistics
import sys

import torch  # noqa: F401  (shared HIP runtime)

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import macroc_amd as M  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--grid", type=int, default=256)
ap.add_argument("--mat", default="aij")
ap.add_argument("--option", default="cg_nt")
ap.add_argument("--values", default="0,1")
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--rtol", default="1e-8")
ap.add_argument("--set", default="", help="options set before the A/B, 'name=value,...'")
a = ap.parse_args()
G = a.grid
m = M.Macroc(["-da_grid_x", G, "-da_grid_y", G, "-da_grid_z", G, "-ksp_rtol", a.rtol, "-dm_mat_type", a.mat])
m.set_timing(True)
m.apply_bc_on_u(m.get_displacement(1))
m.set_strains(); m.homogenize(); m.assembly_res(); m.assembly_jac()
for kv in [kv for kv in a.set.split(",") if kv]:
    m.set_option(kv.split("=")[0], float(kv.split("=")[1]))
vals = [float(v) for v in a.values.split(",")]
res = {v: [] for v in vals}
dus = {}
spmv = {v: [] for v in vals}
for r in range(a.rounds):
    for v in vals:
        m.set_option(a.option, v)
        its, rn, reason = m.solve_Ax()
        t = m.timing()
        res[v].append(t["solve_ms"] / its)
        dus.setdefault(v, (its, m.du()))
        spmv[v].append(t["spmv_ms_total"] / max(t["spmv_launches"], 1))
        print(f"round {r} {a.option}={v:g}: its={its} ms/iter={t['solve_ms'] / its:.4f}", flush=True)
import numpy as np  # noqa: E402
for v in vals:
    same = dus[v][0] == dus[vals[0]][0] and np.array_equal(dus[v][1], dus[vals[0]][1])
    print(f"{a.mat} {G}^3 {a.option}={v:g}: median ms/iter {statistics.median(res[v]):.4f}  its {dus[v][0]}  "
          f"spmv kernel {statistics.median(spmv[v]):.4f} ms  "
          f"du bitwise equal to {a.option}={vals[0]:g}: {same}")
m.finish()
