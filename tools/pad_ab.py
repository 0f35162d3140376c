"""Interleaved A/B of the padded-vector layout (MCX_PAD_ALIGN at context creation: 0 = row pitch
nx + 2, round 4; 1 = pitch rounded to 16 nodes with every row's first owned node on a 128-B line;
2 = the same pitch with the ghost column on the line), one context per layout in one process, the
same Newton system, whole CG solves alternated; du must be bitwise equal across layouts:
    python tools/pad_ab.py --grid 256 --modes 0,1,2 --rounds 3"""
import argparse
import hashlib
import os
import statistics
import sys

import torch  # noqa: F401  (shared HIP runtime)

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import macroc_amd as M  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--grid", type=int, default=256)
ap.add_argument("--modes", default="0,1,2")
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--rtol", default="1e-8")
a = ap.parse_args()
G = a.grid
ctx = {}
for md in [int(v) for v in a.modes.split(",")]:
    os.environ["MCX_PAD_ALIGN"] = str(md)
    m = M.Macroc(["-da_grid_x", G, "-da_grid_y", G, "-da_grid_z", G, "-ksp_rtol", a.rtol])
    m.set_timing(True)
    m.apply_bc_on_u(m.get_displacement(1))
    m.set_strains(); m.homogenize(); m.assembly_res(); m.assembly_jac()
    ctx[md] = m
res = {q: [] for q in ctx}
spmv = {q: [] for q in ctx}
hashes = {}
for r in range(a.rounds):
    for md, m in ctx.items():
        its, rn, reason = m.solve_Ax()
        t = m.timing()
        h = hashlib.sha1(m.du().tobytes()).hexdigest()[:12]
        hashes.setdefault(h, []).append(md)
        res[md].append(t["solve_ms"] / its)
        spmv[md].append(t["spmv_ms_total"] / max(t["spmv_launches"], 1))
        print(f"round {r} pad_align {md}: its={its} reason={reason} ms/iter={t['solve_ms'] / its:.4f} "
              f"spmv_ms={spmv[md][-1]:.4f} du#{h}", flush=True)
for md in ctx:
    print(f"{G}^3 pad_align {md}: median ms/iter {statistics.median(res[md]):.4f} spmv {statistics.median(spmv[md]):.4f}")
print("du bitwise equal across layouts:", len(hashes) == 1)
for m in ctx.values():
    m.finish()
