"""Interleaved A/B of whole CG solves over option sets (same matrix, same process), with a
bitwise check of du between sets:
    python tools/cg_ab2.py --grid 256 --sets "cg_fuse_spmv=0;cg_fuse_spmv=1,vi_scalar=1" --rounds 3"""
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
ap.add_argument("--mat", default="aij")
ap.add_argument("--sets", required=True)
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--rtol", default="1e-8")
a = ap.parse_args()
G = a.grid
sets = [[(kv.split("=")[0], float(kv.split("=")[1])) for kv in s.split(",") if kv] for s in a.sets.split(";")]
m = M.Macroc(["-da_grid_x", G, "-da_grid_y", G, "-da_grid_z", G, "-ksp_rtol", a.rtol, "-dm_mat_type", a.mat])
m.set_timing(True)
m.apply_bc_on_u(m.get_displacement(1))
m.set_strains(); m.homogenize(); m.assembly_res(); m.assembly_jac()
res = {q: [] for q in range(len(sets))}
spmv = {q: [] for q in range(len(sets))}
for r in range(a.rounds):
    for q, s in enumerate(sets):
        for k, v in s:
            m.set_option(k, v)
        its, rn, reason = m.solve_Ax()
        t = m.timing()
        h = hashlib.sha1(m.du().tobytes()).hexdigest()[:12]
        res[q].append(t["solve_ms"] / its)
        spmv[q].append(t["spmv_ms_total"] / max(t["spmv_launches"], 1))
        print(f"round {r} set {q} {s}: its={its} reason={reason} ms/iter={t['solve_ms'] / its:.4f} "
              f"spmv_ms={t['spmv_ms_total'] / max(t['spmv_launches'], 1):.4f} du#{h}", flush=True)
for q, s in enumerate(sets):
    print(f"{a.mat} {G}^3 set {q} {s}: median ms/iter {statistics.median(res[q]):.4f} "
          f"spmv {statistics.median(spmv[q]):.4f}")
m.finish()
