"""Interleaved in-process A/B of SpMV variants (DESIGN rule: compare variants on one device,
one process, alternating rounds).  Usage: python tools/spmv_ab.py --grid 256 --mat aij --subl 0,8,16"""
import argparse
import statistics
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import macroc_amd as M  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--grid", type=int, default=256)
ap.add_argument("--mat", default="aij")
ap.add_argument("--subl", default="0,8")
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--iters", type=int, default=20)
a = ap.parse_args()
N = a.grid
m = M.Macroc(["-da_grid_x", N, "-da_grid_y", N, "-da_grid_z", N, "-dm_mat_type", a.mat])
m.apply_bc_on_u(m.get_displacement(1))
m.set_strains(); m.homogenize(); m.assembly_res(); m.assembly_jac()
m.spmv(m.b())  # p := b (padded), a realistic operand
t = m.timing()
nbytes = None
variants = [int(v) for v in a.subl.split(",")]
res = {v: [] for v in variants}
for r in range(a.rounds):
    for v in variants:
        m.set_option("spmv_subl", v)
        res[v].append(m.time_spmv(a.iters))
tb = m.timing()["spmv_bytes_per_launch"]
for v in variants:
    med = statistics.median(res[v])
    print(f"{a.mat} grid {N}^3 subl={v:3d}: median {med:.4f} ms  min {min(res[v]):.4f}  -> {tb / med / 1e6:.0f} GB/s "
          f"(algorithmic {tb / 1e9:.2f} GB)")
m.finish()
