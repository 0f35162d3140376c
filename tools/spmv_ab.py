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
ap.add_argument("--subl", default="0")
ap.add_argument("--kernels", default="0", help="sbaij kernels to compare: 0 pull, 1 z-marching")
ap.add_argument("--nt", default="0", help="aij non-temporal matrix loads: 0,1")
ap.add_argument("--zblocks", default="0", help="z-marching grid (0 = one resident round)")
ap.add_argument("--split", type=int, default=1, help="aij: -mat_aij_split")
ap.add_argument("--splittx", default="0", help="aij-split tile widths to compare (0 = default)")
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--iters", type=int, default=20)
a = ap.parse_args()
N = a.grid
m = M.Macroc(["-da_grid_x", N, "-da_grid_y", N, "-da_grid_z", N, "-dm_mat_type", a.mat, "-mat_aij_split", a.split])
m.apply_bc_on_u(m.get_displacement(1))
m.set_strains(); m.homogenize(); m.assembly_res(); m.assembly_jac()
m.spmv(m.b())  # p := b (padded), a realistic operand
t = m.timing()
nbytes = None
import numpy as np  # noqa: E402

variants = [(int(s), int(kk), int(nt), int(zb), int(nu), int(tx)) for s in a.subl.split(",")
            for kk in a.kernels.split(",") for nt in a.nt.split(",") for zb in a.zblocks.split(",")
            for nu in ("0",) for tx in a.splittx.split(",")]
res = {v: [] for v in variants}
x = np.random.default_rng(1).uniform(-1, 1, m.n)
ys = {}
for v in variants:
    m.set_option("spmv_subl", v[0])
    m.set_option("spmv_kernel", v[1])
    m.set_option("spmv_nt", v[2])
    m.set_option("spmv_zblocks", v[3])
    if a.mat == "aij" and a.split:
        m.set_option("split_tx", v[5])
    ys[v] = m.spmv(x)
y0 = ys[variants[0]]
for r in range(a.rounds):
    for v in variants:
        m.set_option("spmv_subl", v[0])
        m.set_option("spmv_kernel", v[1])
        m.set_option("spmv_nt", v[2])
        m.set_option("spmv_zblocks", v[3])
        if a.mat == "aij" and a.split:
            m.set_option("split_tx", v[5])
        res[v].append(m.time_spmv(a.iters))
tb = m.timing()["spmv_bytes_per_launch"]
for v in variants:
    med = statistics.median(res[v])
    rel = np.linalg.norm(ys[v] - y0) / np.linalg.norm(y0)
    print(f"{a.mat} grid {N}^3 subl={v[0]:3d} kernel={v[1]} nt={v[2]} zb={v[3]} tx={v[5]}: median {med:.4f} ms  min {min(res[v]):.4f}  -> "
          f"{tb / med / 1e6:.0f} GB/s (algorithmic {tb / 1e9:.2f} GB)  |y-y0|/|y0|={rel:.2e}")
m.finish()
