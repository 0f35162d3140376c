"""Interleaved in-process A/B of SpMV variants (DESIGN rule: compare variants on one device, one
process, alternating rounds).  A variant is a set of mcx_set_option values, e.g.

    python tools/spmv_ab.py --grid 256 --mat aij --variants "split_tx=0;split_tx=128;spmv_zblocks=512"

Options not named by a variant are reset to --base before it runs."""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import macroc_amd as M  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--grid", default="256", help="N or NX,NY,NZ")
ap.add_argument("--mat", default="aij", choices=["aij", "sbaij"])
ap.add_argument("--split", type=int, default=1, help="aij: -mat_aij_split")
ap.add_argument("--vi", type=int, default=1, help="aij: -mat_aij_vi")
ap.add_argument("--vi-bits", type=int, default=4, help="aij value-indexed: 4 (per-slot nibbles) or 8 (bytes)")
ap.add_argument("--vi-block", type=int, default=1, help="aij value-indexed: 1 = one byte per 3x3 block when possible")
ap.add_argument("--variants", default="split_tx=0", help="';'-separated option sets 'name=value,name=value'")
ap.add_argument("--base", default="split_tx=0,spmv_zblocks=0,split_dbg=0", help="options every variant starts from")
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--lib", default="", help="another build of libmacroc_amd.so (e.g. the previous commit's)")
a = ap.parse_args()
if a.lib:
    M.LIB_PATH = os.path.abspath(a.lib)


def parse(spec):
    return [(kv.split("=")[0], float(kv.split("=")[1])) for kv in spec.split(",") if kv]


g = [int(v) for v in a.grid.split(",")]
NX, NY, NZ = g if len(g) == 3 else g * 3
m = M.Macroc(["-da_grid_x", NX, "-da_grid_y", NY, "-da_grid_z", NZ, "-dm_mat_type", a.mat, "-mat_aij_split", a.split,
              "-mat_aij_vi", a.vi])
if a.mat == "aij" and a.vi:
    m.set_option("vi_bits", a.vi_bits)
    m.set_option("vi_block", a.vi_block)
m.apply_bc_on_u(m.get_displacement(1))
m.set_strains(); m.homogenize(); m.assembly_res(); m.assembly_jac()
base = parse(a.base)
variants = [parse(v) for v in a.variants.split(";")]


def select(v):
    for k, val in base + v:
        m.set_option(k, val)


x = np.random.default_rng(1).uniform(-1, 1, m.n)
ys = []
for v in variants:
    select(v)
    ys.append(m.spmv(x))
    inf = m.get_info()
    print(f"  variant {v}: st_listed {inf['st_listed']} tile {inf['spmv_tx']}x{inf['spmv_ty']}x{inf['spmv_kc']}", flush=True)
res = [[] for _ in variants]
for r in range(a.rounds):
    for q, v in enumerate(variants):
        select(v)
        res[q].append(m.time_spmv(a.iters))
tb = m.timing()["spmv_bytes_per_launch"]
print(f"{a.mat} grid {NX}x{NY}x{NZ} storage {m.get_info()['storage']} algorithmic {tb / 1e9:.3f} GB per launch")
for q, v in enumerate(variants):
    med = statistics.median(res[q])
    rel = np.linalg.norm(ys[q] - ys[0]) / np.linalg.norm(ys[0])
    name = ",".join(f"{k}={val:g}" for k, val in v) or "(base)"
    print(f"  {name:40s} median {med:.4f} ms  min {min(res[q]):.4f}  -> {tb / med / 1e6:.0f} GB/s  |y-y0|/|y0|={rel:.2e}")
m.finish()
