"""Per-kernel split of the SpMV variants (run under rocprofv3 --kernel-trace --stats): N launches of
each option set on the 256^3 system (mcx_time_spmv), so the stats CSV gives every kernel's average:
    rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \\
        python3 tools/spmv_kernels.py --grid 256 --sets "vi_st=0;vi_st=1" --iters 50"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import macroc_amd as M  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--grid", type=int, default=256)
ap.add_argument("--sets", default="vi_st=0;vi_st=1")
ap.add_argument("--iters", type=int, default=50)
a = ap.parse_args()
G = a.grid
m = M.Macroc(["-da_grid_x", G, "-da_grid_y", G, "-da_grid_z", G])
m.apply_bc_on_u(m.get_displacement(1))
m.set_strains(); m.homogenize(); m.assembly_res(); m.assembly_jac()
for spec in a.sets.split(";"):
    for kv in [kv for kv in spec.split(",") if kv]:
        k, v = kv.split("=")
        m.set_option(k, float(v))
    print(spec, "avg ms per SpMV (events):", m.time_spmv(a.iters), "st_listed", m.get_info()["st_listed"], flush=True)
m.finish()
