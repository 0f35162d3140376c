"""Multi-rank overhead itemised by a kernel trace.  Runs a fixed number of CG
iterations (-ksp_max_it) either as N in-process subdomain contexts on one GPU (host thread per
rank, the decomposed path: halo pack/unpack, the sent nodes' p update first, the remaining p
update, partial sums + group reduction, k_cg_logic) or as one context of the same subdomain size,
so that `rocprofv3 --kernel-trace` of the two runs can be compared kernel by kernel
(tools/kernel_trace_summary.py).

    rocprofv3 --kernel-trace -d OUT -o run --output-format csv -- python tools/multirank_profile.py --ranks 8
    rocprofv3 --kernel-trace -d OUT1 -o run --output-format csv -- python tools/multirank_profile.py --ranks 1
"""
import argparse
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import macroc_amd as M  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--ranks", type=int, default=8)
ap.add_argument("--sub", type=int, default=256, help="nodes per direction per subdomain")
ap.add_argument("--its", type=int, default=200)
a = ap.parse_args()
grid = {1: (1, 1, 1), 2: (2, 1, 1), 4: (2, 2, 1), 8: (2, 2, 2)}[a.ranks]
N = [a.sub * p for p in grid]
argv = ["-da_grid_x", N[0], "-da_grid_y", N[1], "-da_grid_z", N[2], "-da_processors_x", grid[0],
        "-da_processors_y", grid[1], "-da_processors_z", grid[2], "-ts", 2, "-ksp_rtol", "1e-300",
        "-ksp_max_it", a.its]
res = [None] * a.ranks
errs = []


def body(m):
    m.apply_bc_on_u(m.get_displacement(1))
    m.set_strains(); m.homogenize(); m.assembly_res(); m.assembly_jac()
    m.solve_Ax()  # warm-up solve (same length)
    m.set_timing(True)
    t0 = time.perf_counter()
    its, rn, reason = m.solve_Ax()
    m.synchronize()
    tm = m.timing()
    return {"its": its, "reason": reason, "solve_ms": tm["solve_ms"], "wall_ms": (time.perf_counter() - t0) * 1e3,
            "spmv_avg_ms": tm["spmv_ms_total"] / max(tm["spmv_launches"], 1)}


if a.ranks == 1:
    with M.Macroc(argv) as m:
        res[0] = body(m)
else:
    g = M.LocalGroup(a.ranks)

    def worker(r):
        try:
            m = M.Macroc(argv, rank=r, nranks=a.ranks, group=g)
            try:
                res[r] = body(m)
            finally:
                m.finish()
        except Exception as e:  # surfaced below
            errs.append((r, repr(e)))

    ts = [threading.Thread(target=worker, args=(r,), daemon=True) for r in range(a.ranks)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(900)
    assert not errs, errs
    g.destroy()
for r, o in enumerate(res):
    print(json.dumps({"rank": r, "ranks": a.ranks, "grid": N, **o, "ms_per_cg_iter": o["solve_ms"] / max(o["its"], 1)}),
          flush=True)
