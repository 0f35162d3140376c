"""Where do the default-stencil rows differ from the index path's (diagnosis): one grid, vi_st 0 vs 1
(and vi_st_pair 0), one rank and a 2x1x1 in-process group; prints the differing nodes.
    python tools/dbg_st.py 516 5 4"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import macroc_amd as M  # noqa: E402
from test_gpu_multirank import newton_step, run_group  # noqa: E402

NX, NY, NZ = (int(v) for v in sys.argv[1:4])
x = np.random.default_rng(29).uniform(-1, 1, 3 * NX * NY * NZ)
for procs in ((1, 1, 1), (2, 1, 1)):
    argv = ["-da_grid_x", NX, "-da_grid_y", NY, "-da_grid_z", NZ, "-da_processors_x", procs[0], "-da_processors_y",
            procs[1], "-da_processors_z", procs[2], "-ksp_rtol", "1e-12"]
    n = procs[0] * procs[1] * procs[2]
    outs = {name: run_group(argv, n, newton_step(x, [("vi_stage", 1)] + opts))
            for name, opts in (("idx", [("vi_st", 0)]), ("sp", [("vi_st", 1)]), ("st", [("vi_st", 1), ("vi_st_pair", 0)]))}
    for name in ("sp", "st"):
        for r, (a, b) in enumerate(zip(outs["idx"], outs[name])):
            bad = np.nonzero(a["y"] != b["y"])[0]
            inf = b["info"]
            print(f"procs {procs} rank {r} {name}: {len(bad)} of {len(a['y'])} differ; local {inf['nx']}x{inf['ny']}x{inf['nz']} "
                  f"tile {inf['spmv_tx']}x{inf['spmv_ty']}x{inf['spmv_kc']} listed {inf['st_listed']}")
            import collections
            cnt = collections.Counter()
            where = {float(v): int(q) for q, v in enumerate(a["y"])}
            for d in bad:
                nd = int(d) // 3
                cnt[((nd // inf["nx"]) % inf["ny"], nd // (inf["nx"] * inf["ny"]))] += 1
            print("   bad (j, k):", dict(cnt))
            for d in bad[:6]:
                q = where.get(float(b["y"][d]))
                if q is not None:
                    nq, cq = divmod(q, 3)
                    print(f"   y[{int(d)}] equals idx y at node ({nq % inf['nx']},{(nq // inf['nx']) % inf['ny']},"
                          f"{nq // (inf['nx'] * inf['ny'])}) comp {cq}")
            for d in bad[:4]:
                nd, c = divmod(int(d), 3)
                i, j, k = nd % inf["nx"], (nd // inf["nx"]) % inf["ny"], nd // (inf["nx"] * inf["ny"])
                print(f"   node ({i},{j},{k}) comp {c}: {a['y'][d]!r} vs {b['y'][d]!r}")
