"""Run-to-run and option-to-option bitwise check of the J2 (config 5) Newton path on the GPU:
the per-step KSP iterations, |RES| history, exception-node count and an md5 of u for each
variant of --opts (name=value,...;...).  Diagnosis tool (not a test)."""
import argparse
import hashlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import macroc_amd as M  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--grid", type=int, default=64)
ap.add_argument("--ts", type=int, default=3)
ap.add_argument("--opts", default=";", help="';'-separated option sets, e.g. 'cg_pdb=0;cg_pdb=1'")
a = ap.parse_args()
out = []
for spec in a.opts.split(";"):
    m = M.Macroc(["-da_grid_x", a.grid, "-da_grid_y", a.grid, "-da_grid_z", a.grid, "-mat_law", "plastic",
                  "-ksp_rtol", "1e-8", "-ts", a.ts, "-dt", 0.01])
    for kv in [kv for kv in spec.split(",") if kv]:
        m.set_option(kv.split("=")[0], float(kv.split("=")[1]))
    rec = []
    for t in range(a.ts):
        o = m.time_step(t)
        rec.append((o["ksp_its"], [float(r) for r in o["res"]], m.get_info()["vi_exc_nodes"],
                    hashlib.md5(m.u().tobytes()).hexdigest()))
    m.finish()
    out.append(rec)
    print(spec or "(defaults)", json.dumps(rec), flush=True)
print("all equal:", all(r == out[0] for r in out))
