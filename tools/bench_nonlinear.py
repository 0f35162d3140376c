"""BASELINE config 5 path: 128^3 grid, non-linear Newton with the J2-plastic Gauss-point law behind
the callback (MicroPP material type 1 parameters E, nu, Sy, Ka from -micro_mat_1), time steps
1..T of src/main.c:49-109 (apply BC, Newton to newton_rel_tol, update_vars).  Prints one JSON
line: Newton iterations, CG iterations, wall time per Newton iteration (solve-bearing), DOF/s.
MicroPP's FE2 micro solve (-micro_n 10) is not available; the callback runs the material-point
law, which is MicroPP's homogenised response for identical phase materials."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import macroc_amd as M  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--grid", type=int, default=128)
ap.add_argument("--ts", type=int, default=3, help="time steps (step 0 has zero load)")
ap.add_argument("--mat-type", default="aij")
ap.add_argument("--split", type=int, default=1, help="aij: -mat_aij_split (1: upper blocks + bf16 corrections)")
ap.add_argument("--rtol", type=float, default=1e-8)
ap.add_argument("--dt", type=float, default=0.01, help="load step (U = -ts*dt); 0.01 drives the circle plastic")
ap.add_argument("--maxq", type=int, default=None, help="aij-split: split_maxq (correction quads per node allowed)")
ap.add_argument("--exc-max", type=int, default=None, help="aij value-indexed: vi_exc_max (per-mille of owned nodes "
                "allowed as exception nodes; 0: a per-GP tangent falls back to AIJ-split)")
ap.add_argument("--micro-n", type=int, default=10, help="-micro_n (BASELINE config 5: 10; sizes MicroPP's micro-cell, "
                "which the device law does not have: reported, no effect)")
ap.add_argument("--set", default="", help="options before the run, 'name=value,...'")
ap.add_argument("--ab", default="", help="after the run: re-solve the last Newton system alternating an option's "
                "values, 'name=v1,v2' (same process; per-CG-iteration and SpMV times to stderr)")
ap.add_argument("--ab-rounds", type=int, default=3)
a = ap.parse_args()
N = a.grid
m = M.Macroc(["-da_grid_x", N, "-da_grid_y", N, "-da_grid_z", N, "-mat_law", "plastic", "-ksp_rtol", repr(a.rtol),
              "-dm_mat_type", a.mat_type, "-mat_aij_split", a.split, "-ts", a.ts, "-dt", a.dt, "-micro_n", a.micro_n])
m.set_timing(True)
if a.maxq is not None:
    m.set_option("split_maxq", a.maxq)
if a.exc_max is not None:
    m.set_option("vi_exc_max", a.exc_max)
for kv in [kv for kv in a.set.split(",") if kv]:
    m.set_option(kv.split("=")[0], float(kv.split("=")[1]))
steps = []
t_all = time.perf_counter()
for ts in range(a.ts):
    t0 = time.perf_counter()
    out = m.time_step(ts)
    dt = time.perf_counter() - t0
    nl, fmax = m.nonlinear_stats()
    tm = m.timing()
    steps.append(dict(ts=ts, newton_its=out["newton_its"], ksp_its=out["ksp_its"], res=out["res"], seconds=dt,
                      nonlinear_gps=nl, f_trial_max=fmax, storage=m.get_info()["storage"],
                      vi_exc_nodes=m.get_info()["vi_exc_nodes"],
                      last_phases_ms={k: tm[k] for k in ("strains_ms", "homogenize_ms", "residual_ms", "jacobian_ms",
                                                         "solve_ms")}))
    print(json.dumps(steps[-1]), file=sys.stderr, flush=True)
tot = time.perf_counter() - t_all
nits = sum(s["newton_its"] for s in steps)
info = m.get_info()
print(json.dumps({"workload": f"config 5 path: {N}^3 non-linear Newton (J2 callback), {a.ts} time steps, dt {a.dt}",
                  "micro_n": a.micro_n, "micro_n_note": "no micro-scale FE problem behind the device law (MicroPP out of scope)",
                  "device_gb": m.get_info()["device_bytes"] / 1e9,
                  "mat_type": a.mat_type, "storage": {0: "aij-blocks", 1: "sbaij", 2: "aij-split", 3: "aij-vi"}[info["storage"]],
                  "vi_exc_nodes": info["vi_exc_nodes"], "vi_blocks": info["vi_blocks"],
                  "split_slots": info["split_slots"], "split_bits": info["split_bits"], "newton_its": nits, "cg_its": sum(sum(s["ksp_its"]) for s in steps),
                  "seconds": tot, "ms_per_newton_iter": tot / max(nits, 1) * 1e3,
                  "dof_per_s": 3 * N ** 3 * nits / tot, "steps": steps}))
if a.ab:
    import numpy as np
    import statistics
    name, vals = a.ab.split("=")
    vals = [float(v) for v in vals.split(",")]
    res = {v: [] for v in vals}
    spmv = {v: [] for v in vals}
    dus = {}
    for r in range(a.ab_rounds):
        for v in vals:
            m.set_option(name, v)
            its, rn, reason = m.solve_Ax()
            t = m.timing()
            res[v].append(t["solve_ms"] / its)
            spmv[v].append(t["spmv_ms_total"] / max(t["spmv_launches"], 1))
            dus.setdefault(v, (its, m.du()))
    for v in vals:
        d = np.linalg.norm(dus[v][1] - dus[vals[0]][1]) / np.linalg.norm(dus[vals[0]][1])
        print(f"A/B {N}^3 {name}={v:g}: median ms/CG iter {statistics.median(res[v]):.4f}  spmv kernel "
              f"{statistics.median(spmv[v]):.4f} ms  its {dus[v][0]}  |du-du0|/|du0| {d:.2e}", file=sys.stderr,
              flush=True)
m.finish()
