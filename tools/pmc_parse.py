"""Parse the two rocprofv3 PMC passes of tools/pmc_spmv.sh into per-launch HBM bytes and merge
them into profiles/pmc_spmv.json (read by bench.py's roofline.traffic).  gfx950 correction:
FETCH_SIZE counts half the bytes of 16-B-per-lane streaming reads (MI355X_MICROARCH.md, HBM /
rocprofv3 section), so reads = 2 * FETCH_SIZE; WRITE_SIZE is exact.  Both are in KB."""
import csv
import glob
import json
import os
import statistics
import sys

mat, grid, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]


def per_dispatch(counter):
    files = glob.glob(os.path.join(out, counter, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv for {counter} under {out}")
    vals = {}
    names = {}
    for fn in files:
        with open(fn) as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") != counter:
                    continue
                d = row["Dispatch_Id"]
                vals[d] = vals.get(d, 0.0) + float(row["Counter_Value"])
                names[d] = row["Kernel_Name"]
    return vals, names


fetch, names = per_dispatch("FETCH_SIZE")
write, wnames = per_dispatch("WRITE_SIZE")


def per_kernel(vals, nm):
    """median per kernel (gated launches of a converged chunk do no work: launches that moved > 1 %
    of the kernel's maximum), summed over the kernels: one SpMV may be two launches (the
    default-stencil path: k_spmv_st + k_spmv_face)"""
    by = {}
    for d, v in vals.items():
        by.setdefault(nm[d].split("(")[0], []).append(v)
    med, cnt = {}, 0
    for k, vs in by.items():
        real = [v for v in vs if v > 0.01 * max(vs)]
        med[k] = statistics.median(real)
        cnt = max(cnt, len(real))
    return sum(med.values()), med, cnt


fk, fmed, nf = per_kernel(fetch, names)
wk, wmed, nw = per_kernel(write, wnames)
f_real, w_real = range(nf), range(nw)
hbm = (2 * fk + wk) * 1024
kern = sorted(set(n.split("(")[0] for n in names.values()))
summary = (f"{mat} {grid}^3 kernels {kern}: FETCH_SIZE dispatches={len(fetch)} real={len(f_real)} "
           f"median={fk:.1f} KB; WRITE_SIZE dispatches={len(write)} real={len(w_real)} median={wk:.1f} KB; "
           f"HBM bytes per launch = (2*FETCH + WRITE)*1024 = {hbm / 1e9:.3f} GB")
print(summary)
# accumulate in gpurun_out/pmc/pmc_spmv.json (merged back from the GPU box), seeded from the
# committed profiles/pmc_spmv.json; copy it into profiles/ after review
root = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
path = os.path.join(out, "..", "pmc_spmv.json")
seed = path if os.path.exists(path) else os.path.join(root, "profiles", "pmc_spmv.json")
try:
    with open(seed) as f:
        d = json.load(f)
except (OSError, ValueError):
    d = {}
d[f"{mat}:{grid}x{grid}x{grid}"] = {"hbm_bytes_per_launch": hbm, "fetch_kb_median": fk, "write_kb_median": wk,
                                     "per_kernel_kb": {k: {"fetch": fmed[k], "write": wmed.get(k)} for k in fmed},
                                     "launches": len(f_real), "kernels": kern,
                                     "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE separate passes, "
                                               "--kernel-include-regex, bench.py --steps 1 --warmup 0",
                                     "commit": os.environ.get("MCX_COMMIT")}
with open(path, "w") as f:
    json.dump(d, f, indent=1, sort_keys=True)
with open(os.path.join(out, "summary.txt"), "w") as f:
    f.write(summary + "\n")
