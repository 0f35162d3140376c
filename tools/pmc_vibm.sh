#!/bin/bash
# issue / LDS counters of the block-indexed staged SpMV (k_spmv_st by default, vi_st_pair=1: k_spmv_sp,
# vi_st=0: k_spmv_vibm) at
# 256^3: two --pmc passes,
# kernel trace only, over a short tools/spmv_ab.py run (diagnosis, not the bench)
#   tools/pmc_vibm.sh [VARIANT] [TAG]   e.g. tools/pmc_vibm.sh vi_uni=1 uni
set -euo pipefail
export TMPDIR=/tmp
VAR=${1:-vi_st=1}
TAG=${2:-}
OUT=gpurun_out/pmc_vibm${TAG:+_$TAG}
mkdir -p $OUT
PASSES=(
  "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES"
  "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVES"
)
p=0
for C in "${PASSES[@]}"; do
  p=$((p+1))
  timeout -k 10 120 rocprofv3 --pmc $C --kernel-include-regex 'k_spmv_vibm|k_spmv_st|k_spmv_sp' -d $OUT/p$p -o run --output-format csv -- \
    python3 tools/spmv_ab.py --mat aij --variants "$VAR" --base "" --rounds 1 --iters 5 --grid 256 > $OUT/p$p.log 2>&1
done
OUT=$OUT VAR=$VAR python3 - <<'PY'
import csv, glob, collections, json, os
OUT, VAR = os.environ["OUT"], os.environ["VAR"]
tot = collections.defaultdict(float); n = collections.defaultdict(set)
for fn in glob.glob(OUT + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(fn)):
        tot[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]].add(r["Dispatch_Id"])
c = {k: tot[k] / max(len(n[k]), 1) for k in tot}
with open(OUT + "/summary.txt", "w") as f:
    for k in sorted(c):
        line = f"{k:28s} per launch {c[k]:.4e}  ({len(n[k])} launches)"
        print(line); f.write(line + "\n")
# SQ counters are summed over the 32 shader engines (SQ_BUSY_CYCLES) and the 256 CUs
# (SQ_LDS_IDX_ACTIVE: LDS-array cycles); SQ_WAVE_CYCLES counts in units of 4 cycles
busy_se, lds_cu = c["SQ_BUSY_CYCLES"] / 32, c["SQ_LDS_IDX_ACTIVE"] / 256
waves, planes = c["SQ_WAVES"], 64
d = {"aij-vi:256x256x256": {
    "kernel": ("k_spmv_vibm" if "vi_st=0" in VAR else "k_spmv_sp" if "vi_st_pair=1" in VAR else "k_spmv_st") +
              " 64x16 (" + VAR + ")",
    "commit": os.environ.get("MCX_COMMIT"),
    "method": "rocprofv3 --pmc, two passes of 8 SQ counters, kernel trace only, tools/spmv_ab.py --grid 256 "
              "--iters 5 (tools/pmc_vibm.sh)",
    "counters_per_launch": c, "sq_busy_cycles_per_se": busy_se, "lds_active_cycles_per_cu": lds_cu,
    "lds_busy_frac": lds_cu / busy_se, "lds_bank_conflict_cycles": c["SQ_LDS_BANK_CONFLICT"],
    "valu_insts_per_wave_plane": c["SQ_INSTS_VALU"] / waves / planes,
    "lds_insts_per_wave_plane": c["SQ_INSTS_LDS"] / waves / planes}}
d["aij-vi:256x256x256"]["options"] = VAR
json.dump(d, open(OUT + "/pmc_vibm.json", "w"), indent=1)
print(json.dumps(d["aij-vi:256x256x256"]["lds_busy_frac"]))
PY
