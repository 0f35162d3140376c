#!/bin/bash
# issue / LDS counters of the block-indexed staged SpMV (k_spmv_vibm) at 256^3: two --pmc passes,
# kernel trace only, over a short tools/spmv_ab.py run (diagnosis, not the bench)
set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmc_vibm
mkdir -p $OUT
PASSES=(
  "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES"
  "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVES"
)
p=0
for C in "${PASSES[@]}"; do
  p=$((p+1))
  timeout -k 10 120 rocprofv3 --pmc $C --kernel-include-regex 'k_spmv_vibm' -d $OUT/p$p -o run --output-format csv -- \
    python3 tools/spmv_ab.py --mat aij --variants "vi_tile=0" --base "" --rounds 1 --iters 5 --grid 256 > $OUT/p$p.log 2>&1
done
python3 - <<'PY'
import csv, glob, collections
tot = collections.defaultdict(float); n = collections.defaultdict(set)
for fn in glob.glob("gpurun_out/pmc_vibm/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(fn)):
        tot[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]].add(r["Dispatch_Id"])
with open("gpurun_out/pmc_vibm/summary.txt", "w") as f:
    for k in sorted(tot):
        line = f"{k:28s} per launch {tot[k] / max(len(n[k]), 1):.4e}  ({len(n[k])} launches)"
        print(line); f.write(line + "\n")
PY
