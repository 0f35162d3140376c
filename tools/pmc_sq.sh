#!/bin/bash
# tools/pmc_sq.sh — stall / cache counters of the SpMV kernels (diagnosis, not the bench):
# three separate --pmc passes over short tools/spmv_ab.py runs, kernel trace only.
set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmc_sq
mkdir -p $OUT
PASSES=(
  "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES"
  "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum TCC_EA0_RDREQ_sum"
  "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum"
)
for mat in aij sbaij; do
  V="split_dbg=0"; [ $mat = sbaij ] && V="spmv_kernel=11"
  p=0
  for C in "${PASSES[@]}"; do
    p=$((p+1))
    timeout -k 10 300 rocprofv3 --pmc $C --kernel-include-regex 'k_spmv' -d $OUT/$mat-$p -o run --output-format csv -- \
      python3 tools/spmv_ab.py --mat $mat --variants "$V" --base "" --rounds 1 --iters 5 --grid 256 > $OUT/$mat-$p.log 2>&1
  done
done
python3 - <<'PY'
import csv, glob, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for fn in glob.glob("gpurun_out/pmc_sq/*/**/*counter_collection.csv", recursive=True):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    for r in csv.DictReader(open(fn)):
        d = r["Dispatch_Id"]
        per[d][r["Counter_Name"]] += float(r["Counter_Value"])
        names[d] = r["Kernel_Name"].split("(")[0]
    for d, cs in per.items():
        for c, v in cs.items():
            acc[names[d]][c].append(v)
with open("gpurun_out/pmc_sq/summary.txt", "w") as f:
    for k, cs in sorted(acc.items()):
        line = k + "\n" + "\n".join(f"   {c:36s} {sum(v)/len(v):.4g}  (n={len(v)})" for c, v in sorted(cs.items()))
        print(line)
        f.write(line + "\n")
PY
