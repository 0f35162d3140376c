#!/bin/bash
# round 4b: multi-rank overhead itemised by kernel traces — 8 in-process 256^3 subdomain contexts
# (512^3 as 2x2x2) against one 256^3 context, the same fixed number of CG iterations
set -euo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
ITS=${ITS:-200}
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/r04_mr8 -o run --output-format csv -- \
  python3 tools/multirank_profile.py --ranks 8 --its $ITS > gpurun_out/r04_mr8.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/r04_mr1 -o run --output-format csv -- \
  python3 tools/multirank_profile.py --ranks 1 --its $ITS > gpurun_out/r04_mr1.log 2>&1
for t in mr8 mr1; do
  f=$(find gpurun_out/r04_$t -name '*kernel_trace.csv' | head -1)
  python3 tools/kernel_trace_summary.py "$f" --its $ITS > gpurun_out/r04_${t}_summary.txt
  rm -f "$f"
done
