#!/bin/bash
# round 4o: the headline bench under rocprofv3 --kernel-trace --stats, the PMC HBM-traffic passes
# of its SpMV (tools/pmc_spmv.sh) and the SQ/LDS counters (tools/pmc_vibm.sh); MCX_COMMIT names the code
set -euo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 480 rocprofv3 --kernel-trace --stats -d gpurun_out/r04o_prof -o run --output-format csv -- \
  python3 bench.py --variants '' --config5 0 --bending 0 --cpu-grid 0 \
  > gpurun_out/r04o_bench_under_rocprof.json 2> gpurun_out/r04o_bench_rocprof.log
find gpurun_out/r04o_prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/r04o_rocprof_kernel_stats.csv \;
rm -rf gpurun_out/r04o_prof
bash tools/pmc_spmv.sh aij-vi 256
bash tools/pmc_vibm.sh
