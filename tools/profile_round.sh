#!/bin/bash
# tools/profile_round.sh TAG — the measurements behind the bench line, on the GPU box:
# the default bench, the same command under rocprofv3 --kernel-trace --stats, and the PMC HBM
# traffic passes of the headline SpMV (tools/pmc_spmv.sh).  Everything lands in gpurun_out/.
set -euo pipefail
TAG=${1:-r02}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 420 python3 bench.py > gpurun_out/${TAG}_bench_default.json 2> gpurun_out/${TAG}_bench_default.log
# under the profiler: the headline only (no variants, no config-5 / bending legs, no MPI CPU
# baseline: its ranks would inherit the profiler's preload and each open the GPU)
timeout -k 10 480 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- \
  python3 bench.py --variants '' --config5 0 --bending 0 --cpu-grid 0 \
  > gpurun_out/${TAG}_bench_default_under_rocprof.json 2> gpurun_out/${TAG}_bench_rocprof.log
bash tools/pmc_spmv.sh aij-vi 256
