#!/bin/bash
# round 4j: the driver's bench command and the default bench line on the final code
set -euo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
t0=$SECONDS
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r04j_bench_driver_cmd.json 2> gpurun_out/r04j_bench_driver_cmd.log
echo "$((SECONDS - t0)) s wall (python bench.py --steps 20 --warmup 5)" > gpurun_out/r04j_bench_driver_cmd.wall
timeout -k 10 500 python bench.py > gpurun_out/r04j_bench_default.json 2> gpurun_out/r04j_bench_default.log
