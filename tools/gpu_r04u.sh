#!/bin/bash
# round 4u: the driver bench command on the round's last code
set -euo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
t0=$SECONDS
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r04u_bench_driver_cmd.json 2> gpurun_out/r04u_bench_driver_cmd.log
echo "$((SECONDS - t0)) s wall (python bench.py --steps 20 --warmup 5)" > gpurun_out/r04u_bench_driver_cmd.wall
