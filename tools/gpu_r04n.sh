#!/bin/bash
# round 4n: the final code: the whole GPU suite, smoke(), the driver's bench command, the default bench
set -euo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
AMD_LOG_LEVEL=1 timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread \
  > gpurun_out/r04n_pytest_gpu.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04n_smoke.log 2>&1
t0=$SECONDS
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r04n_bench_driver_cmd.json 2> gpurun_out/r04n_bench_driver_cmd.log
echo "$((SECONDS - t0)) s wall (python bench.py --steps 20 --warmup 5)" > gpurun_out/r04n_bench_driver_cmd.wall
