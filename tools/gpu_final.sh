#!/bin/bash
# round-end measurements of the final code: GPU suite, smoke, the driver's bench command, the
# default bench + the same under rocprofv3 --stats + PMC HBM traffic (profile_round.sh), SQ/LDS counters
# (SKIP_TESTS=1: start at the bench)
set -euo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
TAG=${1:-r02f}
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1
fi
t0=$SECONDS
timeout -k 10 560 python bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench_driver_cmd.json 2> gpurun_out/${TAG}_bench_driver_cmd.log
echo "$((SECONDS - t0)) s wall (python bench.py --steps 20 --warmup 5)" > gpurun_out/${TAG}_bench_driver_cmd.wall
bash tools/profile_round.sh ${TAG}
bash tools/pmc_vibm.sh
