#!/bin/bash
# round 4c: the whole GPU suite on the current code, then the default bench line (headline,
# variants, config 5, the uniformly plastic bending leg, the MPI CPU baseline)
set -euo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread \
  > gpurun_out/r04c_pytest_gpu.log 2>&1
timeout -k 10 600 python -u bench.py > gpurun_out/r04c_bench_default.json 2> gpurun_out/r04c_bench_default.log
