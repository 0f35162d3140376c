#!/bin/bash
# round 4p: grouped LDS-path reads in the exception-node kernel (option vi_lg_exc) on config 5's
# last Newton system and on the bending leg's, same-process A/B
set -euo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "exception_nodes" -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r04p_pytest.log 2>&1
timeout -k 10 300 python -u tools/bench_nonlinear.py --grid 128 --ab vi_lg_exc=0,1 --ab-rounds 3 \
  > gpurun_out/r04_ab_lgexc_c5.json 2> gpurun_out/r04_ab_lgexc_c5.log
