#!/bin/bash
# round 4q: the p update on a (rows, x chunks) grid (option cg_p2d): bitwise test, whole-CG A/B
set -euo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multirank.py -k "cg_pdb_bitwise or quad" -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/r04q_pytest.log 2>&1
timeout -k 10 300 python -u tools/cg_ab.py --grid 256 --option cg_p2d --values 0,1 --rounds 3 \
  > gpurun_out/r04_cg_ab_p2d256.log 2>&1
