#!/bin/bash
# round 4m: grouped LDS-path reads (option vi_lg): parity subset, SpMV and whole-CG A/B
set -euo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "production_tiles" -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/r04m_pytest.log 2>&1
timeout -k 10 200 python -u tools/spmv_ab.py --grid 256 --base "" --rounds 7 --variants "vi_lg=1;vi_lg=2;vi_lg=3" \
  > gpurun_out/r04_ab_lg256.log 2>&1
timeout -k 10 300 python -u tools/cg_ab.py --grid 256 --option vi_lg --values 1,2,3 --rounds 2 \
  > gpurun_out/r04_cg_ab_lg256.log 2>&1
