#!/bin/bash
# round 4t: wave descriptors with the grouped LDS-path reads (vi_wdesc 1 at vi_lg 2): parity subset and A/Bs
set -euo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "production_tiles" -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/r04t_pytest.log 2>&1
timeout -k 10 200 python -u tools/spmv_ab.py --grid 256 --base "" --rounds 7 --variants "vi_wdesc=0;vi_wdesc=1" \
  > gpurun_out/r04_ab_wdesc_lg256.log 2>&1
timeout -k 10 300 python -u tools/cg_ab.py --grid 256 --option vi_wdesc --values 0,1 --rounds 3 \
  > gpurun_out/r04_cg_ab_wdesc_lg256.log 2>&1
