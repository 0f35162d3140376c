#!/bin/bash
# round 4h: wave descriptors (option vi_wdesc): parity subset, SpMV A/B, whole-CG A/B
set -euo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multirank.py -k "production_tiles or exact_rows or single_rank or multirank_vi or cg_pdb_bitwise or determinism" -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/r04h_pytest.log 2>&1
timeout -k 10 200 python -u tools/spmv_ab.py --grid 256 --base "" --rounds 7 --variants \
"vi_wdesc=0,vi_fma=1,split_dbg=0;vi_wdesc=1,vi_fma=1,split_dbg=0;vi_wdesc=2,vi_fma=1,split_dbg=0;vi_wdesc=0,vi_fma=0,split_dbg=0;vi_wdesc=1,vi_fma=0,split_dbg=0;vi_wdesc=0,vi_fma=1,split_dbg=1;vi_wdesc=1,vi_fma=1,split_dbg=1" \
  > gpurun_out/r04_ab_wdesc256.log 2>&1
timeout -k 10 300 python -u tools/cg_ab.py --grid 256 --option vi_wdesc --values 0,1,2 --rounds 2 \
  > gpurun_out/r04_cg_ab_wdesc256.log 2>&1
