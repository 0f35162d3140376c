#!/bin/bash
# round 4d: the paired-y-store A/B of the headline SpMV, its parity test, then the multi-rank
# overhead kernel traces (tools/gpu_r04b.sh)
set -euo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multirank.py -k "production_tiles or exact_rows or split_dense_escapes or exception_nodes or single_rank or multirank_vi" -x -v \
  --timeout 300 --timeout-method thread > gpurun_out/r04d_pytest.log 2>&1
timeout -k 10 200 python -u tools/spmv_ab.py --grid 256 --variants "vi_ypair=0;vi_ypair=1;vi_fma=0" --base "" --rounds 7 \
  > gpurun_out/r04_ab_ypair256.log 2>&1
bash tools/gpu_r04b.sh
