#!/bin/bash
# value-indexed SpMV: VI parity tests, then in-process A/B (staged ring vs gathered x; bytes)
export TMPDIR=/tmp; mkdir -p gpurun_out
TAG=${1:-r02_vim}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multirank.py tests/test_gpu_callback.py -k "vi or device_law" -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 && \
timeout -k 10 200 python -u tools/spmv_ab.py --grid 256 --mat aij --variants "vi_stage=1;vi_stage=0" --base "vi_stage=1" --rounds 5 --iters 20 > gpurun_out/${TAG}_ab256.log 2>&1 && \
timeout -k 10 200 python -u tools/spmv_ab.py --grid 256 --mat aij --vi-bits 8 --variants "vi_stage=0" --base "vi_stage=0" --rounds 3 --iters 20 > gpurun_out/${TAG}_ab256_b8.log 2>&1 && \
timeout -k 10 200 python -u tools/spmv_ab.py --grid 128 --mat aij --variants "vi_stage=1;vi_stage=0" --base "vi_stage=1" --rounds 5 --iters 20 > gpurun_out/${TAG}_ab128.log 2>&1 && \
timeout -k 10 200 python -u tools/spmv_ab.py --grid 64 --mat aij --variants "vi_stage=1;vi_stage=0;spmv_zblocks=512,vi_stage=1" --base "vi_stage=1,spmv_zblocks=0" --rounds 5 --iters 50 > gpurun_out/${TAG}_ab64.log 2>&1
