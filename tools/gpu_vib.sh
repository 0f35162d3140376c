#!/bin/bash
# block-indexed AIJ: VI parity tests, SpMV staged / gathered at 256^3, 128^3, 64^3
export TMPDIR=/tmp; mkdir -p gpurun_out
TAG=${1:-r02_vibm}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multirank.py tests/test_gpu_callback.py -k "vi or device_law" -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 && \
timeout -k 10 200 python -u tools/spmv_ab.py --grid 256 --mat aij --variants "vi_stage=1;vi_stage=0" --base "vi_stage=1" --rounds 5 --iters 20 > gpurun_out/${TAG}_ab256.log 2>&1 && \
timeout -k 10 200 python -u tools/spmv_ab.py --grid 128 --mat aij --variants "vi_stage=1;vi_stage=0" --base "vi_stage=1" --rounds 5 --iters 20 > gpurun_out/${TAG}_ab128.log 2>&1 && \
timeout -k 10 200 python -u tools/spmv_ab.py --grid 64 --mat aij --variants "vi_stage=1;vi_stage=0" --base "vi_stage=1" --rounds 5 --iters 50 > gpurun_out/${TAG}_ab64.log 2>&1
