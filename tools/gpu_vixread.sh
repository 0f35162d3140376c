#!/bin/bash
# block-indexed staged SpMV: x as unpaired ds_read_b64 vs the compiler's ds_read2_b64 pairs
export TMPDIR=/tmp; mkdir -p gpurun_out
TAG=${1:-r02_vixread}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "vi" -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 && \
timeout -k 10 200 python -u tools/spmv_ab.py --grid 256 --mat aij --variants "vi_xread=1;vi_xread=0" --base "vi_xread=1" --rounds 5 --iters 20 > gpurun_out/${TAG}_spmv256.log 2>&1 && \
timeout -k 10 200 python -u tools/spmv_ab.py --grid 128 --mat aij --variants "vi_xread=1;vi_xread=0" --base "vi_xread=1" --rounds 5 --iters 20 > gpurun_out/${TAG}_spmv128.log 2>&1 && \
timeout -k 10 300 python -u tools/cg_ab2.py --grid 256 --sets "vi_xread=1;vi_xread=0" --rounds 3 > gpurun_out/${TAG}_cg256.log 2>&1
