#!/bin/bash
# fused CG p update + wave-uniform dictionary: parity tests, then in-process A/B at 256^3 / 128^3
export TMPDIR=/tmp; mkdir -p gpurun_out
TAG=${1:-r02_fuse}
timeout -k 10 400 python -u -m pytest tests/test_gpu_fused_cg.py tests/test_gpu_parity.py -k "fused or vi" -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 && \
timeout -k 10 200 python -u tools/spmv_ab.py --grid 256 --mat aij --variants "vi_scalar=1;vi_scalar=0" --base "vi_scalar=1" --rounds 5 --iters 20 > gpurun_out/${TAG}_spmv256.log 2>&1 && \
timeout -k 10 300 python -u tools/cg_ab2.py --grid 256 --sets "cg_fuse_spmv=0,vi_scalar=0;cg_fuse_spmv=0,vi_scalar=1;cg_fuse_spmv=1,vi_scalar=0;cg_fuse_spmv=1,vi_scalar=1" --rounds 3 > gpurun_out/${TAG}_cg256.log 2>&1 && \
timeout -k 10 200 python -u tools/cg_ab2.py --grid 128 --sets "cg_fuse_spmv=0,vi_scalar=0;cg_fuse_spmv=1,vi_scalar=1" --rounds 3 > gpurun_out/${TAG}_cg128.log 2>&1
