#!/bin/bash
# small-grid SpMV A/B (tools/spmv_ab.py): SBAIJ kernels at 128^3 (config 5's grid)
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/spmv_ab.py --grid 128 --mat sbaij --variants "spmv_kernel=4;spmv_kernel=1;spmv_kernel=5;spmv_kernel=7;spmv_kernel=8;spmv_kernel=9;spmv_kernel=0" --base "spmv_zblocks=0" --rounds 5 --iters 30 > gpurun_out/r02_ab_sbaij128.log 2>&1
