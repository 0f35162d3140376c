#!/bin/bash
# small-grid SpMV A/B (tools/spmv_ab.py): SBAIJ pull vs z-march kernels at 64^3 (config 2's grid)
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/spmv_ab.py --grid 64 --mat sbaij --variants "spmv_kernel=1;spmv_kernel=0;spmv_kernel=8;spmv_kernel=3;spmv_kernel=0,spmv_subl=-1;spmv_kernel=0,spmv_subl=4" --base "spmv_zblocks=0,spmv_subl=0" --rounds 5 --iters 50 > gpurun_out/r02_ab_sbaij64.log 2>&1
timeout -k 10 300 python -u tools/spmv_ab.py --grid 64 --mat aij --split 0 --variants "spmv_nt=2;spmv_nt=0;spmv_subl=-1" --base "spmv_subl=0" --rounds 5 --iters 50 > gpurun_out/r02_ab_blocks64.log 2>&1
