#!/bin/bash
# A/B: prefetch of the next phase's first block across the phase barriers (split_pf / spmv_kernel 12)
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/spmv_ab.py --grid 256 --mat aij --variants "split_pf=0;split_pf=1" --base "split_tx=0,split_ty=0,split_pf=0" --rounds 5 --iters 20 > gpurun_out/r02_ab_pf_aij.log 2>&1 && \
timeout -k 10 300 python -u tools/spmv_ab.py --grid 256 --mat sbaij --variants "spmv_kernel=11;spmv_kernel=12" --base "spmv_zblocks=0" --rounds 5 --iters 20 > gpurun_out/r02_ab_pf_sbaij.log 2>&1
