#!/bin/bash
# A/B of AIJ-split SpMV variants at 256^3 (tools/spmv_ab.py) after the SpMV parity tests.
# usage: bash tools/gpu_ab_tiles.sh TAG "variant;variant;..." [base]
export TMPDIR=/tmp; mkdir -p gpurun_out
TAG=${1:-r02}
VARS=${2:-"split_ty=0"}
BASE=${3:-"split_tx=0,split_ty=0,spmv_zblocks=0"}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multirank.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_t_spmv.log 2>&1 && \
timeout -k 10 400 python -u tools/spmv_ab.py --grid 256 --mat aij --variants "$VARS" --base "$BASE" --rounds 5 --iters 20 > gpurun_out/${TAG}_ab.log 2>&1
