#!/bin/bash
# tools/pmc_spmv.sh STORAGE GRID (aij-vi | aij-split | aij-blocks | sbaij) — HBM traffic of the CG SpMV kernel from rocprofv3 PMC counters:
# FETCH_SIZE and WRITE_SIZE in separate passes (they do not fit one pass on gfx950), kernel
# trace only (no sys/runtime tracing beside --pmc), one bench step at GRID^3.  Results are
# parsed by tools/pmc_parse.py into gpurun_out/pmc/ and profiles/pmc_spmv.json.
set -euo pipefail
MAT=${1:-aij-split}
G=${2:-256}
case $MAT in
  aij-vi) RE='k_spmv_vib|k_spmv_st|k_spmv_face'; BM=aij ;;  # value-indexed: k_spmv_vibm, or the default-stencil k_spmv_st + k_spmv_face (vi_st)
  aij-split) RE='k_spmv_symp'; BM=aij-split ;;
  aij-blocks) RE='k_spmv<'; BM=aij-blocks ;;
  sbaij) RE='k_spmv_sym'; BM=sbaij ;;
esac
export TMPDIR=/tmp
OUT=gpurun_out/pmc/$MAT-$G
mkdir -p $OUT
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $C --kernel-include-regex "$RE" -d $OUT/$C -o run --output-format csv -- \
    python3 bench.py --steps 1 --warmup 0 --grid $G --mat-type $BM --variants '' --cpu-grid 0 --config5 0 --bending 0 --no-check \
    > $OUT/$C.log 2>&1
done
MCX_COMMIT=${MCX_COMMIT:-} python3 tools/pmc_parse.py $MAT $G $OUT
