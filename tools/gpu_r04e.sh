#!/bin/bash
# round 4e: k_spmv_vibs (option vi_zs, the z-march by source plane): parity tests, SpMV A/B
# against k_spmv_vibm, whole-CG A/B, and the SpMV A/B under rocprofv3 --kernel-trace --stats
set -euo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "source_plane_march or vi_zs_option or production_tiles" -x -v \
  --timeout 300 --timeout-method thread > gpurun_out/r04e_pytest.log 2>&1
timeout -k 10 200 python -u tools/spmv_ab.py --grid 256 --variants "vi_zs=0;vi_zs=16;vi_zs=8" --base "" --rounds 7 \
  > gpurun_out/r04_ab_zs256.log 2>&1
timeout -k 10 300 python -u tools/cg_ab.py --grid 256 --option vi_zs --values 0,16,8 --rounds 2 \
  > gpurun_out/r04_cg_ab_zs256.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04e_prof -o run --output-format csv -- \
  python3 tools/spmv_ab.py --grid 256 --variants "vi_zs=0;vi_zs=16;vi_zs=8" --base "" --rounds 3 \
  > gpurun_out/r04e_prof.log 2>&1
find gpurun_out/r04e_prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/r04e_kernel_stats.csv \;
rm -rf gpurun_out/r04e_prof
