#!/bin/bash
# round 4a: parity + multirank suites after the inode row order and the deterministic exception
# list, the config-5 determinism check (defaults twice in one process), the exception-share sweep
# of the AIJ storages, the CPU baseline's full 128^3 MPI step on the box's 16 cores
set -euo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multirank.py -x -v --timeout 300 \
  --timeout-method thread > gpurun_out/r04a_pytest.log 2>&1
timeout -k 10 200 python -u tools/cg_ab.py --grid 256 --option cg_pdb --values 1,4 --rounds 3 \
  > gpurun_out/r04_cg_ab_pqb256.log 2>&1
timeout -k 10 300 python -u tools/determinism_check.py --grid 128 --ts 3 --opts ';' > gpurun_out/r04_determinism_128.log 2>&1
timeout -k 10 400 python -u tools/exc_sweep.py --grid 128 > gpurun_out/r04_exc_sweep128.log 2>&1
timeout -k 10 400 /opt/conda/bin/mpirun -np 16 oracle/macroc_cpu_mpi -da_grid_x 128 -da_grid_y 128 -da_grid_z 128 \
  -ksp_rtol 1e-8 > gpurun_out/r04_cpu_mpi_128.json 2> gpurun_out/r04_cpu_mpi_128.log
