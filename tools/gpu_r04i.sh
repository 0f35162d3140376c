#!/bin/bash
# round 4i: the whole GPU suite and smoke() on the final code (cg_ublocks A/B appended)
set -euo pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread \
  > gpurun_out/r04i_pytest_gpu.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04i_smoke.log 2>&1
timeout -k 10 300 python -u tools/cg_ab.py --grid 256 --option cg_ublocks --values 0,2048,512 --rounds 2 \
  > gpurun_out/r04_cg_ab_ublocks256.log 2>&1
