#!/bin/bash
# value-indexed AIJ: GPU test suite, SpMV A/B against the split storage, default bench
export TMPDIR=/tmp; mkdir -p gpurun_out
TAG=${1:-r02_vi}
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 && \
timeout -k 10 200 python -u tools/spmv_ab.py --grid 256 --mat aij --variants "spmv_nt=2" --base "spmv_nt=2" --rounds 5 --iters 20 > gpurun_out/${TAG}_ab256_vi.log 2>&1 && \
timeout -k 10 200 python -u tools/spmv_ab.py --grid 64 --mat aij --variants "spmv_nt=2" --base "spmv_nt=2" --rounds 5 --iters 50 > gpurun_out/${TAG}_ab64_vi.log 2>&1 && \
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.log
