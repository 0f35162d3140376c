# round-3 (i): final code — full GPU suite, then the default bench
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 480 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03i_pytest_gpu.txt 2>&1
timeout -k 10 420 python3 bench.py > gpurun_out/r03i_bench_default.json 2> gpurun_out/r03i_bench_default.log
