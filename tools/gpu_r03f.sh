# round-3 (f): exception lanes deferred before the uniformity test — config-5 A/B, exception tests, GPU suite
mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 180 python -u tools/bench_nonlinear.py --grid 128 --ts 3 --ab vi_exc_list=0,2048 > gpurun_out/r03f_c5_ab_exc.json 2> gpurun_out/r03f_c5_ab_exc.log && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multirank.py -k "exception" -x -v --timeout 120 --timeout-method thread > gpurun_out/r03f_pytest_exc.txt 2>&1 && \
timeout -k 10 480 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03f_pytest_gpu.txt 2>&1
